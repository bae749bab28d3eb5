set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for w in 8 16 4; do
  SRT_CULL_WAVES=$w timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/bench_w$w.log 2>&1 || exit 1
done
for c in 512 2048; do
  SRT_CULL_CHUNK=$c timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/bench_chunk$c.log 2>&1 || exit 1
done
