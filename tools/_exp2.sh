set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so timeout -k 10 120 python tools/diag_cull.py > gpurun_out/diag.json 2> gpurun_out/diag.err || { echo "diag rc=$?"; tail -5 gpurun_out/diag.err; exit 1; }
for cfg in "SRT_CULL_CHUNK=100000"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/e_$tag -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/e_$tag.log 2>&1 || { echo "rc=$? $cfg"; exit 1; }
  echo "== $cfg"; grep -o '"value": [0-9.]*' gpurun_out/e_$tag.log; cut -d, -f1,4 gpurun_out/e_$tag/run_kernel_stats.csv | grep srt | sed 's/(srt::(anonymous namespace)::[A-Za-z]*)//; s/srt::(anonymous namespace):://'
done
