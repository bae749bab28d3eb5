source tools/gpu_runs/gpu_lib.sh
for v in ord0 ord1 ord4; do
  SRT_LIB=simpleraytracer_amd/lib_ab/$v/libModelRunner.so run e2e_$v 120 python tools/e2e_probe.py --chunks 4,1 || exit 1
  SRT_LIB=simpleraytracer_amd/lib_ab/$v/libModelRunner.so run bench_$v 200 python bench.py --no-extras --no-cpu-baseline --steps 100 || exit 1
done
for v in ord0 ord1 ord4; do echo $v; cat gpurun_out/e2e_$v.log | grep chunks; python -c "import json;d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_frame'])"; done
