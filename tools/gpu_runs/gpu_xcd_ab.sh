source tools/gpu_runs/gpu_lib.sh
Q="--steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline"
for n in base spatial; do
  if [ $n = base ]; then unset SRT_LIB; else export SRT_LIB=simpleraytracer_amd/lib_ab/$n/libModelRunner.so; fi
  run fetch_$n 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex TraceCullKernel -d gpurun_out/fetch_$n -o run --output-format csv -- python3 bench.py $Q
  run bench_$n 200 python bench.py --no-extras --no-cpu-baseline
done
