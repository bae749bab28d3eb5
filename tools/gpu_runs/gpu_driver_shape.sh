source tools/gpu_runs/gpu_lib.sh
for b in 1 4 7 0; do
  run ds_b$b 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --batch $b || exit 1
  run ds2_b$b 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --batch $b || exit 1
done
