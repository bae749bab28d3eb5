#!/bin/bash
# Round 6: (1) HBM traffic of the record / bin launch in the headline launch shape (PrepareBinKernel,
# 8 frames per launch; two --pmc passes), to put a measured figure beside its algorithmic bytes;
# (2) the C5 one-GPU leg's frame loop, 2 queues x 8 frames per launch against 1 queue x 16, three
# alternating rounds (the single-sample sweep gpu_r6_c5sweep.sh read 57 961 against 59 053).
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
K="--kernel-include-regex PrepareBinKernel"
run bin_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/bin_fetch -o run --output-format csv -- $B
run bin_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/bin_write -o run --output-format csv -- $B
python3 tools/pmc_traffic.py --key "soup-100k 1920x1080 1spp|bin|launch8" --fetch gpurun_out/bin_fetch \
    --write gpurun_out/bin_write --kernel PrepareBinKernel --largest-grid --source "$B" --out gpurun_out/pmc_traffic_bin.json
C5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 10 --warmup 2 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2 3; do
  run c5ab_q2l8_$r 200 $C5 --queues 2 --launch 8
  run c5ab_q1l16_$r 200 $C5 --queues 1 --launch 16
  echo "round $r: q2l8 $(grep -o '"value": [0-9.]*' gpurun_out/c5ab_q2l8_$r.log) q1l16 $(grep -o '"value": [0-9.]*' gpurun_out/c5ab_q1l16_$r.log)"
done
