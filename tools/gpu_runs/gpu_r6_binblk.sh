#!/bin/bash
# Round 6: records per bin block (SRT_BIN_THREADS; tile-info tiles per block SRT_INFO_TILES), two
# interleaved rounds: the headline (driver shape, 2 queues x 8-frame launches) and one frame in flight.
# lib_exp/bt256 = the product's shape, rebuilt the same way as the others.
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  for v in bt256 bt128 bt128i2 bt512; do
    SRT_LIB=simpleraytracer_amd/lib_exp/$v/libModelRunner.so run ${v}_h_$r 150 $B
    SRT_LIB=simpleraytracer_amd/lib_exp/$v/libModelRunner.so run ${v}_s_$r 150 $S
    echo "$v round $r: headline $(grep -o '"value": [0-9.]*' gpurun_out/${v}_h_$r.log) single $(grep -o '"value": [0-9.]*' gpurun_out/${v}_s_$r.log) bin $(grep -o '"bin": [0-9.]*' gpurun_out/${v}_s_$r.log | head -1)"
  done
done
# HBM traffic of the C5 leg's launch shape (1 queue x 16 frames per launch; the product library)
B5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 3 --warmup 1 --queues 1 --launch 16 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
K="--kernel-include-regex TraceCullKernel"
run c5l16_fetch 300 timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/c5l16_fetch -o run --output-format csv -- $B5
run c5l16_write 300 timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/c5l16_write -o run --output-format csv -- $B5
python3 tools/pmc_traffic.py --key "soup-1000k 3840x2160 1spp|cull|launch16" --fetch gpurun_out/c5l16_fetch \
    --write gpurun_out/c5l16_write --kernel TraceCullKernel --largest-grid --source "$B5" --out gpurun_out/pmc_traffic_c5l16.json
