#!/bin/bash
# Round 6: HBM traffic of the C5 record / bin launch (PrepareBinKernel, the C5 leg's 16-frame launches),
# two --pmc passes, against its algorithmic bytes.
source "$(dirname "$0")/gpu_lib.sh"
B5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 3 --warmup 1 --queues 1 --launch 16 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
K="--kernel-include-regex PrepareBinKernel"
run c5bin_fetch 300 timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/c5bin_fetch -o run --output-format csv -- $B5
run c5bin_write 300 timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/c5bin_write -o run --output-format csv -- $B5
python3 tools/pmc_traffic.py --key "soup-1000k 3840x2160 1spp|bin|launch16" --fetch gpurun_out/c5bin_fetch \
    --write gpurun_out/c5bin_write --kernel PrepareBinKernel --largest-grid --source "$B5" --out gpurun_out/pmc_traffic_c5bin.json
run c5_trace 300 timeout -s KILL 290 rocprofv3 --kernel-trace --stats -d gpurun_out/c5l16_trace -o run --output-format csv -- $B5
