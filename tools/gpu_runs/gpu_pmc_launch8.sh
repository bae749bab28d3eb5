#!/bin/bash
# HBM traffic and SQ counters of TraceCullKernel in the headline launch shape (8 frames per
# launch; the largest grid of the bench run), one --pmc pass each, merged into
# profiles/pmc_traffic.json / pmc_sq.json under the bench's launch8 profile key.
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
K="--kernel-include-regex TraceCullKernel"
KEY="soup-100k 1920x1080 1spp|cull|launch8"
run l8_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/l8_fetch -o run --output-format csv -- $B
run l8_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/l8_write -o run --output-format csv -- $B
python3 tools/pmc_traffic.py --key "$KEY" --fetch gpurun_out/l8_fetch --write gpurun_out/l8_write --kernel TraceCullKernel \
    --largest-grid --source "$B" --out gpurun_out/pmc_traffic_l8.json
run l8_sq 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES $K -d gpurun_out/l8_sq -o run --output-format csv -- $B
python3 tools/pmc_sq.py --key "$KEY" --dir gpurun_out/l8_sq --kernel TraceCullKernel --largest-grid --source "$B" --out gpurun_out/pmc_sq_l8.json
