#!/bin/bash
# ShadeIdsKernel of a P = 8 rank (tools/rank_sim.py, 64-frame launches): HBM bytes (FETCH_SIZE,
# WRITE_SIZE) and the instruction / wait mix, one --pmc pass each.
source "$(dirname "$0")/gpu_lib.sh"
R="python3 tools/rank_sim.py --ranks 8 --steps 5"
K="--kernel-include-regex ShadeIdsKernel"
run shade_fetch 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/shade_fetch -o run --output-format csv -- $R
run shade_write 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/shade_write -o run --output-format csv -- $R
python3 tools/pmc_kernels.py gpurun_out/shade_fetch gpurun_out/shade_write
run shade_sq 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY $K -d gpurun_out/shade_sq -o run --output-format csv -- $R
python3 tools/pmc_sq.py --key shade_rank8 --dir gpurun_out/shade_sq --kernel ShadeIdsKernel --out gpurun_out/shade_sq.json && cat gpurun_out/shade_sq.json
