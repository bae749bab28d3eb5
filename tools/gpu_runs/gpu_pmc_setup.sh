#!/bin/bash
# HBM bytes of the per-frame setup kernels (one frame per dispatch): FETCH_SIZE and WRITE_SIZE
# passes, each a run of its own, for TileInfoKernel / PrepareBinKernel / WorkOrderKernel.
source "$(dirname "$0")/gpu_lib.sh"
Q="--steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline"
RE="TileInfoKernel|PrepareBinKernel|WorkOrderKernel|TraceCullKernel"
run pmc_setup_fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" -d gpurun_out/pmc_setup_fetch -o run --output-format csv -- python3 bench.py $Q
run pmc_setup_write 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" -d gpurun_out/pmc_setup_write -o run --output-format csv -- python3 bench.py $Q
echo done
