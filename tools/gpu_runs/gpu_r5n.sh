#!/bin/bash
# Round 5: what bounds the deferred shading (ShadeIdsKernel of a P = 8 rank, rotated all-to-all, one
# queue): SQ wait / issue mix, L2 hit rate, HBM bytes; one --pmc pass each.
source "$(dirname "$0")/gpu_lib.sh"
R="python3 tools/rank_sim.py --ranks ${SH_P:-8} --exchange alltoall --rows rotated --queues 1 --steps 3 --warmup 1"
K="--kernel-include-regex ShadeIdsKernel"
pass() { local n=$1; shift; run sh_$n 120 timeout -s KILL 100 rocprofv3 --pmc "$@" $K -d gpurun_out/sh_$n -o run --output-format csv -- $R; }
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM
pass tcc TCC_HIT_sum TCC_MISS_sum
pass fetch FETCH_SIZE
pass write WRITE_SIZE
for n in sq sq2 tcc fetch write; do
  python3 tools/pmc_sq.py --key shade_p8_$n --dir gpurun_out/sh_$n --kernel ShadeIdsKernel --out gpurun_out/sh_pmc.json
done
cat gpurun_out/sh_pmc.json
timeout -k 5 60 rocprofv3 -L > gpurun_out/avail.txt 2>&1; echo "avail rc=$?"
