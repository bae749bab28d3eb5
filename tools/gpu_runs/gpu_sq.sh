#!/bin/bash
# SQ instruction counters of TraceCullKernel (one rocprofv3 --pmc pass per configuration, 8 SQ
# counters each): the product library, then the diag build with SRT_EXP bits (64 = skip the
# packet walk) to split the counts by phase. Output: gpurun_out/sq_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CNT="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
BENCH=(python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --brute-steps 0 --queues 1)
for cfg in ${CFGS:-product}; do
    case $cfg in
        product) lib=""; exp="" ;;
        diag*) lib=simpleraytracer_amd/lib_diag/libModelRunner.so; exp=${cfg#diag} ;;
    esac
    SRT_LIB=$lib SRT_EXP=$exp timeout -s KILL 90 rocprofv3 --pmc $CNT --kernel-include-regex TraceCullKernel \
        -d gpurun_out/sq_$cfg -o run --output-format csv -- "${BENCH[@]}" > gpurun_out/sq_$cfg.log 2>&1
    rc=$?
    echo "$cfg rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
