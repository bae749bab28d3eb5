#!/bin/bash
# Where a single frame's setup latency goes (one frame per dispatch, one in flight): the diag build's
# PrepareBinKernel with SRT_EXP knockouts (1: no tile ranges / bins, 4: no global list reservations,
# 512: no screen-box solve), and the kernel mix of one P = 8 band rank's stream (rank simulation).
source "$(dirname "$0")/gpu_lib.sh"
Q="--steps 300 --warmup 20 --queues 1 --frames-per-step 1 --no-extras --no-cpu-baseline"
for e in ${EXPS:-0 1 4 512}; do
    SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so SRT_EXP=$e run exp_$e 200 rocprofv3 --kernel-trace --stats \
        -d gpurun_out/exp_$e -o run --output-format csv -- python3 bench.py $Q
done
run prof_rank8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rank8 -o run --output-format csv -- \
    python3 tools/rank_sim.py --ranks 8 --steps 20
run prof_rank1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rank1 -o run --output-format csv -- \
    python3 tools/rank_sim.py --ranks 1 --steps 20
for d in gpurun_out/exp_* gpurun_out/prof_rank8 gpurun_out/prof_rank1; do
  echo "== $d"; f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,re
for r in csv.DictReader(open('$f')):
    m=re.search(r'(\w+)(<[^(]*)?\(', r['Name']); n=m.group(1) if m else r['Name'][:40]
    print(f\"{n:28s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.2f} us  tot {float(r['TotalDurationNs'])/1e6:8.3f} ms\")"
done
