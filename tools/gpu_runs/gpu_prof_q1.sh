#!/bin/bash
# One-frame-in-flight kernel stats (rocprofv3) per library: LIBS="base ..." from lib_ab/.
source "$(dirname "$0")/gpu_lib.sh"
for lib in ${LIBS:-base}; do
  SRT_LIB=simpleraytracer_amd/lib_ab/$lib/libModelRunner.so run prof_q1_$lib 300 rocprofv3 --kernel-trace --stats \
      -d gpurun_out/prof_q1_$lib -o run --output-format csv -- python3 bench.py --steps 300 --warmup 20 --queues 1 \
      --frames-per-step 1 --no-extras --no-cpu-baseline || exit 1
done
for lib in ${LIBS:-base}; do
  echo "== $lib"; f=$(find gpurun_out/prof_q1_$lib -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,re,sys
for r in csv.DictReader(open('$f')):
    m=re.search(r'(\\w+)\\(', r['Name']); n=m.group(1) if m else r['Name']
    print(f\"{n:28s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.2f} us  min {float(r['MinNs'])/1e3:8.2f}\")"
done
