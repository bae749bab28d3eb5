#!/bin/bash
# Cost of the record pass's double screen-box solve in situ: LIBS="base sb2" (lib_ab/, sb2 = make ab
# AB_NAME=sb2 AB_FLAGS=-DSRT_EXP_SB_TWICE, the solve done twice): rank-simulation per-frame time at
# P = 1 and 8 and the one-frame-in-flight kernel stats for each library.
source "$(dirname "$0")/gpu_lib.sh"
for lib in ${LIBS:-base sb2}; do
  SRT_LIB=simpleraytracer_amd/lib_ab/$lib/libModelRunner.so run rank_sim_$lib 300 python tools/rank_sim.py --ranks 1,8
done
LIBS="${LIBS:-base sb2}" bash "$(dirname "$0")/gpu_prof_q1.sh"
