#!/bin/bash
# Round 6: the compositor's deferred shading at P > 1 (rank simulation, rotated all-to-all): the product,
# the shading on a low-priority stream of its own (SRT_SHADE_STREAM=1), and 8 rows per shading thread
# (exp build shade8); two rounds.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    run rs_base_$rep 300 python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 2,8
    SRT_SHADE_STREAM=1 run rs_prio_$rep 300 python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 2,8
    SRT_LIB=simpleraytracer_amd/lib_exp/shade8/libModelRunner.so run rs_shade8_$rep 300 \
        python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 2,8
done
for f in gpurun_out/rs_*_?.log; do echo "$f"; grep -o '"P": [0-9]*\|"slowest_us": [0-9.]*' "$f" | tr '\n' ' '; echo; done
