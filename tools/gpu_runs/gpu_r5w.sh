#!/bin/bash
# Round 5: where a C5 P = 8 rank's time goes (rotated all-to-all, one queue, kernel trace).
source "$(dirname "$0")/gpu_lib.sh"
run c5p8_trace 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5p8_trace -o run --output-format csv -- \
    python3 tools/rank_sim.py --ranks 8 --triangles 1000000 --width 3840 --height 2160 --batch 64 --steps 4 --warmup 2 --queues 1 --exchange alltoall --rows rotated
python3 tools/trace_shapes.py gpurun_out/c5p8_trace | head -12
run c5p1_trace 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5p1_trace -o run --output-format csv -- \
    python3 tools/rank_sim.py --ranks 1 --triangles 1000000 --width 3840 --height 2160 --batch 64 --steps 4 --warmup 2 --queues 1 --exchange alltoall --rows rotated
python3 tools/trace_shapes.py gpurun_out/c5p1_trace | head -8
