#!/bin/bash
# Band simulation (tools/band_sim.py) at C5 (3840x2160, 1M triangles) and at C3 with 2 queues.
source "$(dirname "$0")/gpu_lib.sh"
run band_sim_c5 600 python tools/band_sim.py --width 3840 --height 2160 --triangles 1000000 --steps 200 --warmup 5
run band_sim_q2 300 python tools/band_sim.py --queues 2
echo done
