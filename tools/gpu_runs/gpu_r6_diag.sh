#!/bin/bash
# Round 6: per-block timeline of one frame's cull trace at the final code (diag build; tools/diag_cull.py),
# and of the record / bin launch (tools/diag_setup.py).
source "$(dirname "$0")/gpu_lib.sh"
export SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so
run diag_cull 200 python3 tools/diag_cull.py
run diag_setup 200 python3 tools/diag_setup.py
