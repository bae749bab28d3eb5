#!/bin/bash
# Round 6: bin-launch knobs re-checked at the final code (tile boxes loaded ahead per bin thread
# SRT_BIN_AHEAD 2 / 4 (product) / 8; tile-info tiles per block SRT_INFO_TILES 4 against 2), headline driver
# shape and one frame in flight, two alternating rounds.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  line="round $r:"
  for v in ba4 ba2 ba8 it4; do
    SRT_LIB=$L/$v/libModelRunner.so run k${v}_h_$r 150 $B
    SRT_LIB=$L/$v/libModelRunner.so run k${v}_s_$r 150 $S
    line="$line $v $(grep -o '"value": [0-9.]*' gpurun_out/k${v}_h_$r.log | head -1 | cut -d' ' -f2)/$(grep -o '"value": [0-9.]*' gpurun_out/k${v}_s_$r.log | head -1 | cut -d' ' -f2)"
  done
  echo "$line"
done
