#!/bin/bash
# Round 5: rotated contiguous bands + the band record pass's block skip -- parity first, then the rank
# simulation of every exchange (one GPU), then the stall counters of the headline launch shape.
source "$(dirname "$0")/gpu_lib.sh"
run t_engine 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_engine.py \
    "tests/test_gpu_parity.py::test_band_block_skip_nasty_geometry" "tests/test_gpu_parity.py::test_interleaved_bands_bitwise" \
    "tests/test_golden_full.py::test_gpu_engine_rotated_bands_reproduce_full_c3_fixture" \
    "tests/test_gpu_parity.py::test_cull_nasty_geometry" "tests/test_gpu_parity.py::test_trace_batch_c3_band_of_8"
grep -q " passed" gpurun_out/t_engine.log && ! grep -q "FAILED\|Error" gpurun_out/t_engine.log || { echo "tests failed"; exit 1; }
run rs_rot 300 python3 tools/rank_sim.py --exchange alltoall --rows rotated
run rs_share 300 python3 tools/rank_sim.py --exchange share --ranks 2,4,8
run rs_a2a 300 python3 tools/rank_sim.py --exchange alltoall --ranks 2,4,8
for P in 8 2; do
  run ps_rot$P 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ps_rot$P -o run --output-format csv -- \
      python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 10
done
bash tools/gpu_runs/gpu_r5_stalls.sh
