#!/bin/bash
# Copy a tools/gpu_runs/gpu_round3.sh (or gpu_round.sh) session's outputs from gpurun_out/ into profiles/<dir> (tracked),
# and the PMC summaries bench.py reads into profiles/ itself.
set -eu
dir=${1:?usage: tools/save_evidence.sh profiles/rNN/evidence}
cd "$(dirname "$0")/.."
rm -rf "$dir"
mkdir -p "$dir"
for f in pytest_gpu smoke bench bench_driver_shape bench_c5 rehearse2 rehearse4 rehearse8 rank_sim rank_sim_share rank_sim_alltoall rank_sim_c5 rccl2 \
         band_sim band_sim_b8 host_bands; do
    [ -f "gpurun_out/$f.log" ] && cp "gpurun_out/$f.log" "$dir/$f.log"
done
[ -f gpurun_out/prof/run_kernel_stats.csv ] && cp gpurun_out/prof/run_kernel_stats.csv "$dir/kernel_stats.csv"
[ -f gpurun_out/prof_q1/run_kernel_stats.csv ] && cp gpurun_out/prof_q1/run_kernel_stats.csv "$dir/kernel_stats_one_queue.csv"
for f in pmc_traffic pmc_sq; do
    if [ -f "gpurun_out/$f.json" ]; then
        cp "gpurun_out/$f.json" "$dir/$f.json"
        cp "gpurun_out/$f.json" "profiles/$f.json"
    fi
done
ls "$dir"
