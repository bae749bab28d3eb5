#!/bin/bash
# Full GPU-box session for a round's evidence: parity tests, smoke, the default bench line
# (with cpu_baseline + e2e), 2- and 4-rank gloo rehearsals of the N > 1 band path and the band
# simulation, rocprofv3 kernel stats of the bench (frame queues and one queue), the PMC passes
# of the trace kernel (FETCH_SIZE, WRITE_SIZE and 8 SQ counters, each a run of its own) and the
# host-cost probe of the band step (one-rank RCCL). Every GPU step has its own time limit; a crash-type exit ends the script
# (tests/lib.sh run). Output under gpurun_out/; copy what is judged into profiles/.
source "$(dirname "$0")/gpu_lib.sh"
STEPS=${STEPS:-tests,smoke,bench,c5,rehearse,prof,pmc,host}
KERNEL_RE=${KERNEL_RE:-TraceCullKernel}
KEY=${KEY:-"soup-100k 1920x1080 1spp|cull"}
Q=(--steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline)  # one frame per dispatch
if [[ $STEPS == *tests* ]]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
fi
if [[ $STEPS == *smoke* ]]; then
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == *bench* ]]; then
    run bench 600 python bench.py
    run bench_driver_shape 300 python bench.py --steps 20 --warmup 5
fi
if [[ $STEPS == *c5* ]]; then
    run bench_c5 600 python bench.py --width 3840 --height 2160 --triangles 1000000 --steps 300 --warmup 5 \
        --no-extras --no-cpu-baseline
fi
if [[ $STEPS == *rehearse* ]]; then
    for n in 2 4; do
        SRT_BENCH_BACKEND=gloo SRT_BENCH_ONE_DEVICE=1 run rehearse$n 300 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 20 \
            --warmup 2 --no-extras
    done
    run band_sim 300 python tools/band_sim.py
    run band_sim_b8 300 python tools/band_sim.py --batch 8
fi
if [[ $STEPS == *host* ]]; then
    run host_bands 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29541 tools/host_probe_bands.py
fi
if [[ $STEPS == *prof* ]]; then
    run prof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --steps 300 --warmup 5 --no-extras --no-cpu-baseline
    run prof_stats_q1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q1 -o run --output-format csv -- \
        python3 bench.py "${Q[@]}"
fi
if [[ $STEPS == *pmc* ]]; then
    run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KERNEL_RE" -d gpurun_out/pmc_fetch -o run \
        --output-format csv -- python3 bench.py "${Q[@]}"
    run pmc_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KERNEL_RE" -d gpurun_out/pmc_write -o run \
        --output-format csv -- python3 bench.py "${Q[@]}"
    run pmc_sq 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "$KERNEL_RE" \
        -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py "${Q[@]}"
    python3 tools/pmc_traffic.py --key "$KEY" --kernel "$KERNEL_RE" --fetch gpurun_out/pmc_fetch \
        --write gpurun_out/pmc_write --out gpurun_out/pmc_traffic.json
    python3 tools/pmc_sq.py --key "$KEY" --kernel "$KERNEL_RE" --dir gpurun_out/pmc_sq --out gpurun_out/pmc_sq.json
fi
echo done
