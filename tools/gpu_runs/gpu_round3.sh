#!/bin/bash
# Round-3 evidence session on the one-GPU box (every GPU step under its own time limit; a
# crash-type exit ends the script). STEPS selects: tests, smoke, bench, c5, rehearse, ranks, prof,
# pmc, rccl2. Output under gpurun_out/; tools/save_evidence.sh copies it into profiles/.
source "$(dirname "$0")/gpu_lib.sh"
STEPS=${STEPS:-tests,smoke,bench,c5,rehearse,ranks,prof,pmc}
KERNEL_RE=${KERNEL_RE:-TraceCullKernel}
KEY=${KEY:-"soup-100k 1920x1080 1spp|cull"}
Q=(--steps 60 --warmup 5 --queues 1 --frames-per-step 1 --no-extras --no-cpu-baseline)  # one frame per dispatch
if [[ $STEPS == *tests* ]]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
fi
if [[ $STEPS == *smoke* ]]; then
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == *bench* ]]; then
    run bench 600 python bench.py
    run bench_driver_shape 300 python bench.py --steps 20 --warmup 5
fi
if [[ $STEPS == *c5* ]]; then
    run bench_c5 600 python bench.py --width 3840 --height 2160 --triangles 1000000 --steps 20 --warmup 2 \
        --no-extras --no-cpu-baseline
fi
if [[ $STEPS == *rehearse* ]]; then  # the multi-GPU path in one process on GPU 0 repeated (device copies)
    for n in 2 4 8; do
        SRT_BENCH_ONE_DEVICE=1 run rehearse$n 400 python bench.py --gpus $n --steps 20 --warmup 2 --no-e2e
    done
fi
if [[ $STEPS == *ranks* ]]; then  # per-rank GPU time of the band pipeline (exchange excluded)
    run rank_sim 400 python tools/rank_sim.py --all-ranks
    run rank_sim_c5 400 python tools/rank_sim.py --ranks 1,8 --width 3840 --height 2160 --triangles 1000000 \
        --steps 10
fi
if [[ $STEPS == *rccl2* ]]; then  # two ranks on one GPU over torchrun: does RCCL take it at all?
    SRT_BENCH_ONE_DEVICE=1 run rccl2 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 5 --warmup 1 --no-extras
fi
if [[ $STEPS == *prof* ]]; then
    run prof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --steps 50 --warmup 2 --no-extras --no-cpu-baseline
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
