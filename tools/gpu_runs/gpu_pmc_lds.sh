source tools/gpu_runs/gpu_lib.sh
Q="--steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline"
run pmcA 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex TraceCullKernel -d gpurun_out/pmcA -o run --output-format csv -- python3 bench.py $Q
run pmcB 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex TraceCullKernel -d gpurun_out/pmcB -o run --output-format csv -- python3 bench.py $Q
