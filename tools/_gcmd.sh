set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex "Bin|Trace|Super" -d gpurun_out/pmc_sq2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/pmc_sq2.log 2>&1
