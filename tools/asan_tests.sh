#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against the AddressSanitizer + UBSan builds of the library's
# host code and of the oracle (`make asan`), on a host without a GPU: the CPU backend
# (ML_VISIBLE_DEVICES=cpu: cpu_render.cpp's threads and _Float16 paths), scene files and OBJ import,
# the ml* ABI, the screen-box host solve, the engine's pool failure handling, and the oracle.
# SURVEY.md section 5. Log: profiles/r05/asan/pytest_cpu_asan.log (ASAN_OUT).
set -o pipefail
cd "$(dirname "$0")/.."
make -s asan || exit 1
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
OUT=${ASAN_OUT:-profiles/r05/asan}
mkdir -p "$OUT"
export SRT_LIB="$PWD/simpleraytracer_amd/lib_asan/libModelRunner.so"
export SRT_ORACLE_LIB="$PWD/oracle/build_asan/libsrt_oracle.so"
export SRT_ASAN_RUN=1  # tests/conftest.py: bind the sanitized libraries, children run the normal build
# Leaks: the Python interpreter keeps its own allocations to the end; every other error stops the run.
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
{
    echo "# $(date -u +%FT%TZ) libModelRunner (host code) + oracle under -fsanitize=address,undefined"
    echo "# runtime: $RT"
    echo "# instrumented: libModelRunner $(nm -D "$SRT_LIB" | grep -c ' U __asan_') __asan_ imports," \
         "$(nm -D "$SRT_LIB" | grep -c ' U __ubsan_') __ubsan_ imports; oracle $(nm -D "$SRT_ORACLE_LIB" | grep -c ' U __asan_') __asan_ imports"
    LD_PRELOAD="$RT" python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
} 2>&1 | tee "$OUT/pytest_cpu_asan.log"
