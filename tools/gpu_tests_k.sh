#!/bin/bash
# GPU parity tests selected by PYTEST_K, without stopping at the first failure.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu_k 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "$PYTEST_K"
echo done
