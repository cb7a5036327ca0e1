#!/bin/bash
# Round 2: ingest sort parity.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step sort_tests 600 python -u -m pytest tests/test_gpu_sort.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread
