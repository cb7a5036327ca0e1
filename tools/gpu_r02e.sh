#!/bin/bash
# Round 2 (re-entry): full GPU suite, default bench line, kernel trace of the default bench.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=25
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=4
step bench_default 600 python3 bench.py
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- python3 bench.py --no-cpu-baseline
