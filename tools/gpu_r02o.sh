#!/bin/bash
# Round 2: bench line after the timing changes (+ ApplyBatch scenario test).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step scen 300 python -u -m pytest tests/test_scenarios_gpu.py -x -q --timeout 300 --timeout-method thread
TAILN=2
step bench_default 900 python3 bench.py
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02o -o run -- python3 bench.py --no-cpu-baseline --no-boundary
