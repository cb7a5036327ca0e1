#!/bin/bash
# Round 3: delta folds at one wave per workgroup -- fold parity, then timing.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step fold_tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_scenarios_gpu.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/fold_tests.log && exit 1
TAILN=1
step c3 60 tools/fold_time 3
step c5 60 tools/fold_time 5
step bench_c3 300 python3 bench.py --config 3 --legs none --no-boundary --no-sort --steps 50 --warmup 10
