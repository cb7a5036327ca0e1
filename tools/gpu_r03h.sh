#!/bin/bash
# Round 3: lane-parallel slot-chain AWSet walk: fold parity, stamps, config 3/5.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step fold_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scenarios_gpu.py tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/fold_tests.log && exit 1
TAILN=14
step probe_c3 120 tools/fold_probe 3
TAILN=1
step bench_c5 300 python3 bench.py --config 3 --legs 5 --no-cpu-baseline --no-boundary --no-sort --no-box-probe --steps 20 --warmup 5
