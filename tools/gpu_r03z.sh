#!/bin/bash
# Round 3: lean passes for both fold modes (delta 4 waves, AWSet 6 waves per SIMD).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step fold_tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_scenarios_gpu.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/fold_tests.log && exit 1
TAILN=3
step time_c3_lean 120 tools/fold_time 3
step time_c3_general 120 env FOLD_GENERAL=1 tools/fold_time 3
step time_c5_lean 120 tools/fold_time 5
step time_c5_general 120 env FOLD_GENERAL=1 tools/fold_time 5
TAILN=1
step bench_c35 300 python3 bench.py --config 3 --legs 5 --no-boundary --no-sort --steps 20 --warmup 5
