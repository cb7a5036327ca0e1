#!/bin/bash
# Round 3: delta fold prefetch addresses from an LDS region table (CRDT_FOLD_REGIONS=1)
# vs per-lane pointer selects: timing (one box, interleaved), then fold parity.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2 3; do
step r0_c3_$r 60 tools/fold_time_r0 3
step r1_c3_$r 60 tools/fold_time_r1 3
done
step r0_c5 60 tools/fold_time_r0 5
step r1_c5 60 tools/fold_time_r1 5
TAILN=3
step fold_tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_scenarios_gpu.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread
