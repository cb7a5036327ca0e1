#!/bin/bash
# Round 3: folds with the prefetch registers consumed at the loop top (no in-order vmcnt waits on the stores).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=2
step time_c3 120 tools/fold_time 3
step time_c3g 120 env FOLD_GENERAL=1 tools/fold_time 3
step time_c5 120 tools/fold_time 5
step time_c5g 120 env FOLD_GENERAL=1 tools/fold_time 5
TAILN=4
step fold_tests 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fold or config3 or config5 or gen"
