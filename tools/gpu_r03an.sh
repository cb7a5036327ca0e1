#!/bin/bash
# Round 3: fold prefetch reading its tuple bases from LDS (fewer live kernel-argument scalars) vs HEAD, same box.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
step c3_new$r 60 tools/fold_time 3
step c3_prev$r 60 tools/fold_time_prev 3
step c5_new$r 60 tools/fold_time 5
step c5_prev$r 60 tools/fold_time_prev 5
done
TAILN=3
step fold_tests 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fold or config3 or config5 or gen"
