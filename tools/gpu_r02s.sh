#!/bin/bash
# Round 2: fold parity tests, then phase shares and launch times of the fold.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step fold_tests 400 python -u -m pytest tests/test_gpu_parity.py -k "fold or config3 or config5" -x -q --timeout 200 --timeout-method thread
grep -q " failed\| error" gpurun_out/fold_tests.log && exit 1
TAILN=16
step probe3 120 tools/fold_probe 3
step probe5 120 tools/fold_probe 5
TAILN=2
for v in ${VARIANTS:-w3 w4}; do
  step time3_$v 120 tools/fold_time_$v 3
  step time5_$v 120 tools/fold_time_$v 5
done
