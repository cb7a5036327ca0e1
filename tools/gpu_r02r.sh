#!/bin/bash
# Round 2: phase shares of the fold kernels (stamped build), configs 3 and 5,
# and launch times of the unstamped kernel at 3 vs 4 waves per SIMD.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=16
step probe3 120 tools/fold_probe 3
step probe5 120 tools/fold_probe 5
TAILN=2
for v in ${VARIANTS:-w3 w4}; do
  step time3_$v 120 tools/fold_time_$v 3
  step time5_$v 120 tools/fold_time_$v 5
done
