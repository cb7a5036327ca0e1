#!/bin/bash
# Round 3: AWSet lean pass at 7 waves per SIMD vs 6.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=2
step time_c5_w6 120 tools/fold_time 5
step time_c5_w7 120 tools/fold_time_a7 5
step time_c5_w6b 120 tools/fold_time 5
step time_c5_w7b 120 tools/fold_time_a7 5
