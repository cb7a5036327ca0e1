#!/bin/bash
# Round 3: lean fold passes with one wave per workgroup vs two (one box, interleaved).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2 3; do
step w2_c3_$r 60 tools/fold_time 3
step w1_c3_$r 60 tools/fold_time_w1 3
step w2_c5_$r 60 tools/fold_time 5
step w1_c5_$r 60 tools/fold_time_w1 5
done
