#!/bin/bash
# Round 3: lean fold passes -- waves per workgroup x documents per wave (one box, interleaved; K < 64).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2 3; do
for b in fold_time fold_time_w4k32 fold_time_w2k16 fold_time_w4k16; do
step ${b}_c3_$r 60 tools/$b 3
step ${b}_c5_$r 60 tools/$b 5
done
done
