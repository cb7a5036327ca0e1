#!/bin/bash
# Round 3: fold prefetch tuple loads plain vs non-temporal (one box, interleaved).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
step c3_def$r 60 tools/fold_time 3
step c3_ntl$r 60 tools/fold_time_ntl 3
step c5_def$r 60 tools/fold_time 5
step c5_ntl$r 60 tools/fold_time_ntl 5
done
step ex 120 python3 tools/exchange_time.py
