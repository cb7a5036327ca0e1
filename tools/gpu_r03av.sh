#!/bin/bash
# Round 3: exchange wave kernel with 1/2/8 waves per workgroup vs 4 (one box, interleaved).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
step def$r 120 python3 tools/exchange_time.py
for a in 1 2 8; do step jw$a$r 120 env CRDTGPU_LIB=$PWD/tools/libcrdtgpu_jw$a.so python3 tools/exchange_time.py; done
done
