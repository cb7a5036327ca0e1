#!/bin/bash
# Round 3: exchange output stores with cache policy aux 2 (nt, default) vs 1, 3, 6; one box, interleaved.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
step def$r 120 python3 tools/exchange_time.py
for a in 1 3 6; do step st$a$r 120 env CRDTGPU_LIB=$PWD/tools/libcrdtgpu_st$a.so python3 tools/exchange_time.py; done
done
