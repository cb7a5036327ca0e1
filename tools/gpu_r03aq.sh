#!/bin/bash
# Round 3: exchange input loads with cache policy aux 0 (default) / 1 / 2 (nt) / 3, one box, interleaved.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
step def$r 120 python3 tools/exchange_time.py
for a in 1 2 3; do step ld$a$r 120 env CRDTGPU_LIB=$PWD/tools/libcrdtgpu_ld$a.so python3 tools/exchange_time.py; done
done
