#!/bin/bash
# Round 2: tile shape sweep (config 4), batched local ops parity.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=8
step tile_sweep 300 python3 tools/tile_sweep.py
TAILN=25
step apply_tests 600 python -u -m pytest tests/test_gpu_apply.py -x -v --timeout 300 --timeout-method thread
