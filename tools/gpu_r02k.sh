#!/bin/bash
# Round 2: tile kernel, next tile taken after the look-back -- sweep + parity.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=8
step tile_sweep 300 python3 tools/tile_sweep.py
TAILN=6
step tile_tests 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 600 --timeout-method thread
step gc_tests 300 python -u -m pytest tests/test_gpu_gc.py tests/test_gpu_apply.py -x -q --timeout 300 --timeout-method thread
