#!/bin/bash
# Round 3: tiles of 768 positions (4 workgroups per CU with two LDS tile buffers).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=6
step sweep1 200 python -u tools/tile_sweep.py 16384 5:1 8:1 9:1 9:0 5:1
step sweep2 200 python -u tools/tile_sweep.py 16384 8:1 9:1 5:1
TAILN=3
step tiles 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread -k "shape8 or shape9 or config4"
