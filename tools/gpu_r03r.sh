#!/bin/bash
# Round 3: rank tiles (join_rank_kernel) -- tile parity tests over every shape, then the config-4 sweep.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=8
step tiles 600 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/tiles.log && exit 1
TAILN=12
step sweep 300 python -u tools/tile_sweep.py
