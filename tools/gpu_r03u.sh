#!/bin/bash
# Round 3: pipelined look-back tiles (join_tile_pipe_kernel): tile parity over every shape, config-4 sweep, stamps.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step sweep 300 python -u tools/tile_sweep.py
step tile_probe4 180 python -u tools/tile_probe.py 4
TAILN=6
step tiles 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread
