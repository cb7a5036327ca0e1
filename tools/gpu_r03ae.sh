#!/bin/bash
# Round 3: tile kernels with exact vmcnt waits (unconditional loads, buffer stores), parity + sweep + stamps.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step sweep 300 python -u tools/tile_sweep.py
step tile_probe4 180 python -u tools/tile_probe.py 4
TAILN=4
step tiles 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread
