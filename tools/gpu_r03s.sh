#!/bin/bash
# Round 3: config-4 sweep of the tile shapes (rank tiles taken after the look-back).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step sweep 300 python -u tools/tile_sweep.py
TAILN=16
step probe_c3 120 tools/fold_probe 3
