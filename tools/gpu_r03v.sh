#!/bin/bash
# Round 3: pipelined tiles, next tile taken early vs after the look-back (config-4 sweep, stamps).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step sweep 300 python -u tools/tile_sweep.py
step tile_probe8 180 python -u tools/tile_probe.py 8
