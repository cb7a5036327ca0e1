#!/bin/bash
# Round 3: phase stamps of the config-4 tile kernel (look-back vs dispense split).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step tile_probe2 180 python -u tools/tile_probe.py 2
