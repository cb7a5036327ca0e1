#!/bin/bash
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step tile_probe4 180 python -u tools/tile_probe.py 4
