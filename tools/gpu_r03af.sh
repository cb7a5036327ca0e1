#!/bin/bash
# Round 3: A/B of the tile kernels on one box: HEAD~ library vs working tree.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step sweep_new1 200 python -u tools/tile_sweep.py 16384 4:1 2:1 5:1
step sweep_prev1 200 env CRDTGPU_LIB=$PWD/tools/libcrdtgpu_prev.so python -u tools/tile_sweep.py 16384 4:1 2:1 5:1
step sweep_new2 200 python -u tools/tile_sweep.py 16384 4:1 2:1 5:1
step sweep_prev2 200 env CRDTGPU_LIB=$PWD/tools/libcrdtgpu_prev.so python -u tools/tile_sweep.py 16384 4:1 2:1 5:1
