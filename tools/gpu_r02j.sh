#!/bin/bash
# Round 2: prefetching tile kernel (sweep + parity), apply parity, boundary-cost binary.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=8
step tile_sweep 300 python3 tools/tile_sweep.py
TAILN=6
step tile_tests 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 600 --timeout-method thread
step apply_tests 600 python -u -m pytest tests/test_gpu_apply.py -x -q --timeout 300 --timeout-method thread
TAILN=3
step boundary 300 go-crdt-playground_amd/host/build/boundary_bench 65536
