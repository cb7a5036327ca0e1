#!/bin/bash
# Round 2: precomputed tile geometry -- sweep, full GPU suite, default bench line.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=9
step tile_sweep 300 python3 tools/tile_sweep.py
TAILN=15
step gpu_tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
TAILN=2
step bench_default 900 python3 bench.py
