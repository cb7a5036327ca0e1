#!/bin/bash
# Round 3: swizzled tile LDS slots: tile parity, config 4 timing, PMC.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step tile_tests 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/tile_tests.log && exit 1
TAILN=1
step bench_c4 300 python3 bench.py --config 4 --legs none --no-cpu-baseline --no-boundary --no-sort --no-box-probe --steps 20 --warmup 5
TAILN=30
export FOLD=1
TAG=r03j_c4 CONFIG=4 DOCS=16384 KERNEL=join_tile_kernel BENCH_ARGS="--config 4 --legs none --no-boundary --no-sort --no-box-probe --repeats 1" step pmc_c4 600 bash tools/pmc.sh
TAILN=16
step probe_c3 120 tools/fold_probe 3
