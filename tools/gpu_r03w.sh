#!/bin/bash
# Round 3: deferred-look-back tiles as the default: tile parity, config-4 leg, PMC of the new kernel.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step tiles 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/tiles.log && exit 1
TAILN=1
step bench_c4 300 python3 bench.py --config 4 --legs none --no-boundary --no-sort --steps 20 --warmup 5
TAILN=30
TAG=r03w_c4 CONFIG=4 DOCS=16384 KERNEL=join_tile_pipe_kernel BENCH_ARGS="--config 4 --legs none --no-boundary --no-sort --no-box-probe --repeats 1" FOLD=1 step pmc_c4 600 bash tools/pmc.sh
