#!/bin/bash
# Round 2: PMC passes of the tile kernel (config 4) and the bench line with the boundary leg.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
FOLD=1 TAG=r02_c4t CONFIG=4 DOCS=16384 KERNEL=join_tile_kernel BENCH_ARGS="--config 4 --no-graph --repeats 1" timeout -k 10 500 bash tools/pmc.sh > gpurun_out/pmc_c4t.log 2>&1 || { echo "pmc c4 failed"; tail -30 gpurun_out/pmc_c4t.log; exit 1; }
grep -A30 "^join_tile_kernel" gpurun_out/pmc_r02_c4t/summary.txt | head -32
tail -14 gpurun_out/pmc_r02_c4t/summary.txt
source tools/gpu_step.sh
TAILN=2
step bench_default 900 python3 bench.py
