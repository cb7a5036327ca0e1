#!/bin/bash
# Round 2: tile kernel store policy sweep + write traffic with plain stores.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=9
step tile_sweep 300 python3 tools/tile_sweep.py
export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c4w -o run -- python3 bench.py --config 4 --no-graph --repeats 1 --steps 2 --warmup 1 --no-cpu-baseline --no-boundary > gpurun_out/pmc_c4w.log 2>&1; echo "pmc rc=$?"
python3 tools/traffic.py gpurun_out/pmc_c4w --docs 16384 --config 4 --kernel join_tile_kernel | grep -A3 "^join_tile" | head -4
