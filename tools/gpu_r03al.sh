#!/bin/bash
# Round 3: tile stores in aligned 64-slot windows (shapes 8, 9) vs 4, 5: time and HBM write bytes.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
export TMPDIR=/tmp
TAILN=8
step sweep 200 python -u tools/tile_sweep.py 16384 5:1 9:1 4:1 8:1 5:1 9:1
for sh in 5 9; do
step pmcw_$sh 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$sh -o run -- python3 tools/tile_sweep.py 16384 $sh:1
python3 tools/pmc_kernel_mean.py gpurun_out/pmcw_$sh join_tile_pipe
done
TAILN=3
step tiles 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread -k "shape8 or shape9"
