#!/bin/bash
# Round 3: config-4 tile stores, non-temporal vs plain: HBM write bytes per tile-kernel launch.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
export TMPDIR=/tmp
TAILN=8
for nt in 1 0; do
step pmcw_nt$nt 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_nt$nt -o run -- python3 tools/tile_sweep.py 16384 5:$nt
python3 tools/pmc_kernel_mean.py gpurun_out/pmcw_nt$nt join_tile_pipe
step pmcf_nt$nt 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_nt$nt -o run -- python3 tools/tile_sweep.py 16384 5:$nt
python3 tools/pmc_kernel_mean.py gpurun_out/pmcf_nt$nt join_tile_pipe
done
