#!/bin/bash
# Round 3: fold survivors with plain vs non-temporal stores (time and HBM write bytes).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
export TMPDIR=/tmp
TAILN=1
for r in 1 2; do
step c3_nt$r 60 tools/fold_time 3
step c3_plain$r 60 tools/fold_time_plain 3
step c5_nt$r 60 tools/fold_time 5
step c5_plain$r 60 tools/fold_time_plain 5
done
TAILN=4
for b in fold_time fold_time_plain; do
for c in 3 5; do
step pmc_${b}_$c 90 rocprofv3 --pmc WRITE_SIZE FETCH_SIZE --output-format csv -d gpurun_out/pmc_${b}_$c -o run -- tools/$b $c
python3 tools/pmc_kernel_mean.py gpurun_out/pmc_${b}_$c fold_pipe_kernel
done
done
