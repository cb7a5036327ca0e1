#!/bin/bash
# Round 2: PMC passes (SQ/LDS/FETCH/WRITE + calibration) of the fold kernel (configs 3, 5) and the block join (config 4).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for spec in "3 1048576 fold_pipe_kernel" "5 12500000 fold_pipe_kernel" "4 16384 join_block_kernel"; do
  set -- $spec
  FOLD=1 TAG=r02_c$1 CONFIG=$1 DOCS=$2 KERNEL=$3 BENCH_ARGS="--config $1 --no-graph --repeats 1" timeout -k 10 500 bash tools/pmc.sh > gpurun_out/pmc_c$1.log 2>&1 || { echo "pmc c$1 failed"; tail -30 gpurun_out/pmc_c$1.log; exit 1; }
  tail -60 gpurun_out/pmc_c$1.log
done
