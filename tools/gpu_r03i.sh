#!/bin/bash
# Round 3: PMC passes of the fold kernels after the slot walks (configs 3, 5).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=30
export FOLD=1
TAG=r03i_c3 CONFIG=3 DOCS=1048576 KERNEL="fold_pipe_kernel<32, true>" BENCH_ARGS="--config 3 --legs none --no-boundary --no-sort --no-box-probe" step pmc_c3 600 bash tools/pmc.sh
TAG=r03i_c5 CONFIG=5 DOCS=12500000 KERNEL="fold_pipe_kernel<32, false>" BENCH_ARGS="--config 5 --legs none --no-boundary --no-sort --no-box-probe" step pmc_c5 600 bash tools/pmc.sh
