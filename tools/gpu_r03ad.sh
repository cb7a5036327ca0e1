#!/bin/bash
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=30
TAG=r03ad_c3 CONFIG=3 DOCS=1048576 KERNEL="fold_pipe_kernel<32, true, true, false>" BENCH_ARGS="--config 3 --legs none --no-boundary --no-sort --no-box-probe" FOLD=1 step pmc_c3 600 bash tools/pmc.sh
