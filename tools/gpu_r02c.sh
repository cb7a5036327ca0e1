#!/bin/bash
# Round 2: PMC passes of the fold kernel for configs 3 and 5.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
FOLD=1 TAG=r02_c3 DOCS=1048576 BENCH_ARGS="--config 3 --no-graph" timeout -k 10 400 bash tools/pmc.sh > gpurun_out/pmc_c3.log 2>&1 || { echo "pmc c3 failed"; tail -30 gpurun_out/pmc_c3.log; exit 1; }
tail -40 gpurun_out/pmc_c3.log
FOLD=1 TAG=r02_c5 DOCS=12500000 BENCH_ARGS="--config 5 --no-graph" timeout -k 10 400 bash tools/pmc.sh > gpurun_out/pmc_c5.log 2>&1 || { echo "pmc c5 failed"; tail -30 gpurun_out/pmc_c5.log; exit 1; }
tail -40 gpurun_out/pmc_c5.log
