#!/bin/bash
# Round 2 (after the fold changes): full GPU suite, default bench line, kernel
# trace of the default bench, PMC passes of the fold kernels (configs 3, 5).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=6
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=2
step bench_default 600 python3 bench.py
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_t -o run -- python3 bench.py --no-cpu-baseline --no-boundary
export FOLD=1
TAG=r02t_c3 CONFIG=3 DOCS=1048576 KERNEL="fold_pipe_kernel<32, true>" BENCH_ARGS="--config 3 --legs none --no-boundary" step pmc_c3 600 bash tools/pmc.sh
TAG=r02t_c5 CONFIG=5 DOCS=12500000 KERNEL="fold_pipe_kernel<32, false>" BENCH_ARGS="--config 5 --legs none --no-boundary" step pmc_c5 600 bash tools/pmc.sh
