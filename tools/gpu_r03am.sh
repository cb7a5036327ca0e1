#!/bin/bash
# Round 3 evidence at the final kernels (aligned tile stores): full GPU suite, smoke,
# default bench line under a kernel trace, line-vs-trace check, PMC of the tile kernel.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAILN=1
step bench_traced 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03am -o run -- python3 bench.py
T=$(find gpurun_out/prof_r03am -name "run_kernel_trace.csv" | head -1)
grep '^{"metric"' gpurun_out/bench_traced.log > gpurun_out/r03am_bench.json
python3 tools/trace_check.py gpurun_out/r03am_bench.json "$T" > gpurun_out/r03am_trace_check.json
TAILN=3
TAG=r03am_c4 CONFIG=4 DOCS=16384 KERNEL="join_tile_pipe_kernel" BENCH_ARGS="--config 4 --legs none --no-boundary --no-sort --no-box-probe --repeats 1" FOLD=1 step pmc_c4 600 bash tools/pmc.sh
