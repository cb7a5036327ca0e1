#!/bin/bash
# Round 3 final evidence at HEAD: full GPU suite, smoke, default bench line under a kernel
# trace of the same run, line-vs-trace check, PMC passes of the headline and the three leg kernels.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAILN=1
step bench_traced 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03aw -o run -- python3 bench.py
T=$(find gpurun_out/prof_r03aw -name "run_kernel_trace.csv" | head -1)
grep '^{"metric"' gpurun_out/bench_traced.log > gpurun_out/r03aw_bench.json
python3 tools/trace_check.py gpurun_out/r03aw_bench.json "$T" > gpurun_out/r03aw_trace_check.json
TAILN=3
TAG=r03aw_c2 CONFIG=2 DOCS=1048576 KERNEL="join_wave_kernel<4, 8, 2, true>" BENCH_ARGS="--config 2 --legs none --no-boundary --no-sort --no-box-probe" FOLD=1 step pmc_c2 600 bash tools/pmc.sh
TAG=r03aw_c3 CONFIG=3 DOCS=1048576 KERNEL="fold_pipe_kernel<16, true, true, false>" BENCH_ARGS="--config 3 --legs none --no-boundary --no-sort --no-box-probe" FOLD=1 step pmc_c3 600 bash tools/pmc.sh
TAG=r03aw_c5 CONFIG=5 DOCS=12500000 KERNEL="fold_pipe_kernel<32, false, true, false>" BENCH_ARGS="--config 5 --legs none --no-boundary --no-sort --no-box-probe" FOLD=1 step pmc_c5 600 bash tools/pmc.sh
TAG=r03aw_c4 CONFIG=4 DOCS=16384 KERNEL="join_tile_pipe_kernel" BENCH_ARGS="--config 4 --legs none --no-boundary --no-sort --no-box-probe --repeats 1" FOLD=1 step pmc_c4 600 bash tools/pmc.sh
