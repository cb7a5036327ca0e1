#!/bin/bash
# Round 3, first GPU call: new tests (probe, multirank, apply tomb validation),
# the full GPU suite, smoke, and the default bench line under a kernel trace
# (line and trace from ONE run, so launch_ms and the trace average can be compared).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step new_tests 300 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_multirank.py tests/test_gpu_apply.py tests/test_scenarios_gpu.py -x -v --timeout 250 --timeout-method thread
grep -q " failed\| error" gpurun_out/new_tests.log && exit 1
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1
step bench_traced 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03a -o run -- python3 bench.py
