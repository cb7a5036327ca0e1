#!/bin/bash
# Round 3 final HEAD check: full GPU suite, smoke, default bench line.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1
step bench 600 python3 bench.py
grep '^{"metric"' gpurun_out/bench.log > gpurun_out/r03bk_bench.json
