#!/bin/bash
# Round 3: hand-written ingest sort; walk alignment fix: stamps, config 3/5
# timing, boundary + sort leg.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step sort_tests 300 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread
grep -q " failed\| error" gpurun_out/sort_tests.log && exit 1
TAILN=14
step probe_c5 120 tools/fold_probe 5
step probe_c3 120 tools/fold_probe 3
TAILN=1
step bench_c3 300 python3 bench.py --config 3 --legs 5 --no-cpu-baseline --no-boundary --no-sort --no-box-probe --steps 20 --warmup 5
step bench_c2s 300 python3 bench.py --config 2 --legs none --no-cpu-baseline --no-box-probe --steps 50 --warmup 10
