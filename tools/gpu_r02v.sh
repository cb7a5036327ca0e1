#!/bin/bash
# Round 2 final: tile tests + config-4 timing (look-back DPP sum), full GPU
# suite, smoke, default bench line, kernel trace of the default bench.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step tile_tests 400 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/tile_tests.log && exit 1
TAILN=1
step bench_c4 300 python3 bench.py --config 4 --legs none --no-cpu-baseline --no-boundary --steps 20 --warmup 5
TAILN=4
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1
step bench_default 600 python3 bench.py
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v -o run -- python3 bench.py --no-cpu-baseline --no-boundary
