#!/bin/bash
# Round 3: dense AWSet walk: fold parity (incl. dense spans, panics, config 5),
# stamps, config 3/5 timing, boundary.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step fold_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scenarios_gpu.py tests/test_host_cpp.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/fold_tests.log && exit 1
TAILN=14
step probe_c5 120 tools/fold_probe 5
TAILN=1
step bench_c3 300 python3 bench.py --config 3 --legs 5 --no-cpu-baseline --no-boundary --no-box-probe --steps 20 --warmup 5
step boundary16 300 go-crdt-playground_amd/host/build/boundary_bench 65536
