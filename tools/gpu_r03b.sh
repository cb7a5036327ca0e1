#!/bin/bash
# Round 3: C++ mirror rewrite (hash interning, page-locked staging, in-place
# apply) on the GPU: scenario tests both id modes, boundary bench, probe sweep
# + new config-1 tests, then the default bench line.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=6
step host_tests 300 python -u -m pytest tests/test_host_cpp.py tests/test_scenarios_gpu.py tests/test_gpu_probe.py -x -v --timeout 250 --timeout-method thread
grep -q " failed\| error" gpurun_out/host_tests.log && exit 1
TAILN=2
step boundary 300 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary2 300 go-crdt-playground_amd/host/build/boundary_bench 262144
TAILN=1
step bench_default 700 python3 bench.py
