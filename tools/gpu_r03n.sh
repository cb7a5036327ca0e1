#!/bin/bash
# Round 3: device-side key-order check + packed downloads in the *_batch
# calls: parity (host paths), C++ mirror, boundary.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step host_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scenarios_gpu.py tests/test_host_cpp.py tests/test_gpu_apply.py tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/host_tests.log && exit 1
TAILN=1
step boundary16 300 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary16b 300 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary2 300 go-crdt-playground_amd/host/build/boundary_bench 262144
