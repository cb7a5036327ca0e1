#!/bin/bash
# Round 2: context-reduction tests, the box's clocks/power next to the bandwidth
# probe and the headline (the exchange launch varies 1.21-1.51 ms between boxes).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step ctx_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_comm.py -k "context or comm or allreduce" -x -q --timeout 200 --timeout-method thread
grep -q " failed\| error" gpurun_out/ctx_tests.log && exit 1
TAILN=40
step smi 60 bash -c 'rocm-smi --showpower --showmaxpower --showclocks --showmemuse --showperflevel 2>&1; rocm-smi --showproductname 2>&1 | head -20'
TAILN=12
step bw_probe 120 tools/bw_probe
TAILN=2
step bench_c2 300 python3 bench.py --legs none --no-cpu-baseline --no-boundary
