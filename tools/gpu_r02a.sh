#!/bin/bash
# Round-2 first look: GPU tests, kernel traces of configs 3/4/5, fold graph replay.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
(which go; go version; nproc; echo OMP=$OMP_NUM_THREADS; python -c 'import os; print(len(os.sched_getaffinity(0)))') > gpurun_out/probe.log 2>&1; cat gpurun_out/probe.log
step warm 240 python -c "import torch; print(torch.cuda.get_device_name(0))"
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for c in 3 4 5; do
  step prof_c$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c$c -o run -- python3 bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2
done
step graph_c3 180 python3 bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 2 --force-graph
step graph_c5 240 python3 bench.py --config 5 --no-cpu-baseline --steps 10 --warmup 2 --force-graph
