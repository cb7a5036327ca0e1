#!/bin/bash
# Round 3: after the walk's alignment fix: stamps, config 3/5 timing, boundary.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=14
step probe_c5 120 tools/fold_probe 5
step probe_c3 120 tools/fold_probe 3
TAILN=1
step bench_c3 300 python3 bench.py --config 3 --legs 5 --no-cpu-baseline --no-boundary --no-box-probe --steps 20 --warmup 5
step boundary16 300 go-crdt-playground_amd/host/build/boundary_bench 65536
