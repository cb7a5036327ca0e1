#!/bin/bash
# Round 2: the new bench line (headline + legs) -- quick pass, then the default run.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step bench_quick 400 python3 bench.py --steps 10 --leg-steps 5 --repeats 2 --cpu-budget 1
step bench_default 600 python3 bench.py
