#!/bin/bash
# Round 2: box bandwidth ceiling next to the exchange timing, and a 2-rank
# rehearsal of bench.py's multi-rank path (gloo, both ranks on the one GPU).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=20
step bw_probe 120 tools/bw_probe
TAILN=3
step bench_c2 300 python3 bench.py --legs none --no-cpu-baseline --no-boundary
export CRDT_BENCH_DIST_BACKEND=gloo
step rehearsal 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 5 --leg-steps 3 --leg-warmup 1 --repeats 1 --no-cpu-baseline
