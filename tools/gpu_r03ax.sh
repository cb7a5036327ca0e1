#!/bin/bash
# Round 3: fold kernel array pointers re-read from the kernarg segment in the loop
# (CRDT_FOLD_KARG bits: 1 prefetch, 2 write-out) vs held in SGPRs; one box, interleaved.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2 3; do
for v in 0 1 2 3; do
step k${v}_c3_$r 60 tools/fold_time_k$v 3
step k${v}_c5_$r 60 tools/fold_time_k$v 5
done
done
