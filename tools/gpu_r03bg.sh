#!/bin/bash
# Round 3: is the exchange sensitive to how its buffers are mapped? default caching
# allocator vs expandable segments (virtual-memory mapped, 2 MiB granules); interleaved.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2 3; do
step def$r 120 python3 tools/exchange_time.py
step exp$r 120 env PYTORCH_HIP_ALLOC_CONF=expandable_segments:True python3 tools/exchange_time.py
done
