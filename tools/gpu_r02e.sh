#!/bin/bash
# Round 2: full GPU test suite after the stream-ordering / capture changes.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=25
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
