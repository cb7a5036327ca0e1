#!/bin/bash
# GPU box: bench + kernel-trace profile of configs 3 and 5 (config 2 is gpu_check.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${TAG:-r01}
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_c$c.log 2>&1
  rc=$?; echo "[bench config $c] rc=$rc"; tail -2 gpurun_out/bench_c$c.log | cut -c1-2000
  if [ $rc -ne 0 ]; then exit $rc; fi
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c${c}_$TAG -o run -- python3 bench.py --config $c --no-cpu-baseline > gpurun_out/prof_c$c.log 2>&1
  rc=$?; echo "[prof config $c] rc=$rc"; head -4 gpurun_out/prof_c${c}_$TAG/run_kernel_stats.csv | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
done
