#!/bin/bash
# GPU-box check: tests, smoke, bench, kernel-trace profile.  Every GPU step has
# its own time limit; a fault, abort or timeout ends the script (exit code of
# that step); ordinary test failures (pytest rc 1) do not.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${TAG:-r01}
run() {
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run warm 240 python -c "import torch; print('hip', torch.cuda.is_available(), torch.cuda.get_device_name(0))"
[ "${SKIP_TESTS:-0}" = 1 ] || run gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-}
fi
if [ "${PMC:-0}" = 1 ]; then
  run pmc 900 bash tools/pmc.sh
fi
