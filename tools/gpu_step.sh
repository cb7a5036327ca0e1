#!/bin/bash
# Shared helper for GPU-box scripts: run one step under its own time limit,
# log to gpurun_out/<name>.log, stop the script on a fault/abort/timeout.
# usage: source tools/gpu_step.sh; step NAME SECONDS cmd...
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
  tail -n ${TAILN:-6} "gpurun_out/$name.log" | cut -c1-3000
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
export TMPDIR=/tmp
