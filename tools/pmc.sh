#!/bin/bash
# PMC passes for the join kernel, one counter group per rocprofv3 run (gfx950
# slot limits), plus the known-byte calibration run.  GPU box only.
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r01}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
pass() {
  local name=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?; echo "[pmc $name] rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }
}
cpass() {
  local name=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/calib.py > "$OUT/$name.log" 2>&1
  local rc=$?; echo "[pmc $name] rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }
}
if [ "${FOLD:-0}" = 1 ]; then
  BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
  pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
  pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
  pass lds2 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES
  pass fetch FETCH_SIZE
  pass write WRITE_SIZE
  cpass calib_fetch FETCH_SIZE
  cpass calib_write WRITE_SIZE
  python3 tools/traffic.py "$OUT" --docs ${DOCS:-1048576} --config ${CONFIG:-3} --kernel "${KERNEL:-fold_pipe_kernel}" --emit > "$OUT/summary.txt"; cat "$OUT/summary.txt"
  exit 0
fi
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
pass tcc TCC_HIT_sum TCC_MISS_sum
cpass calib_fetch FETCH_SIZE
cpass calib_write WRITE_SIZE
# the bench's exchange shares one key column between its outputs unless BENCH_ARGS has --own-keys
case "${BENCH_ARGS:-}" in *--own-keys*) SK=0 ;; *) SK=1 ;; esac
python3 tools/traffic.py "$OUT" --docs ${DOCS:-1048576} --config ${CONFIG:-2} --kernel "${KERNEL:-join_wave_kernel}" \
  --shared-keys $SK --emit > "$OUT/summary.txt" && cat "$OUT/summary.txt"
