#!/bin/bash
# PMC passes for one bench config, one counter group per rocprofv3 run (gfx950
# slot limits), plus the known-byte calibration run.  GPU box only.
#
#   CONFIG=2|3|4|5 TAG=r05x bash tools/pmc.sh
#
# Writes gpurun_out/pmc_$TAG/summary.txt and adds the entry (exact kernel
# instance + source id, tools/traffic.py) to profiles/traffic.json.
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r05}
CONFIG=${CONFIG:-2}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
case $CONFIG in
  2) KERNEL=${KERNEL:-"join_wave_kernel<4, 8, 2, true, true>"}; TUS=join.hip; DOCS=1048576; STEPS=3 ;;
  3) KERNEL=${KERNEL:-"fold_pipe_kernel<8, true, true, false>"}; TUS=fold.hip; DOCS=1048576; STEPS=2 ;;
  4) KERNEL=${KERNEL:-"join_tile_pipe_kernel<512, 2, true, true, true>"}; TUS=join.hip,tile.hip; DOCS=16384; STEPS=2 ;;
  5) KERNEL=${KERNEL:-"fold_pipe_kernel<32, false, true, false>"}; TUS=fold.hip; DOCS=12500000; STEPS=2 ;;
  *) echo "CONFIG must be 2..5"; exit 2 ;;
esac
BENCH="python3 bench.py --config $CONFIG --legs none --steps $STEPS --warmup 1 --repeats 1 --no-cpu-baseline --no-box-probe --no-sort --no-boundary ${BENCH_ARGS:-}"
pass() {
  local name=$1; shift
  timeout -k 10 -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?; echo "[pmc $name] rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }
}
cpass() {
  local name=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/calib.py > "$OUT/$name.log" 2>&1
  local rc=$?; echo "[pmc $name] rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
# L2 hits / misses and the memory-side request counts (compare boxes by counters); not fatal
timeout -k 10 -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv \
  -d "$OUT/tcc" -o run -- $BENCH > "$OUT/tcc.log" 2>&1
trc=$?; echo "[pmc tcc] rc=$trc"
case $trc in 124|137|134|139) tail -5 "$OUT/tcc.log"; exit $trc ;; esac  # a kill or a fault ends the script
if [ "${EXTRA:-0}" = 1 ]; then
  pass lds2 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES
fi
cpass calib_fetch FETCH_SIZE
cpass calib_write WRITE_SIZE
FP=stream8
if [ "$CONFIG" = 4 ] && [ -x tools/fetch_calib ]; then  # the tile kernel's element mix, calibrated on its own
  timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_mix" -o run -- tools/fetch_calib \
    > "$OUT/calib_mix.log" 2>&1
  mrc=$?; echo "[pmc calib_mix] rc=$mrc"; [ $mrc -eq 0 ] || { tail -20 "$OUT/calib_mix.log"; exit $mrc; }
  FP=mix
fi
# the bench's config-2 exchange shares one key column between its outputs unless BENCH_ARGS has --own-keys
SK=0
if [ "$CONFIG" = 2 ]; then case "${BENCH_ARGS:-}" in *--own-keys*) SK=0 ;; *) SK=1 ;; esac; fi
python3 tools/traffic.py "$OUT" --docs $DOCS --config $CONFIG --kernel "$KERNEL" --tus $TUS --shared-keys $SK \
  --profile "profiles/${TAG}_pmc_summary.txt" --fetch-pattern $FP --emit > "$OUT/summary.txt" && cat "$OUT/summary.txt"
