# write counters of the config-4 tile kernel per store variant (diagnostic; GPU box only)
#   bash tools/tile_write_probe.sh  ->  gpurun_out/wp/
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/wp
for v in "9 1 0" "9 0 0" "9 1 1" "0 1 0"; do
  n=$(echo $v | tr ' ' '_')
  timeout -k 10 -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/wp/$n -o run -- python3 tools/tile_write_probe.py $v > gpurun_out/wp/$n.log 2>&1
  rc=$?; echo "[wp $n] rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/wp/$n.log; exit $rc; }
  grep "survivor" gpurun_out/wp/$n.log
  python3 tools/pmc_kernel_mean.py gpurun_out/wp/$n "join_tile"
  python3 tools/pmc_kernel_mean.py gpurun_out/wp/$n "join_wave"
done
