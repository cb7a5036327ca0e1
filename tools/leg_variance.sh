# bench legs 3 and 5 with and without the CPU baselines, alternating (diagnostic; GPU box only):
#   bash tools/leg_variance.sh  ->  gpurun_out/legvar_*.log
for i in 1 2; do
  for v in cpu nocpu; do
    a=""; [ "$v" = nocpu ] && a="--no-cpu-baseline"
    timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --repeats 1 --legs 3,5 --no-boundary --no-sort --no-box-probe $a > gpurun_out/legvar_${v}_$i.log 2>&1 || { echo "fail $v $i"; tail -3 gpurun_out/legvar_${v}_$i.log; exit 1; }
    python3 - gpurun_out/legvar_${v}_$i.log $v $i <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith('{"metric"')][-1])
print(sys.argv[2], sys.argv[3], 'c2 %.4f' % l['roofline']['launch_ms'], ' '.join('%s %.4f' % (k, v['roofline']['launch_ms']) for k, v in l['legs'].items()))
PY
  done
done
