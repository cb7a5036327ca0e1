# kernel trace of the fold passes (lean + deferred list) per library: bash tools/fold_list_trace.sh (GPU box; diagnostic)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in ${LTLIBS:-base}; do
  lib=go-crdt-playground_amd/crdtgpu/libcrdtgpu.so; [ "$v" = base ] || lib=tools/libcrdtgpu_$v.so
  for c in 3 5; do
    CRDTGPU_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lt_${v}_c$c -o run -- python3 bench.py --config $c --legs none --steps 30 --warmup 5 --repeats 1 --no-cpu-baseline --no-boundary --no-box-probe --no-sort > gpurun_out/lt_${v}_c$c.log 2>&1 || { echo "fail $v $c"; tail -5 gpurun_out/lt_${v}_c$c.log; exit 1; }
    python3 - gpurun_out/lt_${v}_c$c $v $c <<'PY'
import csv,glob,sys
from collections import defaultdict
d=defaultdict(list)
for f in glob.glob(sys.argv[1]+'/**/*kernel_trace.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        if 'fold' in r['Kernel_Name']: d[r['Kernel_Name'].split('(')[0][-45:]].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in d.items(): v=sorted(v); print(sys.argv[2],'c'+sys.argv[3],k,len(v),'median %.1f us'%v[len(v)//2])
PY
  done
done
