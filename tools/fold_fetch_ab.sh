# FETCH_SIZE / WRITE_SIZE of the config-3 lean delta pass per library (diagnostic; GPU box only):
#   FLIBS="base xcd2" bash tools/fold_fetch_ab.sh  ->  gpurun_out/ffa_*
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in ${FLIBS:-base}; do
  lib=go-crdt-playground_amd/crdtgpu/libcrdtgpu.so; [ "$v" = base ] || lib=tools/libcrdtgpu_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    CRDTGPU_LIB=$PWD/$lib timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/ffa_${v}_$c -o run -- python3 bench.py --config ${FCONFIG:-3} --legs none --steps 2 --warmup 1 --repeats 1 --no-cpu-baseline --no-box-probe --no-sort --no-boundary > gpurun_out/ffa_${v}_$c.log 2>&1 || { echo "fail $v $c"; tail -3 gpurun_out/ffa_${v}_$c.log; exit 1; }
    echo "$v $(python3 tools/pmc_kernel_mean.py gpurun_out/ffa_${v}_$c 'fold_pipe_kernel<' | grep 'true, false>')"
  done
done
