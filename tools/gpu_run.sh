#!/bin/bash
# The one GPU-box script: runs the named recipes in order, each GPU step under its
# own time limit (tools/gpu_step.sh); a fault, abort or timeout ends the script.
#
#   bash tools/gpu_run.sh RECIPE...   (env: TAG=r04x, BENCH_ARGS="--config 3", CONFIGS="2 3 4 5")
#
# recipes:
#   tests    pytest -m gpu (per-config parity tests first, tests/conftest.py)
#   smoke    __graft_entry__.smoke()
#   bench    default bench line -> gpurun_out/$TAG_bench.json
#   prof     rocprofv3 kernel trace + stats of the bench (no CPU baseline) -> gpurun_out/prof_$TAG
#   configs  bench + kernel trace per config in $CONFIGS
#   pmc      PMC passes (tools/pmc.sh; one rocprofv3 --pmc run per counter group)
#   pmcall   PMC passes for every config in $CONFIGS (default 2 3 4 5) -> gpurun_out/pmc_${TAG}_cN/
#   probe    stamped fold probe (tools/fold_probe, built on the CPU side first)
#   multi    the two-process device-summary test alone
#   layout   HBM rate vs workgroup -> address mapping (tools/bw_layout)
#   bthreads boundary_bench at $BTHREADS host threads, with the box's cgroup CPU limits
#   bintr    boundary_bench with the runtime's interrupt-driven waits (default) and with polling waits
#   bpf      boundary_bench with and without the host apply's prefetch (CRDT_HOST_NO_PREFETCH; $BPF: name:ENV pairs)
#   btrace   boundary_bench (C++ mirror ExchangeBatch) with per-phase host stamps, then under a HIP API trace
#   tsweep   config-4 tile shapes (tools/tile_sweep.py, $TSHAPES as shape:nt_stores)
#   tab      config-4 exchange timed and kernel-traced per library build ($TLIBS: base or X = tools/libcrdtgpu_X.so)
#   xab      config-2 exchange store forms A/B (tools/exchange_ab.py)
#   ptest    pytest -m gpu on $PTEST (a -k expression)
#   jab      config-2 exchange timed per library build ($JLIBS: base = the product library, X = tools/libcrdtgpu_X.so)
#   ftime    fold timing builds tools/fold_time_$FTIME (space-separated variant names), interleaved, configs 3 and 5
#   tpass    config-4 exchange in passes of $TCAPS tiles vs one pass (tools/tile_passes.py)
#   bench1   boundary_bench alone (C++ mirror ExchangeBatch, every document checked)
#   lab      configs $LCONFIGS (default 3 5) timed by bench.py per library build ($LLIBS: base or X =
#            tools/libcrdtgpu_X.so), interleaved, three rounds
#   benv     boundary_bench with per-phase stamps under each runtime setting of $BENV (name:VAR=value pairs)
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAG=${TAG:-r04}
BENCH_ARGS=${BENCH_ARGS:-}
for r in "$@"; do
  case $r in
    tests)
      TAILN=4 step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      if grep -q " FAILED\| ERROR" gpurun_out/gpu_tests.log; then echo "tests failed"; exit 1; fi ;;
    smoke)
      TAILN=2 step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      TAILN=1 step bench_$TAG 600 python3 bench.py $BENCH_ARGS
      grep '^{"metric"' gpurun_out/bench_$TAG.log > gpurun_out/${TAG}_bench.json || true ;;
    prof)
      TAILN=2 step prof_$TAG 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
        -- python3 bench.py --no-cpu-baseline $BENCH_ARGS ;;
    configs)
      for c in ${CONFIGS:-2 3 4 5}; do
        TAILN=1 step bench_c${c}_$TAG 300 python3 bench.py --config $c $BENCH_ARGS
        TAILN=3 step prof_c${c}_$TAG 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d gpurun_out/prof_c${c}_$TAG -o run -- python3 bench.py --config $c --no-cpu-baseline $BENCH_ARGS
      done ;;
    pmc)
      TAILN=10 step pmc_$TAG 1200 bash tools/pmc.sh ;;
    pmcall)
      # HEAD PMC of every config's dominant kernel (tools/pmc.sh; one rocprofv3 --pmc run per counter group)
      for c in ${CONFIGS:-2 3 4 5}; do
        CONFIG=$c TAG=${TAG}_c$c TAILN=12 step pmc_${TAG}_c$c 900 bash tools/pmc.sh
        if ! grep -q "hbm_bytes_per_launch" gpurun_out/pmc_${TAG}_c$c.log; then echo "pmc c$c incomplete"; exit 1; fi
      done ;;
    probe)
      TAILN=20 step probe_c3 120 tools/fold_probe 3
      TAILN=20 step probe_c5 120 tools/fold_probe 5 ;;
    multi)
      TAILN=4 step multirank 300 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 240 --timeout-method thread ;;
    jab)
      for r in 1 2 3; do for v in ${JLIBS:-base}; do
        lib=go-crdt-playground_amd/crdtgpu/libcrdtgpu.so; [ "$v" = base ] || lib=tools/libcrdtgpu_$v.so
        TAILN=1 step jab_${v}_$r 180 env CRDTGPU_LIB=$PWD/$lib python3 tools/exchange_time.py
      done; done ;;
    ftime)
      for r in 1 2 3; do for v in ${FTIME:-base}; do for c in 3 5; do
        TAILN=1 step ftime_${v}_c${c}_$r 120 tools/fold_time_$v $c
      done; done; done ;;
    layout)
      TAILN=60 step layout_$TAG 300 tools/bw_layout ;;
    bthreads)
      { cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat 2>&1; nproc; grep Cpus_allowed_list /proc/self/status; } > gpurun_out/cgroup_$TAG.log 2>&1 || true
      for t in ${BTHREADS:-16 12 8}; do
        TAILN=1 step bthreads_${t}_$TAG 200 env CRDT_HOST_THREADS=$t go-crdt-playground_amd/host/build/boundary_bench 65536
      done
      cat /sys/fs/cgroup/cpu.stat >> gpurun_out/cgroup_$TAG.log 2>&1 || true ;;
    bintr)
      TAILN=1 step bintr_default_$TAG 200 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=1 step bintr_poll_$TAG 200 env HSA_ENABLE_INTERRUPT=0 CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=1 step bintr_default2_$TAG 200 env go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=1 step bintr_poll2_$TAG 200 env HSA_ENABLE_INTERRUPT=0 go-crdt-playground_amd/host/build/boundary_bench 65536 ;;
    bsdma)
      TAILN=1 step bsdma_off_$TAG 200 env HSA_ENABLE_SDMA=0 CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=1 step bsdma_on_$TAG 200 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=1 step bsdma_off2_$TAG 200 env HSA_ENABLE_SDMA=0 go-crdt-playground_amd/host/build/boundary_bench 65536 ;;
    bmalloc)
      # is the boundary's blocking first copy the C library returning freed heap to the OS
      # (munmap / madvise -> the GPU driver's MMU-notifier invalidations) during pack/apply?
      TAILN=40 step bmalloc_default_$TAG 200 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=40 step bmalloc_keep_$TAG 200 env CRDT_TRACE_STAGE=1 MALLOC_TRIM_THRESHOLD_=68719476736 MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TOP_PAD_=1073741824 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=2 step bmalloc_keep2_$TAG 200 env MALLOC_TRIM_THRESHOLD_=68719476736 MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TOP_PAD_=1073741824 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=2 step bmalloc_default2_$TAG 200 env go-crdt-playground_amd/host/build/boundary_bench 65536 ;;
    bspan)
      # the mirror's inputs in one page-locked block, staged by one copy (default) vs one copy per array
      for v in "span:" "perarray:CRDT_NO_SPAN_STAGING=1" "span2:" "perarray2:CRDT_NO_SPAN_STAGING=1"; do
        n=${v%%:*}; e=${v#*:}
        TAILN=12 step bspan_${n}_$TAG 200 env CRDT_TRACE_STAGE=1 $e go-crdt-playground_amd/host/build/boundary_bench 65536
      done ;;
    bcoh)
      # is each H2D staging copy's host-side delay the runtime keeping non-coherent page-locked memory coherent?
      for v in "default:" "hipcoh:HIP_HOST_COHERENT=1" "coherent:CRDT_HOST_MALLOC_FLAGS=0x40000000" "noncoh:CRDT_HOST_MALLOC_FLAGS=0x80000000" "default2:"; do
        n=${v%%:*}; e=${v#*:}
        TAILN=12 step bcoh_${n}_$TAG 200 env CRDT_TRACE_STAGE=1 $e go-crdt-playground_amd/host/build/boundary_bench 65536
      done ;;
    bpf)
      # host apply with the map elements requested a document ahead (default) vs not
      for v in ${BPF:-"pf:" "nopf:CRDT_HOST_NO_PREFETCH=1" "pf2:" "nopf2:CRDT_HOST_NO_PREFETCH=1"}; do
        n=${v%%:*}; e=${v#*:}
        TAILN=1 step bpf_${n}_$TAG 200 env $e go-crdt-playground_amd/host/build/boundary_bench 65536
      done ;;
    btrace)
      TAILN=30 step bplain_$TAG 200 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
      CRDT_TRACE_STAGE=1 TAILN=10 step btrace_$TAG 300 rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --stats \
        --output-format csv -d gpurun_out/btrace_$TAG -o run -- go-crdt-playground_amd/host/build/boundary_bench 65536 ;;
    tsweep)
      TAILN=12 step tsweep_$TAG 400 python3 tools/tile_sweep.py 16384 ${TSHAPES:-9:1 10:1 9:1 10:1 9:1 10:1} ;;
    tprobe)
      for sh in ${TPROBE:-9}; do TAILN=14 step tprobe_${sh}_$TAG 200 python3 tools/tile_probe.py $sh; done ;;
    tab)
      # config-4 exchange per library build ($TLIBS as in jab), HIP-event time and a kernel trace of each
      for r in 1 2; do for v in ${TLIBS:-base}; do
        lib=go-crdt-playground_amd/crdtgpu/libcrdtgpu.so; [ "$v" = base ] || lib=tools/libcrdtgpu_$v.so
        TAILN=3 step tab_${v}_$r 200 env CRDTGPU_LIB=$PWD/$lib python3 tools/tile_sweep.py 16384 ${TSHAPE:-9:1}
      done; done
      for v in ${TLIBS:-base}; do
        lib=go-crdt-playground_amd/crdtgpu/libcrdtgpu.so; [ "$v" = base ] || lib=tools/libcrdtgpu_$v.so
        CRDTGPU_LIB=$PWD/$lib TAILN=3 step tabprof_${v}_$TAG 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d gpurun_out/tabprof_${v}_$TAG -o run -- python3 tools/tile_sweep.py 16384 ${TSHAPE:-9:1}
      done ;;
    xab)
      TAILN=12 step xab_$TAG 400 python3 tools/exchange_ab.py ;;
    lab)
      for r in 1 2 3; do for c in ${LCONFIGS:-3 5}; do for v in ${LLIBS:-base}; do
        lib=go-crdt-playground_amd/crdtgpu/libcrdtgpu.so; [ "$v" = base ] || lib=tools/libcrdtgpu_$v.so
        TAILN=0 step lab_${v}_c${c}_$r 200 env CRDTGPU_LIB=$PWD/$lib python3 bench.py --config $c --legs none \
          --steps 50 --warmup 10 --repeats 1 --no-cpu-baseline --no-boundary --no-box-probe --no-sort
        python3 -c "import json,sys; d=json.loads(open('gpurun_out/lab_${v}_c${c}_$r.log').read().strip().splitlines()[-1]); print('lab $v c$c round $r: %.4f ms frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))" || true
      done; done; done ;;
    benv)
      for v in ${BENV:-"default:"}; do
        n=${v%%:*}; e=${v#*:}
        TAILN=6 step benv_${n}_$TAG 200 env CRDT_TRACE_STAGE=1 $e go-crdt-playground_amd/host/build/boundary_bench 65536
      done ;;
    tpass)
      TAILN=14 step tpass_$TAG 300 python3 tools/tile_passes.py 16384 ${TCAPS:-4194304 400000 300000} ;;
    bench1)
      TAILN=2 step boundary_$TAG 300 go-crdt-playground_amd/host/build/boundary_bench 65536
      TAILN=12 step boundary_stages_$TAG 300 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536 ;;
    ptest)
      TAILN=6 step ptest_$TAG 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PTEST"
      if grep -q " FAILED\| ERROR" gpurun_out/ptest_$TAG.log; then echo "tests failed"; exit 1; fi ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
done
