#!/usr/bin/env python3
"""Benchmark: batched AWSet / AWSetDelta merges on MI355X.

Headline = BASELINE config 2 (the metric's configuration), per GPU (weak
scaling): 1,048,576 independent documents x 2 replicas, 64 entries per replica
state, R = 2, synthetic reachable states generated on the device
(csrc/gen.hip).  One step = one pass of the hot path over the batch: for every
document the two merges A <- B and B <- A of one snapshot (one exchange launch,
crdt_awset_exchange_async), then the per-GPU causal-context summary
(elementwise max of the output VVs), all-reduced (max, u64) across GPUs over
RCCL when N > 1 (torch.distributed's nccl backend; --engine-comm: the
engine's own communicator through the C ABI, crdt_comm_init +
crdt_context_allreduce_async, the form a Go caller binds).

The same JSON line carries one "legs" entry per other BASELINE config, each
timed the same way (warmup, barrier + synchronize, K steps, max over ranks),
with its own roofline, graph-replay check and CPU baseline:
  config3: 10 ordered AWSetDelta sources folded into each of 1,048,576 docs (R = 16)
  config4: 16,384 docs with Zipf(1.1)-like sizes up to 2^20 entries, 50%
           concurrent add/remove conflicts, both directions (block path)
  config5: 12.5M docs per GPU (100M over 8 GPUs) x 8 replicas of 16 entries
           (R = 8) folded r0 <- r1 <- ... <- r7, plus the global causal context
Inputs are resident in HBM before every timed region.  Metric: replica
merges/s (whole job); roofline: the dominant kernel's algorithmic HBM bytes
per launch / its mean launch time (HIP events on its stream) against 8 TB/s;
cpu_baseline: the hash-map C++ restatement of the reference merge
(oracle/awset_map.cpp) on every host core, with the 1-core figures and the
sorted-array C oracle beside it; the CPU baselines run after every GPU timing
(their samples are copied to the host as each config finishes).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--legs 3,4,5|none]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-crdt-playground_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
COPY_MEASURED_GBS = 6290.0  # float4 copy measured on MI355X (MI355X_MICROARCH.md; SURVEY.md 8d second denominator)


def box_probe(eng, dev, nbytes=2 << 30, reps=10):
    """This box's own HBM ceiling, measured before any timing (crdt_bw_probe):
    streaming read, write and copy over 2 GiB buffers (8x the 256 MiB
    Infinity Cache), with non-temporal and plain stores and 8/16/32
    workgroups per CU; each ceiling is the best variant, GB/s.  Boxes of one
    pool differ, so the line states the ceiling of the box that
    produced it."""
    import torch

    from crdtgpu import abi

    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(0x5A)
    torch.cuda.synchronize()
    kinds = {"read": abi.CRDT_PROBE_READ, "write_nt": abi.CRDT_PROBE_WRITE, "write_plain": abi.CRDT_PROBE_WRITE_PLAIN,
             "copy_nt": abi.CRDT_PROBE_COPY, "copy_plain": abi.CRDT_PROBE_COPY_PLAIN,
             "mix_nt": abi.CRDT_PROBE_MIX, "mix_plain": abi.CRDT_PROBE_MIX_PLAIN}
    variants = {}
    for slab in (0, 1):  # grid-stride sweep; one contiguous slab per workgroup
        eng.set_option("probe_slab", slab)
        for bpc in (8, 16, 32):
            eng.set_option("probe_blocks_per_cu", bpc)
            for name, kind in kinds.items():
                src = None if name.startswith("write") else a
                variants["%s@%d%s" % (name, bpc, "/slab" if slab else "")] = eng.bw_probe(kind, src, b, nbytes, reps)
    eng.set_option("probe_blocks_per_cu", 16)
    eng.set_option("probe_slab", 0)
    del a, b
    torch.cuda.synchronize()
    torch.cuda.empty_cache()

    def best(prefix):
        return max(v for k, v in variants.items() if k.startswith(prefix))

    ident = box_identity(dev)  # right after the probes: the clock levels under load, if the driver shows them
    return {"bytes": nbytes, "reps": reps, "read_gbs": best("read"), "write_gbs": best("write"),
            "copy_gbs": best("copy"), "mix_gbs": best("mix"), "sclk_mhz": eng.clock_probe(), "variants": variants,
            "identity": ident}


def _sysfs_card(pci):
    """The /sys/class/drm card directory of the PCI function `pci` (e.g. 0000:75:00.0), or None."""
    import glob

    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            if os.path.basename(os.path.realpath(d)).lower() == pci.lower():
                return d
        except OSError:
            continue
    return None


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def box_identity(dev):
    """What the bandwidth probes alone do not say about this box (the
    same exchange kernel ran 0.99 ms on one box and 1.23 ms on another): the
    GPU's PCI function, its compute units and XCDs as the process sees them,
    the compute / memory partition modes, and the memory (mclk), fabric (fclk)
    and shader (sclk) clock levels the driver exposes, the active level marked
    '*'.  sysfs, read-only; fields the box does not expose are null."""
    import torch

    p = torch.cuda.get_device_properties(dev)
    pci = "%04x:%02x:%02x.0" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                getattr(p, "pci_device_id", 0))
    cus = int(p.multi_processor_count)
    out = {"pci": pci, "name": p.name, "gcn_arch": getattr(p, "gcnArchName", None), "cus": cus,
           "xcds": cus // 32 if cus % 32 == 0 else None, "l2_bytes": getattr(p, "L2_cache_size", None),
           "total_mem_bytes": int(p.total_memory)}
    d = _sysfs_card(pci)
    out["sysfs"] = d
    if d:
        for f in ("current_compute_partition", "current_memory_partition", "available_compute_partition",
                  "available_memory_partition"):
            out[f] = _read(os.path.join(d, f))
        for f in ("pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_sclk", "pp_dpm_socclk"):
            v = _read(os.path.join(d, f))
            out[f] = v.splitlines() if v else None
            act = [x for x in (out[f] or []) if x.endswith("*")]
            out[f + "_active"] = act[0] if act else None
        out["power_dpm_force_performance_level"] = _read(os.path.join(d, "power_dpm_force_performance_level"))
        out["mem_info_vram_used"] = _read(os.path.join(d, "mem_info_vram_used"))
    return out


def _np_copy(t, n, dt):
    return t[:n].cpu().numpy().view(dt).copy()


def _host_batch(o, n_sample, R):
    """First n_sample docs of a device batch/output, as a host batch."""
    import numpy as np

    from crdtgpu.batch import AWSetBatch

    off = _np_copy(o.offsets, n_sample + 1, np.uint32)
    end = int(off[-1])
    return AWSetBatch(R, off, _np_copy(o.keys, end, np.uint64), _np_copy(o.actors, end, np.uint32),
                      _np_copy(o.counters, end, np.uint64), _np_copy(o.vv, R * n_sample, np.uint64),
                      counts=_np_copy(o.counts, n_sample, np.uint32))


def _host_srcs(S, n_sample, R, per_doc, E, X):
    """First n_sample docs' sources of a device SrcBuffers (per_doc sources of E entries / X tombstones each)."""
    import numpy as np

    from crdtgpu.batch import SrcBatch

    k = n_sample * per_doc
    u32, u64 = np.uint32, np.uint64
    if X:
        tomb = (_np_copy(S.tomb_off, k + 1, u32), _np_copy(S.tkeys, k * X, u64), _np_copy(S.tactors, k * X, u32),
                _np_copy(S.tcounters, k * X, u64))
    else:
        tomb = ()
    return SrcBatch(R, _np_copy(S.doc_srcs, n_sample + 1, u32), _np_copy(S.src_actor, k, u32),
                    _np_copy(S.vv, k * R, u64), _np_copy(S.entry_off, k + 1, u32), _np_copy(S.keys, k * E, u64),
                    _np_copy(S.actors, k * E, u32), _np_copy(S.counters, k * E, u64), *tomb)


def _time_cpu(fn, merges_per_call, budget_s):
    merges, t0 = 0, time.perf_counter()
    while True:
        fn()
        merges += merges_per_call
        el = time.perf_counter() - t0
        if el >= budget_s:
            return merges, el


def _cpu_baselines(label, map_bench, sorted_run, sorted_merges, budget_s):
    """The hash-map restatement on every host core (the reported value), on one
    core, and the sorted-array C oracle on one core, each for ~budget_s."""
    from oracle import oracle

    threads = oracle.cpu_threads()
    m_all, t_all = map_bench(threads, budget_s)
    m_one, t_one = map_bench(1, budget_s)
    m_arr, t_arr = _time_cpu(sorted_run, sorted_merges, budget_s)
    return {
        "value": m_all / t_all, "unit": "merges/s", "cores": threads, "kind": "port",
        "sample": "%s; C++ std::unordered_map<std::string,Dot> restatement of the reference merge "
                  "(oracle/awset_map.cpp; map[string]Dot as awset.go:55-59), %d threads over documents, maps cloned "
                  "untimed per pass, %d merges in %.1f s timed (no Go toolchain on the box: the Go reference itself "
                  "cannot run)" % (label, threads, m_all, t_all),
        "one_core": {"value": m_one / t_one, "unit": "merges/s", "cores": 1, "kind": "port",
                     "sample": "same restatement, 1 thread, %d merges in %.1f s" % (m_one, t_one)},
        "sorted_array_one_core": {"value": m_arr / t_arr, "unit": "merges/s", "cores": 1, "kind": "port",
                                  "sample": "C oracle (oracle/awset_oracle.c, sorted SoA arrays), 1 thread, "
                                            "%d merges in %.1f s" % (m_arr, t_arr)},
    }


def _outs(*bufs):
    return [getattr(b, f) for b in bufs for f in ("offsets", "counts", "keys", "actors", "counters", "vv")]


class Config2:
    """Full-state join, both directions of one snapshot (BASELINE configs[1])."""

    R = 2
    name = "config2"
    kernel = "join_wave_kernel"
    tus = ("join.hip",)  # translation units of the timed kernels (crdtgpu.srcid)
    metric = "replica-merges/sec (AWSet full-state join) + achieved HBM GB/s (% roofline)"
    exchange = True  # both merges from one read (crdt_awset_exchange_async); --separate: two join launches
    shared_keys = True  # the two outputs share one key column (same keys, same slots); --own-keys: one each
    cpu_docs = 65536

    def __init__(self, eng, n, seed, dev, stream):
        import torch

        from crdtgpu.batch import OutBuffers

        self.eng, self.n, self.stream = eng, n, stream
        R = self.R
        eng.reserve(n, 0)
        eng.set_max_doc_entries(64)  # the pair workload holds exactly 64 entries per replica
        self.A = OutBuffers(n, R, n * 64, device=dev)
        self.B = OutBuffers(n, R, n * 64, device=dev)
        eng.gen_pair_async(seed, n, self.A, self.B, stream=stream)
        self.oab = OutBuffers(n, R, 2 * n * 64, device=dev)
        self.oba = OutBuffers(n, R, 2 * n * 64, device=dev, shared_keys=self._key_owner())
        self.ctx_ab = torch.zeros(R, dtype=torch.int64, device=dev)
        self.a, self.b = self.A.as_batch(), self.B.as_batch()
        self.merges_per_step = 2 * n

    @property
    def kernel_instance(self):
        """The exact template instance the timed call launches (the ABI's default
        options: 8 docs per wave, non-temporal stores, staged stores)."""
        return "join_wave_kernel<4, 8, 2, %s, true>" % ("true" if self.exchange else "false")

    def _key_owner(self):
        """B <- A uses A <- B's key column when the exchange shares one."""
        return self.oab if (self.exchange and self.shared_keys) else None

    def _structs(self):
        if not hasattr(self, "_cs"):
            self._cs = (self.a.c(), self.b.c(), self.oab.c(), self.oba.c())
        return self._cs

    def hot(self, s):
        """The dominant launch(es): A <- B and B <- A for every doc."""
        ca, cb, cab, cba = self._structs()
        if self.exchange:
            self.eng.exchange_async(ca, cb, cab, cba, stream=s)
        else:
            self.eng.join_async(ca, cb, cab, stream=s)
            self.eng.join_async(cb, ca, cba, stream=s)

    def outputs(self):
        return _outs(self.oab, self.oba)

    def post(self, s):
        """Per-GPU causal-context summary of the outputs; returns the R-vector.
        Both merges of a pair end with the same clock, dstVV max srcVV
        (awset.go:160, crdt-misc.go:43-55, written to both outputs by the
        exchange), so the max over every output clock is the max over the A <- B
        outputs' clocks: one summary pass, not two plus a max (the oracle parity
        of both outputs' clocks: tests/test_gpu_parity.py)."""
        eng, n, R = self.eng, self.n, self.R
        eng.causal_context_async(self.oab.vv, n, R, self.ctx_ab, stream=s)
        return self.ctx_ab

    def launches_per_step(self):
        return 1 if self.exchange else 2

    def bytes_per_launch(self):
        """Algorithmic bytes of one launch: the exchange reads both states once and
        writes both outputs (workloads.exchange_bytes); separate joins: SURVEY 8d
        per merge.  Also returns the per-merge SURVEY 8d sum, for reference."""
        from crdtgpu import workloads

        cA, cB = self.A.counts.cpu().numpy(), self.B.counts.cpu().numpy()
        cab, cba = self.oab.counts.cpu().numpy(), self.oba.counts.cpu().numpy()
        per_merge = workloads.join_bytes(cA, cB, cab, self.R) + workloads.join_bytes(cB, cA, cba, self.R)
        if self.exchange:
            return workloads.exchange_bytes(cA, cB, cab, cba, self.R, self.exchange and self.shared_keys), per_merge
        return per_merge // 2, per_merge

    @property
    def kernel_name(self):
        return self.kernel + ((" (exchange: both merges of one snapshot, one read; %s)" % self._keys_what())
                              if self.exchange else "")

    def _keys_what(self):
        return ("one key column shared by the two outputs, survivors staged in LDS and stored as whole lines"
                if self.shared_keys else "a key column per output, survivors staged in LDS and stored as whole lines")

    def describe(self, world):
        return {"workload": "config2: %d docs/GPU x 2 replicas x 64 entries, R=2, full-state join: the two merges "
                            "A<-B and B<-A of one snapshot (%s) + causal-context allreduce(max,u64)" % (
                                self.n, ("one exchange launch, " + self._keys_what()) if self.exchange
                                else "two join launches"),
                "docs_per_gpu": self.n, "replicas": 2, "entries_per_replica": 64, "R": self.R,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, budget_s):
        from oracle import oracle

        n_sample = min(self.cpu_docs, self.n)
        ha, hb = _host_batch(self.A, n_sample, self.R), _host_batch(self.B, n_sample, self.R)

        def run():
            rc1, _ = oracle.join(ha, hb)
            rc2, _ = oracle.join(hb, ha)
            assert rc1 == 0 and rc2 == 0

        return lambda: _cpu_baselines("first %d docs of the batch, A<-B and B<-A" % n_sample,
                                      lambda th, b: oracle.map_bench_join(ha, hb, True, th, b), run, 2 * n_sample,
                                      budget_s)


class Config4(Config2):
    """Skewed sizes (Zipf(1.1)-like, up to 2^20 entries) with 50% concurrent
    add/remove conflicts, full-state join both directions (BASELINE configs[3])."""

    R = 2
    name = "config4"
    kernel = "join_tile_pipe_kernel"
    tus = ("join.hip", "tile.hip")
    # the tile kernel is latency-bound: one shared key column saves 0.3 % of its
    # time (9.84 vs 9.87 ms), so this leg keeps a key column per output
    shared_keys = False
    metric = "replica-merges/sec (AWSet join, Zipf sizes, config 4) + achieved HBM GB/s (% roofline)"
    cpu_docs = 96

    def __init__(self, eng, n, seed, dev, stream):
        import numpy as np
        import torch

        from crdtgpu.batch import OutBuffers
        from crdtgpu.engine import zipf_sizes

        self.eng, self.n, self.stream = eng, n, stream
        R = self.R
        sizes = zipf_sizes(seed, n)
        offs = np.zeros(n + 1, dtype=np.uint32)
        np.cumsum(sizes, out=offs[1:])
        self.total = int(offs[-1])
        self.d_offs = torch.from_numpy(offs.view(np.int32).copy()).to(dev)
        eng.reserve(n, 0)
        eng.set_max_doc_entries()  # no size promise: documents up to 2^20 entries
        self.A = OutBuffers(n, R, self.total, device=dev)
        self.B = OutBuffers(n, R, self.total, device=dev)
        eng.gen_zipf_async(seed, n, self.d_offs, self.A, self.B, stream=stream)
        self.oab = OutBuffers(n, R, 2 * self.total, device=dev)
        self.oba = OutBuffers(n, R, 2 * self.total, device=dev, shared_keys=self._key_owner())
        self.ctx_ab = torch.zeros(R, dtype=torch.int64, device=dev)
        self.a, self.b = self.A.as_batch(), self.B.as_batch()
        self.merges_per_step = 2 * n
        self.sizes = sizes

    @property
    def kernel_instance(self):
        return "join_tile_pipe_kernel<512, 2, %s, true, true>" % ("true" if self.exchange else "false")

    @property
    def kernel_name(self):
        return ("join_tile_pipe_kernel (exchange call: join_wave_kernel for docs <= 64 per side, tile plan, merge-path "
                "tiles of 1024 positions placed by a look-back deferred by one tile, stores in aligned 64-slot windows; "
                "%s; timed as the whole call)" % ("one key column shared by the two outputs" if self.shared_keys
                                                  else "a key column per output"))

    def describe(self, world):
        return {"workload": "config4: %d docs/GPU, Zipf(1.1)-like sizes in [1, 2^20) (mean %.0f, max %d, %d entries "
                            "per side), 50%% concurrent add/remove conflicts, R=2, full-state join: A<-B and B<-A of "
                            "one snapshot" % (self.n, self.sizes.mean(), self.sizes.max(), self.total),
                "docs_per_gpu": self.n, "R": self.R, "entries_per_side": self.total,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, budget_s):
        from oracle import oracle

        n_sample = min(self.cpu_docs, self.n)
        ha, hb = _host_batch(self.A, n_sample, self.R), _host_batch(self.B, n_sample, self.R)

        def run():
            rc1, _ = oracle.join(ha, hb)
            rc2, _ = oracle.join(hb, ha)
            assert rc1 == 0 and rc2 == 0

        return lambda: _cpu_baselines("first %d docs of the batch (%d entries per side), A<-B and B<-A" % (
            n_sample, int(ha.offsets[-1])), lambda th, b: oracle.map_bench_join(ha, hb, True, th, b), run,
            2 * n_sample, budget_s)


class Config3:
    """Delta-state anti-entropy: M ordered AWSetDelta sources folded per doc (BASELINE configs[2])."""

    R = 16
    M = 10
    name = "config3"
    kernel = "fold_pipe_kernel"
    kernel_instance = "fold_pipe_kernel<8, true, true, false>"
    tus = ("fold.hip",)
    kernel_name = ("fold_pipe_kernel<8, true, true, false> (per-document fold, delta: lean slot-walk pass, then the "
                   "general pass over the documents it defers; timed as the whole call)")
    metric = "replica-merges/sec (AWSetDelta fold, config 3) + achieved HBM GB/s (% roofline)"
    mode = 1  # CRDT_FOLD_DELTA
    cpu_docs = 32768

    def __init__(self, eng, n, seed, dev, stream):
        import torch

        from crdtgpu.batch import OutBuffers, SrcBuffers

        self.eng, self.n, self.stream = eng, n, stream
        R, M = self.R, self.M
        self.D = OutBuffers(n, R, n * 64, device=dev)
        self.S = SrcBuffers(R, n, n * M, n * M * 8, n * M * 2, device=dev)
        eng.gen_delta_async(seed, n, R, M, self.D, self.S, stream=stream)
        self.out = OutBuffers(n, R, n * 64 + n * M * 8, device=dev)
        eng.reserve(n, self.out.slots)
        self.ctx = torch.zeros(R, dtype=torch.int64, device=dev)
        self.d = self.D.as_batch()
        self.merges_per_step = n * M

    def hot(self, s):
        if not hasattr(self, "_cs"):
            self._cs = (self.d.c(), self.S.c(), self.out.c())
        self.eng.fold_async(self.mode, *self._cs, stream=s)

    def outputs(self):
        return _outs(self.out)

    def post(self, s):
        self.eng.causal_context_async(self.out.vv, self.n, self.R, self.ctx, stream=s)
        return self.ctx

    def launches_per_step(self):
        return 1

    def bytes_per_launch(self):
        from crdtgpu import workloads

        n, M = self.n, self.M
        b = workloads.fold_bytes(self.D.counts.cpu().numpy(), self.out.counts.cpu().numpy(), n * M * 8,
                                 n * M * 2, n * M, self.R)
        return b, b

    def describe(self, world):
        return {"workload": "config3: %d dst docs/GPU x 64 entries, R=16, %d ordered AWSetDelta sources per doc "
                            "(8 entries + 2 tombstones each), delta fold" % (self.n, self.M),
                "docs_per_gpu": self.n, "deltas_per_doc": self.M, "R": self.R,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, budget_s):
        from oracle import oracle

        n_sample = min(self.cpu_docs, self.n)
        hd = _host_batch(self.D, n_sample, self.R)
        hs = _host_srcs(self.S, n_sample, self.R, self.M, 8, 2)
        mode, merges = self.mode, n_sample * self.M  # (the thunk holds host copies only, not the device batch)

        def run():
            rc, _ = oracle.fold(mode, hd, hs)
            assert rc == 0

        return lambda: _cpu_baselines("first %d docs of the batch (%d deltas)" % (n_sample, merges),
                                      lambda th, b: oracle.map_bench_fold(mode, hd, hs, th, b), run, merges, budget_s)


class Config5(Config3):
    """100M docs x 8 replicas over 8 GPUs (BASELINE configs[4]): per GPU 12.5M docs,
    8 AWSet states of 16 entries (R = 8) folded r0 <- r1 <- ... <- r7 (7 merges
    per doc), then the global causal context: per-GPU VV max + RCCL all-reduce."""

    R = P = 8
    E = 16
    name = "config5"
    kernel = "fold_pipe_kernel"
    kernel_instance = "fold_pipe_kernel<32, false, true, false>"
    kernel_name = ("fold_pipe_kernel<32, false, true, false> (per-document fold, awset: lean slot-walk pass, then the "
                   "general pass over the documents it defers; timed as the whole call)")
    metric = "replica-merges/sec (AWSet fold r0<-..<-r7, config 5) + achieved HBM GB/s (% roofline)"
    mode = 0  # CRDT_FOLD_AWSET
    cpu_docs = 32768

    def __init__(self, eng, n, seed, dev, stream):
        import torch

        from crdtgpu.batch import OutBuffers, SrcBuffers

        self.eng, self.n, self.stream = eng, n, stream
        P, E, R = self.P, self.E, self.R
        self.D = OutBuffers(n, R, n * E, device=dev)
        self.S = SrcBuffers(R, n, n * (P - 1), n * (P - 1) * E, 0, device=dev)
        eng.gen_replicas_async(seed, n, P, E, self.D, self.S, stream=stream)
        self.out = OutBuffers(n, R, n * E * P, device=dev)
        # a doc never exceeds 16 + 7*16 = 128 slots: it stays on the wave path
        eng.reserve(n, 0)
        self.ctx = torch.zeros(R, dtype=torch.int64, device=dev)
        self.d = self.D.as_batch()
        self.merges_per_step = n * (P - 1)

    def bytes_per_launch(self):
        from crdtgpu import workloads

        n, P, E = self.n, self.P, self.E
        b = workloads.fold_bytes(self.D.counts.cpu().numpy(), self.out.counts.cpu().numpy(), n * (P - 1) * E, 0,
                                 n * (P - 1), self.R)
        return b, b

    def describe(self, world):
        return {"workload": "config5: %d docs/GPU x 8 replicas x 16 entries, R=8, fold r0<-r1<-..<-r7 + global "
                            "causal-context allreduce(max,u64) over RCCL" % self.n,
                "docs_per_gpu": self.n, "replicas": self.P, "entries_per_replica": self.E, "R": self.R,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, budget_s):
        from oracle import oracle

        n_sample = min(self.cpu_docs, self.n)
        hd = _host_batch(self.D, n_sample, self.R)
        hs = _host_srcs(self.S, n_sample, self.R, self.P - 1, self.E, 0)
        mode, merges = self.mode, n_sample * (self.P - 1)  # (the thunk holds host copies only)

        def run():
            rc, _ = oracle.fold(mode, hd, hs)
            assert rc == 0

        return lambda: _cpu_baselines("first %d docs of the batch (%d merges per pass)" % (n_sample, merges),
                                      lambda th, b: oracle.map_bench_fold(mode, hd, hs, th, b), run, merges, budget_s)


CONFIGS = {2: Config2, 3: Config3, 4: Config4, 5: Config5}
DEFAULT_DOCS = {2: 1 << 20, 3: 1 << 20, 4: 16_384, 5: 12_500_000}


def _traffic(path, config, n, W):
    """HBM bytes per launch of this kernel from the PMC passes (tools/pmc.sh ->
    tools/traffic.py --emit), or None.  An entry counts only when it was taken
    on exactly what is timed: the same config, docs, exchange form and key
    sharing, the exact kernel instance (W.kernel_instance) and the same source
    id (crdtgpu.srcid over the kernel's translation units, W.tus).  Returns
    (bytes or None, note, entry)."""
    from crdtgpu.srcid import source_id

    want_id = source_id(W.tus)
    exch = bool(getattr(W, "exchange", False))
    inst = W.kernel_instance
    if not os.path.exists(path):
        return None, "no %s" % os.path.basename(path), None
    try:
        table = json.load(open(path))
    except Exception as e:
        return None, "%s unreadable: %s" % (os.path.basename(path), e), None
    stale = None
    for e in table:
        if (e.get("docs") == n and e.get("config") == config and e.get("kernel") == inst
                and bool(e.get("exchange")) == exch
                and (not exch or bool(e.get("shared_keys", False)) == bool(W.shared_keys))):
            if e.get("src_id") == want_id:
                return e.get("hbm_bytes_per_launch"), "PMC of %s at source id %s (%s)" % (
                    inst, want_id, e.get("profile", "?")), e
            stale = e
    if stale is not None:
        return None, "the PMC entry for %s was taken at source id %s, the library is at %s: not reported" % (
            inst, stale.get("src_id"), want_id), None
    return None, "no PMC entry for %s (config %d, %d docs)" % (inst, config, n), None


def _box_fields(roof, box):
    """frac against this box's measured copy ceiling and against SURVEY 8d's 6.29 TB/s."""
    a = roof["achieved"]
    roof["frac_vs_6290"] = a / COPY_MEASURED_GBS
    if box:
        roof["box_read_gbs"] = box["read_gbs"]
        roof["box_write_gbs"] = box["write_gbs"]
        roof["box_copy_gbs"] = box["copy_gbs"]
        roof["frac_vs_box"] = a / box["copy_gbs"] if box["copy_gbs"] else None
        roof["box_mix_gbs"] = box.get("mix_gbs")
        roof["frac_vs_box_mix"] = a / box["mix_gbs"] if box.get("mix_gbs") else None
        roof["box_sclk_mhz"] = box.get("sclk_mhz")
        ident = box.get("identity") or {}
        roof["box_mclk"] = ident.get("pp_dpm_mclk_active")
        roof["box_partition"] = "%s/%s" % (ident.get("current_compute_partition"), ident.get("current_memory_partition"))
        roof["box_xcds"] = ident.get("xcds")


def run_config(config, n, args, ctx, steps, warmup, repeats, cpu, box=None):
    """Build one workload, time it, and return its result dict (the bench line's
    fields).  Inputs are generated on the device before any timing."""
    import numpy as np
    import torch

    from crdtgpu.dist import u64_max_allreduce

    eng, dev, stream, dist, world, rank, engine_comm = ctx
    backend_is_host = dist is not None and dist.get_backend() != "nccl"
    seed = args.seed + (rank << 40)  # each rank owns its own documents (weak scaling)
    cls = CONFIGS[config]
    if args.separate and config in (2, 4):
        cls.exchange = False
    if args.own_keys and config in (2, 4):
        cls.shared_keys = False
    W = cls(eng, n, seed, dev, stream)
    eng.sync(stream)

    # The dominant launch is captured once into a HIP graph and replayed each
    # step: one host call per step instead of the ABI calls of every kernel.
    # Before timing, the replayed output is compared bitwise with an eager launch.
    graph, post_graph, replay_check, graph_error, graph_ctx = None, None, None, None, None
    if not args.no_graph:
        try:
            for t in W.outputs():  # poison, so a replay that writes nothing cannot pass
                t.fill_(-1)
            W.hot(stream)  # eager launch; also warms the workspaces (no allocation during capture)
            torch.cuda.synchronize()
            eager = [t.clone() for t in W.outputs()]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                W.hot(torch.cuda.current_stream())
            gp = torch.cuda.CUDAGraph()  # the per-GPU causal-context summary, its own graph
            with torch.cuda.graph(gp):
                graph_ctx = W.post(torch.cuda.current_stream())
            torch.cuda.synchronize()
            for t in W.outputs():
                t.fill_(-1)
            g.replay()
            torch.cuda.synchronize()
            replay_check = all(bool(torch.equal(a, b)) for a, b in zip(eager, W.outputs()))
            del eager
            graph, post_graph = g, gp
        except Exception as e:  # capture refused: report it and launch eagerly
            graph_error = "%s: %s" % (type(e).__name__, e)
            torch.cuda.synchronize()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        if graph is not None:
            graph.replay()
        else:
            W.hot(stream)
        if ev is not None:
            ev[1].record(stream)
        if graph is not None:
            post_graph.replay()
            local_ctx = graph_ctx
        else:
            local_ctx = W.post(stream)
        if dist is not None:
            if backend_is_host:  # gloo rehearsal: torch.distributed on host copies
                return u64_max_allreduce(dist, local_ctx.cpu()).to(dev)
            if engine_comm:
                # the engine's own RCCL communicator, through the C ABI a Go caller binds
                eng.context_allreduce_async(local_ctx, W.R, stream=stream)
            else:  # torch.distributed over RCCL (nccl backend), u64 max via the sign flip
                return u64_max_allreduce(dist, local_ctx)
        return local_ctx

    if graph is None:
        W.hot(stream)
    eng.sync(stream)
    bytes_launch, per_merge_bytes = W.bytes_per_launch()  # from the actual output sizes
    for _ in range(warmup):  # right before the timed steps, no host pause in between
        step()
    eng.sync(stream)

    def timed():
        events = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = None
        for k in range(steps):
            g = step(events[k])
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64, device="cpu" if backend_is_host else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        # mean duration of one launch of the dominant kernel, HIP events on its stream
        tl = sum(e[0].elapsed_time(e[1]) for e in events) / steps / 1e3 / W.launches_per_step()
        return el, tl, g

    elapsed, t_launch, g = timed()
    extra = [timed()[:2] for _ in range(max(0, repeats - 1))]
    eng.sync(stream)
    achieved = bytes_launch / t_launch / 1e9
    traffic, traffic_note, _ = _traffic(args.traffic_json, config, n, W)
    merges = W.merges_per_step * world * steps
    res = {
        "metric": W.metric,
        "value": merges / elapsed,
        "unit": "merges/s",
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "launch": "hip graph replay" if graph is not None else "eager",
        "config": W.describe(world),
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_note,
            "kernel": getattr(W, "kernel_name", W.kernel), "kernel_instance": W.kernel_instance,
            "algorithmic_bytes_per_launch": bytes_launch, "launch_ms": t_launch * 1e3,
        },
        "replay_check": replay_check,
        "global_causal_context": g.cpu().numpy().view(np.uint64).tolist() if g is not None else [],
    }
    _box_fields(res["roofline"], box)
    if per_merge_bytes != bytes_launch:
        res["roofline"]["survey_8d_per_merge_bytes"] = per_merge_bytes
    if graph_error:
        res["graph_error"] = graph_error
    if extra:
        res["repeats"] = [{"ms_per_step": e / steps * 1e3, "launch_ms": t * 1e3} for e, t in extra]
    if traffic:
        res["roofline"]["traffic_gbs"] = traffic / t_launch / 1e9
        res["roofline"]["traffic_frac"] = traffic / t_launch / 1e9 / HBM_PEAK_GBS
    if cpu and rank == 0 and world == 1:
        # the host samples are copied now; the CPU work itself runs after every GPU
        # timing of the bench (main): ~10 s of an idle GPU before a leg lowered its
        # clocks for the leg's short warmup (configs 3 and 5 3.5 % / 6 % slower,
        # profiles/r06zp_leg_cpu_baseline_order.log)
        res["_cpu_baseline"] = W.cpu_baseline(args.cpu_budget)
    del graph, post_graph, W
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def ingest_sort_leg(eng, dev, stream, n, seed, reps=10):
    """The hand-written ingest sort (crdt_awset_sort_async, csrc/sort.hip) on
    one replica of the config-2 pair with every document's live entries put in
    a random order first -- the order a producer packing Go maps in iteration
    order hands over (awset.go:55-59).  Timed with HIP events on the launch
    stream; checked against the generator's sorted replica."""
    import torch

    from crdtgpu.batch import AWSetBatch, OutBuffers

    R, E = 2, 64
    A = OutBuffers(n, R, n * E, device=dev)
    B = OutBuffers(n, R, n * E, device=dev)
    eng.gen_pair_async(seed, n, A, B, stream=stream)
    torch.cuda.synchronize()
    del B
    offs = A.offsets.to(torch.int64)
    if not bool((offs[:n] == torch.arange(n, device=dev) * E).all()):
        return {"error": "generator layout is not 64 slots per doc"}
    cnt = A.counts.to(torch.int64).view(n, 1)
    pos = torch.arange(E, device=dev).view(1, E)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    # live entries first in a random order, the slack after them
    perm = torch.argsort(torch.rand(n, E, device=dev, generator=g) + (pos >= cnt).to(torch.float32) * 2, dim=1)
    perm = (perm + torch.arange(n, device=dev).view(n, 1) * E).view(-1)
    keys, acts, ctrs = A.keys[perm].contiguous(), A.actors[perm].contiguous(), A.counters[perm].contiguous()
    inb = AWSetBatch(R, A.offsets, keys, acts, ctrs, A.vv, counts=A.counts)
    out = OutBuffers(n, R, n * E, device=dev)
    eng.sort_async(inb, n * E, out, stream=stream)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with torch.cuda.stream(stream):
        ev[0].record(stream)
        for _ in range(reps):
            eng.sort_async(inb, n * E, out, stream=stream)
        ev[1].record(stream)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    live = (pos < cnt).view(-1)
    exact = bool(torch.equal(out.keys[live], A.keys[live]) and torch.equal(out.actors[live], A.actors[live])
                 and torch.equal(out.counters[live], A.counters[live]) and torch.equal(out.counts, A.counts))
    n_live = int(A.counts.to(torch.int64).sum())
    nbytes = n_live * 40 + n * (R * 16 + 16)  # entries read + written (20 B each way), VVs, bounds and counts
    return {"docs": n, "entries": n_live, "ms": ms, "docs_per_s": n / (ms * 1e-3), "entries_per_s": n_live / (ms * 1e-3),
            "achieved_gbs": nbytes / (ms * 1e-3) / 1e9, "exact": exact,
            "what": "crdt_awset_sort_async on one config-2 replica (64 slots/doc) with each doc's live entries "
                    "shuffled on the device first; %d launches timed with HIP events, result equal to the "
                    "generator's sorted replica" % reps}


def boundary_cost(n_docs):
    """the host side of the drop-in, phase by phase, through
    the C++ host mirror's ExchangeBatch (tests/cpp/boundary_bench.cpp):
    pack (hash interning with an exact per-document collision check, entries
    sorted into page-locked SoA), device (H2D + exchange + D2H), apply (results
    applied to the maps in place), next to the reference merge on the same maps
    on every host thread.  Never part of `value` (inputs there are already
    resident in HBM)."""
    import subprocess

    exe = os.path.join(ROOT, "go-crdt-playground_amd", "host", "build", "boundary_bench")
    if not os.path.exists(exe):
        return {"error": "boundary_bench not built (__graft_entry__.build())"}
    try:
        r = subprocess.run([exe, str(n_docs)], capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            return {"error": "exit %d: %s" % (r.returncode, (r.stdout + r.stderr)[-300:])}
        out = json.loads(r.stdout.strip().splitlines()[-1])
        out["what"] = ("C++ host mirror (go-crdt-playground_amd/host/crdt.hpp) ExchangeBatch: map[string]Dot-shaped "
                       "states in, both merges of every doc, the same maps updated in place; config-2-shaped docs "
                       "with 12-16 byte string keys; cpu_same_states = the reference merge on the same maps, every "
                       "host thread")
        return out
    except Exception as e:  # reported, never fatal to the bench line
        return {"error": "%s: %s" % (type(e).__name__, e)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5], help="the headline workload")
    ap.add_argument("--legs", default=None,
                    help="comma-separated configs timed after the headline (default with --config 2: 3,4,5; "
                         "otherwise none); 'none' for the headline only")
    ap.add_argument("--leg-steps", type=int, default=50)
    ap.add_argument("--leg-warmup", type=int, default=10)
    ap.add_argument("--repeats", type=int, default=3, help="timed runs of the headline (the first is the value)")
    ap.add_argument("--docs", type=int, default=None, help="documents per GPU for the headline")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-budget", type=float, default=3.0, help="seconds per CPU baseline variant")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--separate", action="store_true", help="configs 2/4: two join launches instead of one exchange")
    ap.add_argument("--own-keys", action="store_true",
                    help="configs 2/4: a key column per exchange output instead of one shared column")
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a captured HIP graph")
    ap.add_argument("--no-boundary", action="store_true", help="skip the host boundary-cost leg")
    ap.add_argument("--no-box-probe", action="store_true", help="skip the box bandwidth probes")
    ap.add_argument("--no-sort", action="store_true", help="skip the ingest-sort leg")
    ap.add_argument("--boundary-docs", type=int, default=65536)
    ap.add_argument("--engine-comm", action="store_true",
                    help="N > 1: all-reduce the summary on the engine's own RCCL communicator through the C ABI "
                         "(crdt_comm_init + crdt_context_allreduce_async) instead of torch.distributed's")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    args = ap.parse_args()

    import torch

    import crdtgpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # CRDT_BENCH_DIST_BACKEND=gloo: a rehearsal of the multi-rank path on a box
    # with fewer GPUs than ranks (ranks share GPUs; collectives on host copies).
    # The driver's runs use nccl (RCCL), one GPU per rank.
    backend = os.environ.get("CRDT_BENCH_DIST_BACKEND", "nccl")
    gpu = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream()
    eng = crdtgpu.Engine(gpu)
    collective = None
    engine_comm = False
    if world > 1:
        if backend == "nccl" and args.engine_comm:
            # crdt_comm_unique_id on rank 0, the id shared once over torch.distributed,
            # crdt_comm_init on every rank: the per-step summary all-reduce is then
            # crdt_context_allreduce_async (RCCL, u64 max) on the engine's communicator.
            # Opt-in: this form has run at one rank only (the pool's boxes have one GPU;
            # tests/test_gpu_comm.py::test_engine_comm_two_ranks runs it when >= 2 are visible).
            from crdtgpu.dist import engine_comm_handshake

            engine_comm_handshake(dist, world, rank, eng.comm_init)
            engine_comm = True
            collective = ("crdt_context_allreduce_async: RCCL all-reduce(max, u64) of R words on the engine's own "
                          "communicator (crdt_comm_unique_id + crdt_comm_init), once per step")
        elif backend == "nccl":
            collective = ("torch.distributed all-reduce(MAX) over RCCL (nccl backend) of the R-word summary, u64 order "
                          "by a sign-bit flip (crdtgpu/dist.py u64_max_allreduce), once per step")
        else:
            collective = "torch.distributed %s all-reduce of host copies (rehearsal)" % backend
    ctx = (eng, dev, stream, dist, world, rank, engine_comm)

    if args.legs is None:
        legs = [3, 4, 5] if args.config == 2 else []
    elif args.legs == "none":
        legs = []
    else:
        legs = [int(x) for x in args.legs.split(",") if x and int(x) != args.config]

    box = None if args.no_box_probe else box_probe(eng, dev)
    n = args.docs or DEFAULT_DOCS[args.config]
    head = run_config(args.config, n, args, ctx, args.steps, args.warmup, args.repeats, not args.no_cpu_baseline, box)
    result = {
        "metric": head.pop("metric"),
        "value": head.pop("value"),
        "unit": head.pop("unit"),
        "n_gpus": world,
        "steps": head.pop("steps"),
        "warmup": head.pop("warmup"),
        "ms_per_step": head.pop("ms_per_step"),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (AWSet states generated on device, csrc/gen.hip)",
    }
    result.update(head)
    if collective:
        result["config"]["collective"] = collective
    if box:
        result["box_probe"] = dict(box, what="crdt_bw_probe on this box before timing: streaming read (16 B/lane), "
                                             "write, copy (read+write bytes) and a 3:4 read:write mix (all bytes), "
                                             "best of nt/plain stores, 8/16/32 workgroups per CU and two block orders "
                                             "(grid-stride; one contiguous slab per workgroup, '/slab', which reaches "
                                             "the box's ceiling); roofline.frac_vs_box = achieved / copy_gbs, "
                                             "frac_vs_box_mix = achieved / mix_gbs; sclk_mhz: "
                                             "shader clock under an all-CU integer load (crdt_clock_probe)")
    if legs:
        result["legs"] = {}
        for c in legs:
            result["legs"]["config%d" % c] = run_config(c, DEFAULT_DOCS[c], args, ctx, args.leg_steps,
                                                        args.leg_warmup, 1, not args.no_cpu_baseline, box)
    if rank == 0 and world == 1 and not args.no_sort:
        result["ingest_sort"] = ingest_sort_leg(eng, dev, stream, DEFAULT_DOCS[2], args.seed)
    if rank == 0 and world == 1 and not args.no_boundary:
        result["boundary"] = boundary_cost(args.boundary_docs)
        if not args.no_sort:
            bs = ingest_sort_leg(eng, dev, stream, args.boundary_docs, args.seed)
            if "ms" in bs:
                # both replicas of the boundary batch, were they packed in map order
                result["boundary"]["sort_s"] = 2 * bs["ms"] * 1e-3
                result["boundary"]["sort_what"] = ("device ingest sort of both replicas of the boundary batch packed "
                                                   "in map iteration order (not on the mirror's path, which places "
                                                   "entries by id directly while packing)")
    # CPU baselines last, once the GPU timings are done (run_config)
    for r in [result] + list(result.get("legs", {}).values()):
        thunk = r.pop("_cpu_baseline", None)
        if thunk is not None:
            r["cpu_baseline"] = thunk()
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
