#!/usr/bin/env python3
"""Benchmark: batched AWSet / AWSetDelta merges on MI355X.

Default workload = BASELINE config 2 (the metric's configuration), per GPU
(weak scaling): 1,048,576 independent documents x 2 replicas, 64 entries per
replica state, R = 2, synthetic reachable states generated on the device
(csrc/gen.hip).  One step = one pass of the hot path over the batch:
  A <- B and B <- A for every document (2 merges per doc, crdt_awset_join_async),
  then the per-GPU causal-context summary (elementwise max of the output VVs),
  all-reduced (max, u64) across GPUs over RCCL when N > 1.
--config 3: delta-state anti-entropy -- 10 ordered AWSetDelta sources folded
  into each of 1,048,576 docs (R = 16): 10,485,760 merges per step.
--config 4: 16,384 docs with Zipf(1.1)-like sizes up to 2^20 entries, 50%
  concurrent add/remove conflicts, joined both directions (block path).
--config 5: 12.5M docs per GPU (100M over 8 GPUs) x 8 replicas of 16 entries
  (R = 8) folded r0 <- r1 <- ... <- r7, plus the global causal context.
Inputs are resident in HBM before the timed region.  Metric: replica merges/s
(whole job), with the dominant kernel's achieved algorithmic HBM bandwidth
against the 8 TB/s roofline and the C oracle timed on the host beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
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


def _time_cpu(fn, merges_per_call, budget_s):
    merges, t0 = 0, time.perf_counter()
    while True:
        fn()
        merges += merges_per_call
        el = time.perf_counter() - t0
        if el >= budget_s:
            return merges, el


class Config2:
    """Full-state join, both directions (BASELINE configs[1])."""

    R = 2
    kernel = "join_wave_kernel"
    metric = "replica-merges/sec (AWSet full-state join) + achieved HBM GB/s (% roofline)"

    exchange = True  # both directions from one read (crdt_awset_exchange_async); --separate: two joins
    graph_ok = True  # hot() is one kernel launch, replayed from a captured HIP graph (validated on MI355X)

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
        self.oba = OutBuffers(n, R, 2 * n * 64, device=dev)
        self.ctx_ab = torch.zeros(R, dtype=torch.int64, device=dev)
        self.ctx_ba = torch.zeros(R, dtype=torch.int64, device=dev)
        self.a, self.b = self.A.as_batch(), self.B.as_batch()
        self.merges_per_step = 2 * n

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

    def post(self, s):
        """Per-GPU causal-context summary of the outputs; returns the R-vector."""
        eng, n, R = self.eng, self.n, self.R
        eng.causal_context_async(self.oab.vv, n, R, self.ctx_ab, stream=s)
        eng.causal_context_async(self.oba.vv, n, R, self.ctx_ba, stream=s)
        eng.vv_max_async(self.ctx_ab, self.ctx_ba, R, stream=s)
        return self.ctx_ab

    def launches_per_step(self):
        return 1 if self.exchange else 2

    def bytes_per_launch(self):
        """SURVEY 8d per-merge bytes x the merges one launch performs (exchange: 2 per doc)."""
        from crdtgpu import workloads

        cA, cB = self.A.counts.cpu().numpy(), self.B.counts.cpu().numpy()
        b1 = workloads.join_bytes(cA, cB, self.oab.counts.cpu().numpy(), self.R)
        b2 = workloads.join_bytes(cB, cA, self.oba.counts.cpu().numpy(), self.R)
        return (b1 + b2) if self.exchange else (b1 + b2) // 2

    @property
    def kernel_name(self):
        return self.kernel + (" (exchange: both directions, one read)" if self.exchange else "")

    def describe(self, world):
        return {"workload": "config2: %d docs/GPU x 2 replicas x 64 entries, R=2, full-state join both directions "
                            "(%s) + causal-context allreduce(max,u64)" % (
                                self.n, "one exchange launch" if self.exchange else "two join launches"),
                "docs_per_gpu": self.n, "replicas": 2, "entries_per_replica": 64, "R": self.R,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, n_sample, budget_s):
        from oracle import oracle

        ha, hb = _host_batch(self.A, n_sample, self.R), _host_batch(self.B, n_sample, self.R)

        def run():
            rc1, _ = oracle.join(ha, hb)
            rc2, _ = oracle.join(hb, ha)
            assert rc1 == 0 and rc2 == 0

        merges, el = _time_cpu(run, 2 * n_sample, budget_s)
        return {"value": merges / el, "unit": "merges/s", "cores": 1, "kind": "port",
                "sample": "first %d docs of the config-2 batch, both directions, C oracle (oracle/awset_oracle.c, "
                          "sorted-array restatement of awset.go:107-161), 1 thread, %d merges in %.1f s "
                          "(no Go toolchain on the box: the reference itself cannot run)" % (n_sample, merges, el)}


class Config4(Config2):
    """Skewed sizes (Zipf(1.1)-like, up to 2^20 entries) with 50% concurrent
    add/remove conflicts, full-state join both directions (BASELINE configs[3])."""

    R = 2
    kernel = "join_block_kernel"
    graph_ok = False  # worklist path (several kernels): eager launches
    metric = "replica-merges/sec (AWSet join, Zipf sizes, config 4) + achieved HBM GB/s (% roofline)"

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
        self.A = OutBuffers(n, R, self.total, device=dev)
        self.B = OutBuffers(n, R, self.total, device=dev)
        eng.gen_zipf_async(seed, n, self.d_offs, self.A, self.B, stream=stream)
        self.oab = OutBuffers(n, R, 2 * self.total, device=dev)
        self.oba = OutBuffers(n, R, 2 * self.total, device=dev)
        self.ctx_ab = torch.zeros(R, dtype=torch.int64, device=dev)
        self.ctx_ba = torch.zeros(R, dtype=torch.int64, device=dev)
        self.a, self.b = self.A.as_batch(), self.B.as_batch()
        self.merges_per_step = 2 * n
        self.sizes = sizes

    def describe(self, world):
        return {"workload": "config4: %d docs/GPU, Zipf(1.1)-like sizes in [1, 2^20) (mean %.0f, max %d, %d entries "
                            "per side), 50%% concurrent add/remove conflicts, R=2, full-state join both directions"
                            % (self.n, self.sizes.mean(), self.sizes.max(), self.total),
                "docs_per_gpu": self.n, "R": self.R, "entries_per_side": self.total,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, n_sample, budget_s):
        from oracle import oracle

        n_sample = min(n_sample, 256)
        ha, hb = _host_batch(self.A, n_sample, self.R), _host_batch(self.B, n_sample, self.R)

        def run():
            rc1, _ = oracle.join(ha, hb)
            rc2, _ = oracle.join(hb, ha)
            assert rc1 == 0 and rc2 == 0

        merges, el = _time_cpu(run, 2 * n_sample, budget_s)
        return {"value": merges / el, "unit": "merges/s", "cores": 1, "kind": "port",
                "sample": "first %d docs of the config-4 batch (%d entries per side), both directions, C oracle, "
                          "1 thread, %d merges in %.1f s" % (n_sample, int(ha.offsets[-1]), merges, el)}


class Config3:
    """Delta-state anti-entropy: M ordered AWSetDelta sources folded per doc (BASELINE configs[2])."""

    R = 16
    M = 10
    kernel = "fold_sort_kernel"
    metric = "replica-merges/sec (AWSetDelta fold, config 3) + achieved HBM GB/s (% roofline)"

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

    mode = 1  # CRDT_FOLD_DELTA
    graph_ok = False  # eager launches (graph replay of the fold path not validated yet)

    def hot(self, s):
        if not hasattr(self, "_cs"):
            self._cs = (self.d.c(), self.S.c(), self.out.c())
        self.eng.fold_async(self.mode, *self._cs, stream=s)

    def post(self, s):
        self.eng.causal_context_async(self.out.vv, self.n, self.R, self.ctx, stream=s)
        return self.ctx

    def launches_per_step(self):
        return 1

    def bytes_per_launch(self):
        from crdtgpu import workloads

        n, M = self.n, self.M
        return workloads.fold_bytes(self.D.counts.cpu().numpy(), self.out.counts.cpu().numpy(), n * M * 8,
                                    n * M * 2, n * M, self.R)

    def describe(self, world):
        return {"workload": "config3: %d dst docs/GPU x 64 entries, R=16, %d ordered AWSetDelta sources per doc "
                            "(8 entries + 2 tombstones each), delta fold" % (self.n, self.M),
                "docs_per_gpu": self.n, "deltas_per_doc": self.M, "R": self.R,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, n_sample, budget_s):
        import numpy as np

        import crdtgpu
        from crdtgpu.batch import SrcBatch
        from oracle import oracle

        M, R, S = self.M, self.R, self.S
        hd = _host_batch(self.D, n_sample, R)
        k = n_sample * M
        u32, u64 = np.uint32, np.uint64
        hs = SrcBatch(R, _np_copy(S.doc_srcs, n_sample + 1, u32), _np_copy(S.src_actor, k, u32),
                      _np_copy(S.vv, k * R, u64), _np_copy(S.entry_off, k + 1, u32), _np_copy(S.keys, k * 8, u64),
                      _np_copy(S.actors, k * 8, u32), _np_copy(S.counters, k * 8, u64),
                      _np_copy(S.tomb_off, k + 1, u32), _np_copy(S.tkeys, k * 2, u64),
                      _np_copy(S.tactors, k * 2, u32), _np_copy(S.tcounters, k * 2, u64))

        def run():
            rc, _ = oracle.fold(crdtgpu.CRDT_FOLD_DELTA, hd, hs)
            assert rc == 0

        merges, el = _time_cpu(run, k, budget_s)
        return {"value": merges / el, "unit": "merges/s", "cores": 1, "kind": "port",
                "sample": "first %d docs of the config-3 batch (%d deltas), C oracle (oracle/awset_oracle.c, "
                          "restatement of awset-delta_test.go:51-166), 1 thread, %d merges in %.1f s" % (
                              n_sample, k, merges, el)}


class Config5:
    """100M docs x 8 replicas over 8 GPUs (BASELINE configs[4]): per GPU 12.5M docs,
    8 AWSet states of 16 entries (R = 8) folded r0 <- r1 <- ... <- r7 (7 merges
    per doc), then the global causal context: per-GPU VV max + RCCL all-reduce."""

    R = P = 8
    E = 16
    kernel = "fold_sort_kernel"
    metric = "replica-merges/sec (AWSet fold r0<-..<-r7, config 5) + achieved HBM GB/s (% roofline)"

    def __init__(self, eng, n, seed, dev, stream):
        import torch

        from crdtgpu.batch import OutBuffers, SrcBuffers

        self.eng, self.n, self.stream = eng, n, stream
        P, E, R = self.P, self.E, self.R
        self.D = OutBuffers(n, R, n * E, device=dev)
        self.S = SrcBuffers(R, n, n * (P - 1), n * (P - 1) * E, 0, device=dev)
        eng.gen_replicas_async(seed, n, P, E, self.D, self.S, stream=stream)
        self.out = OutBuffers(n, R, n * E * P, device=dev)
        # a doc never exceeds 16 + 7*16 = 128 slots: it stays on the LDS wave path
        eng.reserve(n, 0)
        self.ctx = torch.zeros(R, dtype=torch.int64, device=dev)
        self.d = self.D.as_batch()
        self.merges_per_step = n * (P - 1)

    mode = 0  # CRDT_FOLD_AWSET
    graph_ok = False
    hot = Config3.hot
    post = Config3.post
    launches_per_step = Config3.launches_per_step

    def bytes_per_launch(self):
        from crdtgpu import workloads

        n, P, E = self.n, self.P, self.E
        return workloads.fold_bytes(self.D.counts.cpu().numpy(), self.out.counts.cpu().numpy(), n * (P - 1) * E, 0,
                                    n * (P - 1), self.R)

    def describe(self, world):
        return {"workload": "config5: %d docs/GPU x 8 replicas x 16 entries, R=8, fold r0<-r1<-..<-r7 + global "
                            "causal-context allreduce(max,u64) over RCCL" % self.n,
                "docs_per_gpu": self.n, "replicas": self.P, "entries_per_replica": self.E, "R": self.R,
                "merges_per_step": self.merges_per_step * world, "parallelism": "doc-sharded x%d" % world}

    def cpu_baseline(self, n_sample, budget_s):
        import numpy as np

        import crdtgpu
        from crdtgpu.batch import SrcBatch
        from oracle import oracle

        P, E, R, S = self.P, self.E, self.R, self.S
        hd = _host_batch(self.D, n_sample, R)
        k = n_sample * (P - 1)
        u32, u64 = np.uint32, np.uint64
        hs = SrcBatch(R, _np_copy(S.doc_srcs, n_sample + 1, u32), _np_copy(S.src_actor, k, u32),
                      _np_copy(S.vv, k * R, u64), _np_copy(S.entry_off, k + 1, u32), _np_copy(S.keys, k * E, u64),
                      _np_copy(S.actors, k * E, u32), _np_copy(S.counters, k * E, u64))

        def run():
            rc, _ = oracle.fold(crdtgpu.CRDT_FOLD_AWSET, hd, hs)
            assert rc == 0

        merges, el = _time_cpu(run, k, budget_s)
        return {"value": merges / el, "unit": "merges/s", "cores": 1, "kind": "port",
                "sample": "first %d docs of the config-5 batch (%d merges per pass), C oracle (oracle/awset_oracle.c, "
                          "restatement of awset.go:107-161), 1 thread, %d merges in %.1f s" % (n_sample, k, merges, el)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--docs", type=int, default=None,
                    help="documents per GPU (default 1,048,576; config 5: 12,500,000 = 100M / 8)")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-sample", type=int, default=65536)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--separate", action="store_true", help="configs 2/4: two join launches instead of one exchange")
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a captured HIP graph")
    ap.add_argument("--force-graph", action="store_true", help="replay a captured HIP graph for every config")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    args = ap.parse_args()

    import numpy as np
    import torch

    import crdtgpu
    from crdtgpu.dist import u64_max_allreduce

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream()

    n = args.docs or {5: 12_500_000, 4: 16_384}.get(args.config, 1 << 20)
    eng = crdtgpu.Engine(local)
    # each rank owns its own documents (weak scaling; no data-path exchange)
    seed = args.seed + (rank << 40)
    cls = {2: Config2, 3: Config3, 4: Config4, 5: Config5}[args.config]
    if args.separate:
        cls.exchange = False
    W = cls(eng, n, seed, dev, stream)
    eng.sync(stream)

    # The dominant launch is captured once into a HIP graph and replayed each
    # step: one host call per step instead of the ctypes/ABI calls of every
    # kernel, so a loaded host cannot stretch the step.
    graph = None
    if not args.no_graph and (W.graph_ok or args.force_graph):
        W.hot(stream)  # warm the workspaces before capture (no allocation inside)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            W.hot(torch.cuda.current_stream())
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
        local_ctx = W.post(stream)
        if dist is not None:
            return u64_max_allreduce(dist, local_ctx)
        return local_ctx

    for _ in range(args.warmup):
        step()
    eng.sync(stream)
    bytes_launch = W.bytes_per_launch()  # algorithmic bytes from the actual output sizes

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = None
    for k in range(args.steps):
        g = step(events[k])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.sync(stream)
    replay_check = None
    if graph is not None and hasattr(W, "out"):
        # graph-replayed output vs an eager launch of the same call (bitwise)
        snap = [t.clone() for t in (W.out.counts, W.out.keys, W.out.actors, W.out.counters, W.out.vv)]
        W.hot(stream)
        eng.sync(stream)
        replay_check = all(bool(torch.equal(a, b)) for a, b in
                           zip(snap, (W.out.counts, W.out.keys, W.out.actors, W.out.counters, W.out.vv)))
        del snap
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # mean duration of one launch of the dominant kernel, HIP events on its stream
    t_launch = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps / 1e3 / W.launches_per_step()
    achieved = bytes_launch / t_launch / 1e9
    global_ctx = g.cpu().numpy().view(np.uint64).tolist() if g is not None else []

    # HBM bytes per launch of this kernel from the PMC passes (tools/pmc.sh ->
    # tools/traffic.py --emit), matched on config, docs and kernel instance
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            for e in json.load(open(args.traffic_json)):
                if (e.get("docs") == n and e.get("config") == args.config and e.get("kernel", "").startswith(W.kernel)
                        and bool(e.get("exchange")) == bool(getattr(W, "exchange", False))):
                    traffic = e.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    merges = W.merges_per_step * world * args.steps
    result = {
        "metric": W.metric,
        "value": merges / elapsed,
        "unit": "merges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (AWSet states generated on device, csrc/gen.hip)",
        "launch": "hip graph replay" if graph is not None else "eager",
        "config": W.describe(world),
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": getattr(W, "kernel_name", W.kernel),
            "algorithmic_bytes_per_launch": bytes_launch, "launch_ms": t_launch * 1e3,
        },
        "global_causal_context": global_ctx,
        "replay_check": replay_check,
    }
    if traffic:
        result["roofline"]["traffic_gbs"] = traffic / t_launch / 1e9
        result["roofline"]["traffic_frac"] = traffic / t_launch / 1e9 / HBM_PEAK_GBS
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = W.cpu_baseline(min(args.cpu_sample, n), args.cpu_budget)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
