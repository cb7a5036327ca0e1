#!/usr/bin/env python3
"""Benchmark: batched AWSet full-state join on MI355X (BASELINE config 2).

Workload (per GPU, weak scaling): 1,048,576 independent documents x 2 replicas,
64 entries per replica state, R = 2 (synthetic reachable states generated on
the device: csrc/gen.hip).  One step = one pass of the hot path over the batch:
  A <- B and B <- A for every document (2 merges per doc, crdt_awset_join_async),
  then the per-GPU causal-context summary (elementwise max of the output VVs),
  all-reduced (max, u64) across GPUs over RCCL when N > 1.
Inputs are resident in HBM before the timed region.  Metric: replica merges/s
(whole job), with the join kernel's achieved algorithmic HBM bandwidth against
the 8 TB/s roofline.

  python bench.py [--gpus N] [--steps K] [--warmup W]
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


def cpu_baseline(A, B, n_sample, budget_s):
    """Time the C oracle (single thread, the 'port' baseline) on the first
    n_sample docs of this rank's batch, both directions, repeated for ~budget_s."""
    import numpy as np

    from crdtgpu.batch import AWSetBatch
    from oracle import oracle

    def host(o):
        off = o.offsets[: n_sample + 1].cpu().numpy().view(np.uint32).copy()
        cnt = o.counts[:n_sample].cpu().numpy().view(np.uint32).copy()
        end = int(off[-1])
        return AWSetBatch(2, off, o.keys[:end].cpu().numpy().view(np.uint64).copy(),
                          o.actors[:end].cpu().numpy().view(np.uint32).copy(),
                          o.counters[:end].cpu().numpy().view(np.uint64).copy(),
                          o.vv[: 2 * n_sample].cpu().numpy().view(np.uint64).copy(), counts=cnt)

    ha, hb = host(A), host(B)
    merges, t0 = 0, time.perf_counter()
    while True:
        rc1, _ = oracle.join(ha, hb)
        rc2, _ = oracle.join(hb, ha)
        assert rc1 == 0 and rc2 == 0
        merges += 2 * n_sample
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": merges / el, "unit": "merges/s", "cores": 1, "kind": "port",
            "sample": "first %d docs of the config-2 batch, both directions, C oracle (oracle/awset_oracle.c, "
                      "sorted-array restatement of awset.go:107-161), 1 thread, %d merges in %.1f s "
                      "(no Go toolchain on the box: the reference itself cannot run)" % (n_sample, merges, el)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--docs", type=int, default=1 << 20, help="documents per GPU")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-sample", type=int, default=65536)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    args = ap.parse_args()

    import numpy as np
    import torch

    import crdtgpu
    from crdtgpu.batch import OutBuffers
    from crdtgpu import workloads
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

    n = args.docs
    R = 2
    eng = crdtgpu.Engine(local)
    eng.reserve(n, 0)
    eng.set_max_doc_entries(64)  # the pair workload holds exactly 64 entries per replica
    # each rank owns its own documents (weak scaling; no data-path exchange)
    seed = args.seed + (rank << 40)
    A = OutBuffers(n, R, n * 64, device=dev)
    B = OutBuffers(n, R, n * 64, device=dev)
    eng.gen_pair_async(seed, n, A, B, stream=stream)
    oab = OutBuffers(n, R, 2 * n * 64, device=dev)
    oba = OutBuffers(n, R, 2 * n * 64, device=dev)
    ctx_ab = torch.zeros(R, dtype=torch.int64, device=dev)
    ctx_ba = torch.zeros(R, dtype=torch.int64, device=dev)
    a, b = A.as_batch(), B.as_batch()
    eng.sync(stream)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        eng.join_async(a, b, oab, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        eng.join_async(b, a, oba, stream=stream)
        if ev is not None:
            ev[2].record(stream)
        eng.causal_context_async(oab.vv, n, R, ctx_ab, stream=stream)
        eng.causal_context_async(oba.vv, n, R, ctx_ba, stream=stream)
        eng.vv_max_async(ctx_ab, ctx_ba, R, stream=stream)
        if dist is not None:
            return u64_max_allreduce(dist, ctx_ab)
        return ctx_ab

    for _ in range(args.warmup):
        step()
    eng.sync(stream)

    # algorithmic bytes per join launch, from the actual output sizes
    n_out_ab = int(oab.counts.to(torch.int64).sum().item())
    n_out_ba = int(oba.counts.to(torch.int64).sum().item())
    n_in = int(A.counts.to(torch.int64).sum().item()), int(B.counts.to(torch.int64).sum().item())
    bytes_ab = 20 * (n_in[0] + n_in[1] + n_out_ab) + (24 * R + 12) * n
    bytes_ba = 20 * (n_in[0] + n_in[1] + n_out_ba) + (24 * R + 12) * n
    assert bytes_ab == workloads.join_bytes(A.counts.cpu().numpy(), B.counts.cpu().numpy(),
                                            oab.counts.cpu().numpy(), R)

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        g = step(events[k])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.sync(stream)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    t_ab = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps / 1e3  # s per launch
    t_ba = sum(e[1].elapsed_time(e[2]) for e in events) / args.steps / 1e3
    t_launch = (t_ab + t_ba) / 2
    achieved = (bytes_ab + bytes_ba) / 2 / t_launch / 1e9
    global_ctx = g.cpu().numpy().view(np.uint64).tolist()

    merges = 2 * n * world * args.steps
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("docs") == n and tj.get("kernel", "").startswith("join_wave_kernel"):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    result = {
        "metric": "replica-merges/sec (AWSet full-state join) + achieved HBM GB/s (% roofline)",
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
        "data": "synthetic (reachable AWSet states generated on device, csrc/gen.hip)",
        "config": {
            "workload": "config2: %d docs/GPU x 2 replicas x 64 entries, R=2, full-state join both directions "
                        "+ causal-context allreduce(max,u64)" % n,
            "docs_per_gpu": n, "replicas": 2, "entries_per_replica": 64, "R": R,
            "merges_per_step": 2 * n * world, "parallelism": "doc-sharded x%d" % world,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": "join_wave_kernel<4>",
            "algorithmic_bytes_per_launch": (bytes_ab + bytes_ba) // 2,
            "launch_ms": t_launch * 1e3,
        },
        "global_causal_context": global_ctx,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(A, B, min(args.cpu_sample, n), args.cpu_budget)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
