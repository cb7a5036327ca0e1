"""CPU, world_size 2 over gloo: the multi-GPU path's only collective (global
causal-context all-reduce, u64 max) and the document sharding, exercised with
real torch.distributed processes."""

import os
import socket

import numpy as np
import pytest

from crdtgpu import dist as cdist
from oracle import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, vvs, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # this rank's documents, and its local summary (host oracle stands in for
    # the device kernel: on CPU only the collective is under test)
    lo, hi = cdist.shard(len(vvs), world, rank)
    R = vvs.shape[1]
    local = oracle.causal_context(vvs[lo:hi].reshape(-1), hi - lo, R)
    t = torch.from_numpy(local.view(np.int64).copy())
    g = cdist.u64_max_allreduce(dist, t)
    q.put((rank, lo, hi, g.numpy().view(np.uint64).tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_context_allreduce_gloo(world):
    import torch.multiprocessing as mp

    rng = np.random.default_rng(world)
    R = 8
    vvs = rng.integers(0, 2**64 - 1, size=(1001, R), dtype=np.uint64)
    vvs[17, 3] = np.uint64(2**64 - 1)  # values above 2^63 must survive the signed transport
    vvs[500, 0] = np.uint64(2**63)
    want = oracle.causal_context(vvs.reshape(-1), vvs.shape[0], R).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, vvs, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    assert [r[1] for r in res] == [cdist.shard(1001, world, r)[0] for r in range(world)]
    assert res[-1][2] == 1001
    for _, _, _, g in res:
        assert g == want


def _handshake_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = []
    uid = cdist.engine_comm_handshake(dist, world, rank, lambda w, r, u: seen.append((w, r, u)))
    q.put((rank, uid, seen))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_engine_comm_id_handshake_gloo(world):
    """bench.py's multi-rank setup of the engine's own RCCL communicator,
    rehearsed over gloo: rank 0's crdt_comm_unique_id (RCCL loads on a host
    without a GPU) reaches every rank unchanged, and every rank calls
    crdt_comm_init's stand-in exactly once with (world, its rank, that id)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_handshake_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    uid = res[0][1]
    assert len(uid) == 128 and any(uid)
    for rank, u, seen in res:
        assert u == uid and seen == [(world, rank, uid)]


def test_shard_covers_all_docs():
    for n, w in [(0, 2), (1, 2), (10, 3), (100_000_000, 8), (7, 8)]:
        spans = [cdist.shard(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
        assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
