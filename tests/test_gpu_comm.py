"""GPU: the global causal context through the C ABI's RCCL entry points
(crdt_global_context_allreduce, crdt_comm_init + crdt_context_allreduce_async),
SURVEY.md §8b/§8e.  On the one-GPU box the communicator has one rank, so the
all-reduce(max, u64) is the identity on the per-GPU summary: what is checked
is the binding (RCCL found at run time, ncclUint64 + ncclMax, in-place on the
device buffer, ordering after the summary kernel on another stream) and the
unsigned transport of values >= 2^63, against the host restatement
oracle.causal_context (max over every merged VersionVector, crdt-misc.go:43-55)."""

import numpy as np
import pytest

import crdtgpu
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


def _vvs(R, n=5000, seed=3):
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 2**64 - 1, size=(n, R), dtype=np.uint64)
    v[17, 0] = np.uint64(2**64 - 1)
    v[123, R - 1] = np.uint64(2**63)
    return v


@pytest.mark.parametrize("R", [2, 8, 64])
def test_global_context_allreduce_single_process(torch, R):
    dev = torch.device("cuda:0")
    vv = _vvs(R)
    want = oracle.causal_context(vv.reshape(-1), vv.shape[0], R).tolist()
    eng = crdtgpu.Engine(0)
    try:
        d_vv = torch.from_numpy(vv.reshape(-1).view(np.int64).copy()).to(dev)
        summ = torch.zeros(R, dtype=torch.int64, device=dev)
        side = torch.cuda.Stream()
        eng.causal_context_async(d_vv, vv.shape[0], R, summ, stream=side)  # summary on another stream
        got = crdtgpu.global_context_allreduce([eng], [summ], R)
        assert got == want
        assert summ.cpu().numpy().view(np.uint64).tolist() == want
        # second call reuses the communicator
        assert crdtgpu.global_context_allreduce([eng], [summ], R) == want
    finally:
        eng.close()


def test_context_allreduce_one_rank_per_process(torch):
    R = 16
    dev = torch.device("cuda:0")
    vv = _vvs(R, seed=4)
    want = oracle.causal_context(vv.reshape(-1), vv.shape[0], R).tolist()
    eng = crdtgpu.Engine(0)
    try:
        uid = crdtgpu.comm_unique_id()
        assert len(uid) == 128
        eng.comm_init(1, 0, uid)
        d_vv = torch.from_numpy(vv.reshape(-1).view(np.int64).copy()).to(dev)
        summ = torch.zeros(R, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream()
        eng.causal_context_async(d_vv, vv.shape[0], R, summ, stream=s)
        eng.context_allreduce_async(summ, R, stream=s)
        eng.sync(s)
        assert summ.cpu().numpy().view(np.uint64).tolist() == want
    finally:
        eng.close()


def test_allreduce_rejects_bad_arguments(torch):
    eng = crdtgpu.Engine(0)
    try:
        summ = torch.zeros(4, dtype=torch.int64, device="cuda:0")
        with pytest.raises(crdtgpu.CrdtError):
            crdtgpu.global_context_allreduce([eng, eng], [summ, summ], 4)  # one context per GPU
        with pytest.raises(crdtgpu.CrdtError):
            eng.context_allreduce_async(summ, 4)  # no crdt_comm_init yet
    finally:
        eng.close()


def _comm_worker(rank, world, port, q):
    """One rank of test_engine_comm_two_ranks: its own GPU, the engine's own
    communicator (id made by rank 0, shared over gloo), one all-reduce."""
    try:
        import os

        import torch
        import torch.distributed as dist

        import crdtgpu
        from crdtgpu import dist as cdist

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", rank)
        torch.cuda.set_device(dev)
        eng = crdtgpu.Engine(rank)
        cdist.engine_comm_handshake(dist, world, rank, eng.comm_init)
        R = 16
        vv = _vvs(R, n=3000, seed=10 + rank)
        local = oracle.causal_context(vv.reshape(-1), vv.shape[0], R).tolist()
        d_vv = torch.from_numpy(vv.reshape(-1).view(np.int64).copy()).to(dev)
        summ = torch.zeros(R, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream()
        eng.causal_context_async(d_vv, vv.shape[0], R, summ, stream=s)
        eng.context_allreduce_async(summ, R, stream=s)
        eng.sync(s)
        got = summ.cpu().numpy().view(np.uint64).tolist()
        eng.close()
        dist.destroy_process_group()
        q.put((rank, local, got, None))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, None, None, "%s: %s" % (type(e).__name__, e)))


def test_engine_comm_two_ranks(torch):
    """bench.py --engine-comm at N = 2: crdt_comm_unique_id + crdt_comm_init +
    crdt_context_allreduce_async across two processes, one GPU each, against
    the elementwise u64 max of both ranks' oracle summaries (crdt-misc.go:43-55).
    The pool's boxes have one GPU, so this runs only where two are visible."""
    import socket

    import torch.multiprocessing as mp

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL cannot hold two ranks of one communicator on one GPU)")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    assert not [r[3] for r in res if r[3]], res
    want = [max(res[0][1][i], res[1][1][i]) for i in range(16)]
    assert res[0][1] != res[1][1]
    for _, _, got, _ in res:
        assert got == want
