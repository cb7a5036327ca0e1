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
