"""GPU parity of the batched local ops (crdt_awset_apply_*, csrc/apply.hip)
against the C oracle (oracle_awset_apply, itself pinned to the map-based
restatement of AWSet.Add / AWSet.Del / AWSetDelta.Del by
tests/test_apply_oracle.py): random op scripts on random states, hot keys with
many ops, states far larger than the op list, the 256-op limit, panics and
malformed lists, device-resident inputs through the async ABI, and a
1,048,576-document batch checked exactly."""

import random

import numpy as np
import pytest

import crdtgpu
from apply_cases import doc_of, make_case
from crdtgpu.batch import AWSetBatch, OpBatch, OutBuffers, TombBatch, TombBuffers
from oracle import oracle
from test_gpu_parity import host_out

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


@pytest.fixture(scope="module")
def eng(torch):
    e = crdtgpu.Engine(0)
    yield e
    e.close()


def check_same(eng, st, op, tb, R, n_docs):
    rc, wo, wt = oracle.apply(st, op, tb)
    assert rc == 0
    go, gt = eng.apply(st, op, tb)
    assert (go.offsets == wo.offsets).all() and (gt.offsets == wt.offsets).all()
    for d in range(n_docs):
        assert doc_of(go, gt, d, R) == doc_of(wo, wt, d, R), d


@pytest.mark.parametrize("R,state,ops", [(2, 0, 8), (3, 20, 40), (8, 64, 64), (8, 64, 65), (16, 100, 256),
                                         (64, 30, 256)])
def test_apply_random(eng, R, state, ops):
    rng = random.Random(R * 100 + ops)
    st, tb, op, _ = make_case(rng, 1500, R, lambda: rng.randint(0, state), lambda: rng.randint(0, ops))
    check_same(eng, st, op, tb, R, 1500)


def test_apply_hot_keys_and_big_states(eng):
    """Few keys hit by many ops (long runs, DELTA_DEL_KEY effective only after
    an ADD in the run), and states of thousands of entries streamed past a
    handful of ops; tombstone lists of hundreds."""
    rng = random.Random(3)
    R = 4
    st, tb, op, _ = make_case(rng, 200, R, lambda: rng.choice([0, 5, 3000, 9000]), lambda: rng.randint(100, 256),
                              universe=12, tomb_size=lambda: rng.choice([0, 2, 400]))
    check_same(eng, st, op, tb, R, 200)
    st, tb, op, _ = make_case(rng, 200, R, lambda: rng.choice([2000, 5000]), lambda: rng.randint(0, 6),
                              universe=20000, tomb_size=lambda: rng.choice([0, 300]))
    check_same(eng, st, op, tb, R, 200)


def test_apply_errors(eng):
    R = 2
    st = AWSetBatch.from_docs(R, [([(1, 0, 1)], [1, 0]), ([], [0, 0])])
    add = crdtgpu.CRDT_OP_ADD
    with pytest.raises(crdtgpu.CrdtError) as ei:  # Add with actor == len(vv): Go index panic
        eng.apply(st, OpBatch.from_lists([[(add, 5)], []], [R, 0]))
    assert ei.value.code == crdtgpu.CRDT_E_ACTOR_RANGE
    with pytest.raises(crdtgpu.CrdtError) as ei:  # more than CRDT_MAX_OPS_PER_DOC ops
        eng.apply(st, OpBatch.from_lists([[(add, k) for k in range(257)], []], [0, 1]))
    assert ei.value.code == crdtgpu.CRDT_E_INVALID
    ddk = [(crdtgpu.CRDT_OP_DELTA_DEL, 0), (crdtgpu.CRDT_OP_DELTA_DEL_KEY, 1)]
    with pytest.raises(crdtgpu.CrdtError) as ei:  # AWSetDelta.Del with nowhere to record Deleted
        eng.apply(st, OpBatch.from_lists([ddk, []], [0, 1]), with_tombs=False)
    assert ei.value.code == crdtgpu.CRDT_E_INVALID
    # a Del-only doc with an out-of-range actor is fine (no clock bump), and the
    # engine is usable after errors
    op = OpBatch.from_lists([[(crdtgpu.CRDT_OP_DEL, 1)], ddk[:1]], [R + 3, 1])
    check_same(eng, st, op, None, R, 2)
    # malformed tombstone batches are refused on the host before any launch
    # (the kernel sizes its staging by the counts and binary-searches the keys)
    u32, u64 = np.uint32, np.uint64
    ops = OpBatch.from_lists([[(add, 3)], [(add, 4)]], [0, 1])
    over = TombBatch(np.array([0, 1, 2], u32), np.array([2, 7], u64), np.zeros(2, u32), np.ones(2, u64),
                     counts=np.array([2, 1], u32))
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.apply(st, ops, over)
    assert ei.value.code == crdtgpu.CRDT_E_CAPACITY
    unsorted = TombBatch(np.array([0, 2, 2], u32), np.array([7, 2], u64), np.zeros(2, u32), np.ones(2, u64))
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.apply(st, ops, unsorted)
    assert ei.value.code == crdtgpu.CRDT_E_UNSORTED
    check_same(eng, st, ops, None, R, 2)  # still usable


def test_apply_device_async(eng, torch):
    rng = random.Random(4)
    R = 8
    n = 3000
    st, tb, op, _ = make_case(rng, n, R, lambda: rng.randint(0, 80), lambda: rng.randint(0, 40))
    rc, wo, wt = oracle.apply(st, op, tb)
    assert rc == 0
    dev = torch.device("cuda:0")
    nops = int(op.op_off[-1])
    out = OutBuffers(n, R, int(st.offsets[-1]) + nops, device=dev)
    tout = TombBuffers(n, int(tb.offsets[-1]) + nops, device=dev)
    eng.apply_async(st.to(dev), op.to(dev), out, tb.to(dev), tout)
    eng.sync()
    ho = host_out(out, torch)
    ht = TombBatch(*(t.cpu().numpy().view(np.uint32 if t.dtype == torch.int32 else np.uint64)
                     for t in (tout.offsets, tout.keys, tout.actors, tout.counters)),
                   counts=tout.counts.cpu().numpy().view(np.uint32))
    for d in range(n):
        assert doc_of(ho, ht, d, R) == doc_of(wo, wt, d, R), d


def test_apply_million_docs(eng, torch):
    """1,048,576 docs x (64-entry state, 16 ops): every doc exact (vectorised)."""
    rng = np.random.default_rng(6)
    n, R, E, M = 1 << 20, 4, 64, 16
    keys = np.sort(rng.integers(0, 1 << 20, size=(n, E), dtype=np.uint64), axis=1)
    keys = keys + np.arange(E, dtype=np.uint64)[None, :]  # strictly ascending per doc
    st = AWSetBatch(R, (np.arange(n + 1, dtype=np.uint64) * E).astype(np.uint32), keys.reshape(-1),
                    rng.integers(0, R, n * E).astype(np.uint32), rng.integers(1, 50, n * E).astype(np.uint64),
                    rng.integers(0, 50, n * R).astype(np.uint64))
    kinds = rng.choice(np.array([0, 0, 1, 2, 3], dtype=np.uint8), size=(n, M))
    kinds[:, 0] = np.where(kinds[:, 0] == 3, 2, kinds[:, 0])
    # a DELTA_DEL_KEY must follow a DELTA_DEL or another key of the call
    for j in range(1, M):
        bad = (kinds[:, j] == 3) & ~np.isin(kinds[:, j - 1], [2, 3])
        kinds[bad, j] = 2
    opkeys = np.where(rng.random((n, M)) < 0.5, keys[np.arange(n)[:, None], rng.integers(0, E, (n, M))],
                      rng.integers(0, 1 << 21, (n, M), dtype=np.uint64))
    op = OpBatch((np.arange(n + 1, dtype=np.uint64) * M).astype(np.uint32), kinds.reshape(-1), opkeys.reshape(-1),
                 rng.integers(0, R, n).astype(np.uint32))
    rc, wo, wt = oracle.apply(st, op, None)
    assert rc == 0
    go, gt = eng.apply(st, op, None)
    for a, b in ((go, wo), (gt, wt)):
        assert (np.asarray(a.offsets) == np.asarray(b.offsets)).all()
        assert (np.asarray(a.counts) == np.asarray(b.counts)).all()
        cnt = np.asarray(b.counts).astype(np.int64)
        starts = np.asarray(b.offsets[:-1]).astype(np.int64)
        idx = np.repeat(starts, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
        for f in ("keys", "actors", "counters"):
            assert (np.asarray(getattr(a, f))[idx] == np.asarray(getattr(b, f))[idx]).all(), f
    assert (go.vv == wo.vv).all()
