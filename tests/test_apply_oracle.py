"""CPU: the C oracle's batched local ops (oracle_awset_apply) against the
map-based line-by-line restatement of the reference's state producers
(AWSet.Add awset.go:89-94, AWSet.Del :96-101, AWSetDelta.Del
awset-delta_test.go:14-33), including the index-out-of-range panic of a clock
bump with actor >= len(vv) and the malformed-op-list errors."""

import random

import pytest

import crdtgpu
from apply_cases import doc_of, make_case
from crdtgpu.batch import AWSetBatch, OpBatch, TombBatch
from oracle import oracle


@pytest.mark.parametrize("R,state,ops", [(2, 0, 8), (3, 20, 40), (8, 64, 256), (16, 5, 200)])
def test_oracle_apply_matches_reference_replay(R, state, ops):
    rng = random.Random(R * 7 + ops)
    st, tb, op, want = make_case(rng, 300, R, lambda: rng.randint(0, state), lambda: rng.randint(0, ops))
    rc, out, tout = oracle.apply(st, op, tb)
    assert rc == 0
    for d, w in enumerate(want):
        assert doc_of(out, tout, d, R) == (w[0], w[1], w[2]), d


def test_oracle_apply_panics_like_the_reference():
    rng = random.Random(5)
    R = 3
    for _ in range(40):
        st, tb, op, want = make_case(rng, 1, R, lambda: rng.randint(0, 6), lambda: rng.randint(1, 12), panic_rate=1.0)
        rc, _, _ = oracle.apply(st, op, tb)
        assert (rc == crdtgpu.CRDT_E_ACTOR_RANGE) == (want[0] is None)


def test_oracle_apply_rejects_malformed_lists():
    st = AWSetBatch.from_docs(2, [([(1, 0, 1)], [1, 0])])
    bad = OpBatch.from_lists([[(crdtgpu.CRDT_OP_DELTA_DEL_KEY, 1)]], [0])  # key without its call
    assert oracle.apply(st, bad)[0] == crdtgpu.CRDT_E_INVALID
    ok = OpBatch.from_lists([[(crdtgpu.CRDT_OP_DELTA_DEL, 0), (crdtgpu.CRDT_OP_DELTA_DEL_KEY, 1)]], [0])
    assert oracle.apply(st, ok, with_tombs=False)[0] == crdtgpu.CRDT_E_INVALID  # nowhere to put Deleted
    rc, out, tout = oracle.apply(st, ok)
    assert rc == 0 and int(out.counts[0]) == 0 and tout.doc(0) == [(1, 0, 2)] and out.vv.tolist() == [2, 0]
    long = OpBatch.from_lists([[(crdtgpu.CRDT_OP_ADD, k) for k in range(257)]], [0])
    assert oracle.apply(st, long)[0] == crdtgpu.CRDT_E_INVALID
    odd = OpBatch.from_lists([[(7, 1)]], [0])
    assert oracle.apply(st, odd)[0] == crdtgpu.CRDT_E_INVALID


def test_oracle_apply_del_call_without_present_keys_still_bumps():
    # awset-delta_test.go:15: the clock moves even when no key is recorded
    st = AWSetBatch.from_docs(2, [([], [0, 4])])
    op = OpBatch.from_lists([[(crdtgpu.CRDT_OP_DELTA_DEL, 0), (crdtgpu.CRDT_OP_DELTA_DEL_KEY, 9)]], [1])
    rc, out, tout = oracle.apply(st, op, TombBatch.from_lists([[]]))
    assert rc == 0 and out.vv.tolist() == [0, 5] and tout.doc(0) == []
