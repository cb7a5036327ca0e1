"""CPU: the hash-map restatement (oracle/awset_map.cpp, map[string]Dot as in
awset.go:55-59) agrees with the sorted-array C oracle (oracle/awset_oracle.c)
on arbitrary states: full-state joins, ordered AWSet folds and AWSetDelta
folds, including which documents panic (actor == len(VV)).  It is the CPU
baseline bench.py reports, so it must compute the same merges it is timed on;
its bench entry points are exercised on a small batch with 2 threads."""

import random

import pytest

from crdtgpu import CRDT_FOLD_AWSET, CRDT_FOLD_DELTA
from helpers import batch_of, outs_equal, random_state, src_batch_of
from oracle import oracle


def _join_docs(rng, n, R, actor_hi=None):
    a = [random_state(rng, R, rng.randint(0, 40), 64, 12, actor_hi) for _ in range(n)]
    b = [random_state(rng, R, rng.randint(0, 40), 64, 12, actor_hi) for _ in range(n)]
    return a, b


def _fold_docs(rng, n, R, delta, actor_hi=None):
    dsts, per = [], []
    for _ in range(n):
        dsts.append(random_state(rng, R, rng.randint(0, 20), 32, 6, actor_hi))
        chain = []
        for _ in range(rng.randint(0, 5)):
            e, vv = random_state(rng, R, rng.randint(0, 10), 32, 6, actor_hi)
            t = random_state(rng, R, rng.randint(0, 4), 32, 6, actor_hi)[0] if delta else []
            chain.append((rng.randrange(R), vv, e, t))
        per.append(chain)
    return dsts, per


def test_map_join_matches_c_oracle():
    rng = random.Random(11)
    R = 4
    a, b = _join_docs(rng, 400, R)
    A, B = batch_of(R, a), batch_of(R, b)
    rc1, want = oracle.join(A, B)
    rc2, got = oracle.map_join(A, B)
    assert rc1 == rc2 == 0
    assert outs_equal(got, want, A.n_docs, R) is None


@pytest.mark.parametrize("mode", [CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
def test_map_fold_matches_c_oracle(mode):
    rng = random.Random(12 + mode)
    R = 3
    dsts, per = _fold_docs(rng, 400, R, mode == CRDT_FOLD_DELTA)
    D, S = batch_of(R, dsts), src_batch_of(R, per)
    rc1, want = oracle.fold(mode, D, S)
    rc2, got = oracle.map_fold(mode, D, S)
    assert rc1 == rc2 == 0
    assert outs_equal(got, want, D.n_docs, R) is None


@pytest.mark.parametrize("mode", [None, CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
def test_map_panics_where_c_oracle_panics(mode):
    """One document per call, actors up to R + 1: both restatements agree on the verdict."""
    rng = random.Random(13 + (mode if mode is not None else 7))
    R = 2
    verdicts = set()
    for _ in range(150):
        if mode is None:
            a, b = _join_docs(rng, 1, R, actor_hi=R + 1 if rng.random() < 0.3 else None)
            A, B = batch_of(R, a), batch_of(R, b)
            rc1, w = oracle.join(A, B)
            rc2, g = oracle.map_join(A, B)
        else:
            dsts, per = _fold_docs(rng, 1, R, mode == CRDT_FOLD_DELTA,
                                   actor_hi=R + 1 if rng.random() < 0.3 else None)
            D, S = batch_of(R, dsts), src_batch_of(R, per)
            rc1, w = oracle.fold(mode, D, S)
            rc2, g = oracle.map_fold(mode, D, S)
        assert rc1 == rc2
        if rc1 == 0:
            assert outs_equal(g, w, 1, R) is None
        verdicts.add(rc1)
    assert len(verdicts) == 2  # both outcomes were exercised


def test_map_bench_entry_points():
    rng = random.Random(14)
    R = 2
    a, b = _join_docs(rng, 64, R)
    m, t = oracle.map_bench_join(batch_of(R, a), batch_of(R, b), True, 2, 0.05)
    assert m >= 128 and m % 128 == 0 and t > 0
    dsts, per = _fold_docs(rng, 64, R, True)
    S = src_batch_of(R, per)
    m, t = oracle.map_bench_fold(CRDT_FOLD_DELTA, batch_of(R, dsts), S, 2, 0.05)
    ns = sum(len(c) for c in per)
    assert m >= ns and m % max(ns, 1) == 0 and t > 0
    assert oracle.cpu_threads() >= 1
