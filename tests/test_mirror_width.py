"""CPU: the host mirrors size each output VersionVector by replaying the fold
on the VVs alone (crdtgpu/awset.py _fold_width, host/crdt.hpp
detail::fold_width).  A no-op delta step (awset-delta_test.go:60) skips
VersionVector.Merge, so a longer source VV must not lengthen the destination
there.  Checked against the map-based restatement of the reference
(oracle/awset_ref.py) on random states whose VVs have unequal lengths."""

import random

from crdtgpu import abi
from crdtgpu.awset import AWSetDelta, Dot, _fold_width
from helpers import ref, ref_state


def _rand(rng, n_vv, universe, tombs):
    vv = [rng.randint(0, 5) for _ in range(n_vv)]
    ents = sorted((k, rng.randrange(n_vv), rng.randint(1, 6)) for k in rng.sample(range(universe),
                                                                                  rng.randint(0, universe // 2)))
    dele = sorted((k, rng.randrange(n_vv), rng.randint(1, 6)) for k in rng.sample(range(universe),
                                                                                  rng.randint(0, 3))) if tombs else []
    return ents, vv, dele


def _mirror(actor, ents, vv, dele):
    return AWSetDelta(actor, vv, {"%012d" % k: Dot(a, c) for k, a, c in ents},
                      {"%012d" % k: Dot(a, c) for k, a, c in dele} or None)


def test_delta_fold_width_matches_reference():
    rng = random.Random(71)
    checked = shorter = 0
    for _ in range(3000):
        ents, vv, _ = _rand(rng, rng.randint(1, 4), 10, False)
        chain = []
        for _ in range(rng.randint(1, 4)):
            e, svv, dele = _rand(rng, rng.randint(1, 4), 10, True)
            chain.append((rng.randrange(4), e, svv, dele))
        x = ref_state(ents, vv, cls=ref.AWSetDelta)
        try:
            for act, e, svv, dele in chain:
                x.Merge(ref_state(e, svv, actor=act, cls=ref.AWSetDelta, deleted=dele))
        except ref.GoPanic:
            continue
        want = len(x.VersionVector)
        got = _fold_width(abi.CRDT_FOLD_DELTA, _mirror(0, ents, vv, []),
                          [_mirror(act, e, svv, dele) for act, e, svv, dele in chain])
        assert got == want, (ents, vv, chain)
        checked += 1
        shorter += want < max([len(vv)] + [len(c[2]) for c in chain])
    assert checked > 1000 and shorter > 5  # the no-op rule really kept some VVs short


def test_join_panic_check_matches_reference_for_unequal_lengths():
    """Zero-padded VVs hide Go's panic at HasDot(actor == len(vv)) of the shorter
    vector from the kernels (they flag actor == R); the mirrors find it on the
    host (awset.py _join_panics, crdt.hpp detail::join_panics).  Exactly where
    the map-based restatement raises GoPanic."""
    from crdtgpu.awset import AWSet, _join_panics

    rng = random.Random(72)
    panics = 0
    for _ in range(4000):
        ea, va, _ = _rand(rng, rng.randint(1, 4), 8, False)
        eb, vb, _ = _rand(rng, rng.randint(1, 4), 8, False)
        # actors up to 4 so that actor == len(shorter vv) happens often
        ea = [(k, rng.randrange(5), c) for k, _, c in ea]
        eb = [(k, rng.randrange(5), c) for k, _, c in eb]
        x, y = ref_state(ea, va), ref_state(eb, vb)
        try:
            x.Merge(y)
            want = False
        except ref.GoPanic:
            want = True
        a = AWSet(0, va, {"%012d" % k: Dot(p, c) for k, p, c in ea})
        b = AWSet(1, vb, {"%012d" % k: Dot(p, c) for k, p, c in eb})
        assert _join_panics(a, b) == want
        panics += want
    assert panics > 200


def _ragged_chain(rng, delta, n_src):
    """dst + ordered sources with VVs of 1..4 words and actors up to 4, so that
    actor == len(vv) of a shorter vector is frequent."""
    def st(tombs):
        e, vv, dele = _rand(rng, rng.randint(1, 4), 8, tombs)
        e = [(k, rng.randrange(5), c) for k, _, c in e]
        dele = [(k, rng.randrange(5), c) for k, _, c in dele]
        return e, vv, dele
    dst = st(False)
    return dst, [(rng.randrange(5),) + st(delta) for _ in range(n_src)]


def test_fold_replay_checks_match_reference_panics():
    """_replay_checks (the mirrors' host check for folds over VVs of unequal
    lengths) says "panic" exactly where the map restatement of the reference
    raises GoPanic: Counter(src.Actor) awset-delta_test.go:53, the HasDot of
    MakeDeltaMergeData :85, phase 1 awset.go:133 / :137, phase 2 awset.go:152 /
    tombstones :153 -- for AWSet folds and AWSetDelta folds."""
    from crdtgpu.awset import _replay_checks

    rng = random.Random(73)
    seen = {True: 0, False: 0}
    for delta in (False, True):
        mode = abi.CRDT_FOLD_DELTA if delta else abi.CRDT_FOLD_AWSET
        cls = ref.AWSetDelta if delta else ref.AWSet
        for _ in range(3000):
            (e0, v0, _), chain = _ragged_chain(rng, delta, rng.randint(1, 4))
            x = ref_state(e0, v0, cls=cls)
            try:
                for act, e, svv, dele in chain:
                    x.Merge(ref_state(e, svv, actor=act, cls=cls, deleted=dele if delta else None))
                want = False
            except ref.GoPanic:
                want = True
            got = _replay_checks(mode, _mirror(0, e0, v0, []),
                                 [_mirror(act, e, svv, dele if delta else []) for act, e, svv, dele in chain], 5)
            assert (got == "panic") == want, (delta, e0, v0, chain)
            seen[want] += 1
    assert seen[True] > 500 and seen[False] > 500


def test_ragged_width_avoids_actor_collisions():
    """The padded width R skips values some actor of a short document takes
    (the kernels flag actor == R where Go, on the shorter vector, says false)."""
    from crdtgpu.awset import AWSet, _ragged_checks

    a = AWSet(0, [1, 1], {"x": Dot(2, 1)})     # shorter than the longest vector: a "short" document
    b = AWSet(1, [1, 1, 1], {"x": Dot(3, 1)})  # actor 3 == the longest length: R = 3 collides, R = 4 does not
    assert _ragged_checks(abi.CRDT_FOLD_AWSET, [[a, b]], "t") == 4
    c = AWSet(0, [1, 1, 1], {"y": Dot(3, 1)})
    d = AWSet(1, [1, 1, 1], {"y": Dot(0, 1)})
    assert _ragged_checks(abi.CRDT_FOLD_AWSET, [[c, d]], "t") == 3  # equal lengths: the kernels are exact at R

    # a counter-0 src dot past the end of the shorter dst vector: Go's HasDot says
    # false (add), the zero pad would say true (skip) -> refused, CRDT_E_INVALID
    import pytest

    e = AWSet(0, [1], {})
    f = AWSet(1, [1, 1, 1], {"q": Dot(2, 0)})
    with pytest.raises(abi.CrdtError) as ei:
        _ragged_checks(abi.CRDT_FOLD_AWSET, [[e, f]], "t")
    assert ei.value.code == abi.CRDT_E_INVALID
