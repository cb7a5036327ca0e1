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
