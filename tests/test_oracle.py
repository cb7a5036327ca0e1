"""CPU: pin the oracles.

1. The map-based restatement (oracle/awset_ref.py) replays the reference tests
   (golden fixture regenerated and compared byte for byte).
2. The C SoA oracle (oracle/awset_oracle.c) reproduces every golden merge
   (entries, dots, version vectors).
3. The C oracle agrees with the map-based restatement on random reachable
   histories and on arbitrary states, for full-state merges, ordered folds and
   AWSetDelta folds, including the actor == len(vv) panic.
"""

import json
import random
import subprocess
import sys

import numpy as np
import pytest

from helpers import GOLDEN, KEYS, ROOT, batch_of, ents, out_doc, pad, random_history, random_state, ref, \
    ref_entries, ref_state, snap_entries, src_batch_of
from oracle import oracle

from crdtgpu import CRDT_E_ACTOR_RANGE, CRDT_FOLD_AWSET, CRDT_FOLD_DELTA

KID = {k: i for i, k in enumerate(KEYS)}


def load_golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_golden_fixture_is_current(tmp_path):
    """Regenerating the fixture from the restatement reproduces the committed file."""
    before = open(GOLDEN).read()
    subprocess.check_call([sys.executable, "tests/golden/make_golden.py"], cwd=ROOT, stdout=subprocess.DEVNULL)
    assert open(GOLDEN).read() == before


def test_version_vector_kat6():
    g = load_golden()["version_vector"]
    a, b = ref.VersionVector(g["a"]), ref.VersionVector(g["b"])
    a.Merge(b)
    assert list(a) == g["a_merge_b"]
    b.Merge(a)
    assert list(b) == g["b_merge_a"]
    out = oracle.causal_context(np.array(g["a"] + g["b"], dtype=np.uint64), 2, 4)
    assert out.tolist() == g["a_merge_b"]


def golden_merge_cases():
    for sc in load_golden()["scenarios"]:
        for i, m in enumerate(sc["merges"]):
            yield pytest.param(sc["kind"], m, id="%s#%d" % (sc["name"].split()[0], i))


@pytest.mark.parametrize("kind,m", list(golden_merge_cases()))
def test_c_oracle_golden_merge(kind, m):
    keys = sorted({e[0] for s in (m["dst"], m["src"], m["out"]) for e in s["entries"] + s.get("deleted", [])})
    ids = {k: i for i, k in enumerate(keys)}
    R = len(m["dst"]["vv"])
    dst = batch_of(R, [(snap_entries(m["dst"], ids), m["dst"]["vv"])])
    if kind == "awset":
        src = batch_of(R, [(snap_entries(m["src"], ids), m["src"]["vv"])])
        rc, out = oracle.join(dst, src)
    else:
        s = m["src"]
        dele = sorted((ids[k], a, c) for k, a, c in s["deleted"])
        srcs = src_batch_of(R, [[(s["actor"], s["vv"], snap_entries(s, ids), dele)]])
        rc, out = oracle.fold(CRDT_FOLD_DELTA, dst, srcs)
    assert rc == 0
    e, vv = out_doc(out, 0, R)
    assert e == snap_entries(m["out"], ids)
    assert vv == m["out"]["vv"]


def hist_doc(s, R):
    return [(KID[k], d.actor, d.counter) for k, d in sorted(s.Entries.items())], pad(s.VersionVector, R)


def hist_src(s, R):
    dele = [(KID[k], d.actor, d.counter) for k, d in sorted((getattr(s, 'Deleted', None) or {}).items())]
    e, vv = hist_doc(s, R)
    return (s.Actor, vv, e, dele)


def hist_entries(s):
    return [(KID[k], d.actor, d.counter) for k, d in sorted(s.Entries.items())]


@pytest.mark.parametrize("R", [2, 3, 5])
def test_c_oracle_vs_ref_reachable_join(R):
    rng = random.Random(100 + R)
    dsts, srcs, want = [], [], []
    for _ in range(60):
        reps = random_history(rng, R, rng.randint(5, 60), rng.choice([4, 10, 40]), delta=False)
        a, b = rng.sample(range(R), 2)
        dsts.append(hist_doc(reps[a], R))
        srcs.append(hist_doc(reps[b], R))
        x = reps[a].Clone()
        x.Merge(reps[b])
        want.append((hist_entries(x), list(x.VersionVector)))
    rc, out = oracle.join(batch_of(R, dsts), batch_of(R, srcs))
    assert rc == 0
    for d, w in enumerate(want):
        assert out_doc(out, d, R) == w


@pytest.mark.parametrize("delta", [False, True])
def test_c_oracle_vs_ref_reachable_fold(delta):
    rng = random.Random(7 if delta else 8)
    R = 4
    mode = CRDT_FOLD_DELTA if delta else CRDT_FOLD_AWSET
    dsts, per_doc, want = [], [], []
    for _ in range(50):
        pool = []
        reps = random_history(rng, R, 10, 12, delta)
        for _ in range(6):  # snapshot states as the histories advance
            for r in reps:
                pool.append(r.Clone())
            for _ in range(rng.randint(1, 8)):
                r = rng.randrange(R)
                if rng.random() < 0.5:
                    reps[r].Add(rng.choice(KEYS[:12]))
                elif rng.random() < 0.5:
                    reps[r].Del(rng.choice(KEYS[:12]))
                else:
                    reps[r].Merge(reps[rng.randrange(R)])
        dst = rng.choice(pool).Clone()
        chain = [rng.choice(pool) for _ in range(rng.randint(0, 6))]
        dsts.append(hist_doc(dst, R))
        per_doc.append([hist_src(s, R) for s in chain])
        for s in chain:
            dst.Merge(s)
        want.append((hist_entries(dst), list(dst.VersionVector)))
    rc, out = oracle.fold(mode, batch_of(R, dsts), src_batch_of(R, per_doc))
    assert rc == 0
    for d, w in enumerate(want):
        assert out_doc(out, d, R) == w, d


def test_c_oracle_vs_ref_arbitrary_join():
    rng = random.Random(5)
    R = 4
    dsts, srcs, want = [], [], []
    for _ in range(300):
        a = random_state(rng, R, rng.randint(0, 40), 64, 12)
        b = random_state(rng, R, rng.randint(0, 40), 64, 12)
        dsts.append(a)
        srcs.append(b)
        x = ref_state(*a)
        x.Merge(ref_state(*b))
        want.append((ref_entries(x), list(x.VersionVector)))
    rc, out = oracle.join(batch_of(R, dsts), batch_of(R, srcs))
    assert rc == 0
    for d, w in enumerate(want):
        assert out_doc(out, d, R) == w


def test_c_oracle_vs_ref_arbitrary_delta_fold():
    rng = random.Random(6)
    R = 3
    dsts, per_doc, want = [], [], []
    for _ in range(200):
        a = random_state(rng, R, rng.randint(0, 20), 32, 6)
        chain = []
        for _ in range(rng.randint(1, 4)):
            e, vv = random_state(rng, R, rng.randint(0, 10), 32, 6)
            t, _ = random_state(rng, R, rng.randint(0, 6), 32, 6)
            chain.append((rng.randrange(R), vv, e, t))
        dsts.append(a)
        per_doc.append(chain)
        x = ref_state(*a, cls=ref.AWSetDelta)
        for act, vv, e, t in chain:
            x.Merge(ref_state(e, vv, actor=act, cls=ref.AWSetDelta, deleted=t))
        want.append((ref_entries(x), list(x.VersionVector)))
    rc, out = oracle.fold(CRDT_FOLD_DELTA, batch_of(R, dsts), src_batch_of(R, per_doc))
    assert rc == 0
    for d, w in enumerate(want):
        assert out_doc(out, d, R) == w, d


def test_c_oracle_actor_range_panics():
    # dst-only entry with actor == R: phase 2 calls srcVV.HasDot -> Go panics
    R = 2
    dst = batch_of(R, [([(1, 2, 1)], [1, 1])])
    src = batch_of(R, [([], [1, 1])])
    with pytest.raises(ref.GoPanic):
        x = ref_state([(1, 2, 1)], [1, 1])
        x.Merge(ref_state([], [1, 1]))
    rc, _ = oracle.join(dst, src)
    assert rc == CRDT_E_ACTOR_RANGE
    # actor > R is "never seen" -> no panic, kept
    rc, out = oracle.join(batch_of(R, [([(1, 3, 1)], [1, 1])]), src)
    assert rc == 0 and out_doc(out, 0, R)[0] == [(1, 3, 1)]
    # common key with actor == R: HasDot is never called -> no panic
    rc, out = oracle.join(batch_of(R, [([(1, 2, 1)], [1, 1])]), batch_of(R, [([(1, 2, 1)], [1, 1])]))
    assert rc == 0
    # delta path select: Counter(src.Actor == R) panics
    srcs = src_batch_of(R, [[(2, [1, 1], [], [])]])
    rc, _ = oracle.fold(CRDT_FOLD_DELTA, batch_of(R, [([], [1, 1])]), srcs)
    assert rc == CRDT_E_ACTOR_RANGE


def test_c_oracle_empty_docs():
    R = 2
    dst = batch_of(R, [([], [0, 0]), ([(5, 0, 1)], [1, 0]), ([], [3, 3])])
    src = batch_of(R, [([], [0, 0]), ([], [0, 0]), ([(9, 1, 2)], [0, 2])])
    rc, out = oracle.join(dst, src)
    assert rc == 0
    assert out_doc(out, 0, R) == ([], [0, 0])
    assert out_doc(out, 1, R) == ([(5, 0, 1)], [1, 0])
    assert out_doc(out, 2, R) == ([], [3, 3])  # (B 2) covered by dst VV [3,3]: skip
