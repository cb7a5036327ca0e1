"""CPU: the per-key restatement of the ordered fold that fold_pipe_kernel
(go-crdt-playground_amd/csrc/fold.hip) implements, checked against the C oracle
(step-by-step replay of awset.go:103-161 / awset-delta_test.go:51-166) on
randomized adversarial documents -- tombstones (effective and re-added),
no-op delta steps, first contact (Counter(src.Actor) == 0), keys known only to
sources, actor == len(VV) panics and actor > len(VV).

The model follows the kernel's phases literally (schedule, keep/tag, sort by
(key, tag), then the element-parallel resolve of fold.hip sort_resolve: a
segmented scan for the current dot, the gap removals, a segmented scan for the
presence), and keeps the sequential event walk per key beside it as a second
restatement, so a pass here says the formulation is the reference's
semantics, including which HasDot calls can panic; the GPU tests then check
the kernel against the same oracle."""

import itertools
import random

import pytest

from crdtgpu import CRDT_FOLD_AWSET, CRDT_FOLD_DELTA
from crdtgpu.batch import AWSetBatch, SrcBatch
from oracle import oracle


def resolve_scan(tup, chain, full, Vs, R, delta):
    """fold.hip sort_resolve over the sorted kept tuples: returns (err, out)."""
    M = len(chain)
    n = len(tup)
    err = False
    step = [-1 if z[1] == 0 else (z[1] >> 1) - 1 for z in tup]
    tomb = [z[1] & 1 == 1 for z in tup]
    ent = [not x for x in tomb]
    head = [i == 0 or tup[i][0] != tup[i - 1][0] for i in range(n)]
    tail = [i == n - 1 or tup[i + 1][0] != tup[i][0] for i in range(n)]

    def scan_last(marked, val):
        """inclusive / exclusive 'last marked value' (None = no mark)."""
        inc, exc, cur = [], [], None
        for i in range(n):
            exc.append(cur)
            if marked[i]:
                cur = val[i]
            inc.append(cur)
        return inc, exc

    # the clock before the tuple's step has the tuple's dot (source tuples)
    hv = [step[i] >= 0 and tup[i][2] < R and Vs[step[i]][tup[i][2]] >= tup[i][3] for i in range(n)]
    f = []  # 1 present, 2 absent, 0 unchanged
    for i in range(n):
        if step[i] < 0:
            f.append(1)
        elif tomb[i]:
            f.append(0 if hv[i] else 2)
        elif full[step[i]]:
            f.append(0 if hv[i] else 1)
        else:
            f.append(1)
    dinc, _ = scan_last([head[i] or ent[i] for i in range(n)], [i if ent[i] else None for i in range(n)])
    da = [tup[dinc[i]][2] if dinc[i] is not None else 0 for i in range(n)]
    dc = [tup[dinc[i]][3] if dinc[i] is not None else 0 for i in range(n)]
    gaps, G = [], []
    for i in range(n):
        jn = M if tail[i] else step[i + 1]
        g = [j for j in range(step[i] + 1, jn) if full[j]]
        gaps.append(g)
        G.append(da[i] < R and any(chain[j][1][da[i]] >= dc[i] for j in g))
    h = [2 if G[i] else f[i] for i in range(n)]
    pinc, pexc = scan_last([head[i] or h[i] != 0 for i in range(n)], [h[i] == 1 for i in range(n)])
    out = []
    for i in range(n):
        before = not head[i] and bool(pexc[i])
        after = f[i] == 1 or (f[i] == 0 and before)
        a = tup[i][2]
        if step[i] >= 0 and full[step[i]] and ent[i] and not before and a == R:
            err = True
        if delta and tomb[i] and before and a == R:
            err = True
        if after and da[i] == R and gaps[i]:
            err = True
        if tail[i] and pinc[i]:
            out.append((tup[i][0], da[i], dc[i]))
    return err, out


def model_fold(mode, ents, vv0, chain):
    """Per-key replay of one document; returns (err, entries, vv)."""
    R = len(vv0)
    delta = mode == CRDT_FOLD_DELTA
    err = False

    def has_dot(vv, a, c):
        nonlocal err
        if a >= R:
            err |= a == R  # crdt-misc.go:28-34: vv[a] with a == len panics
            return False
        return vv[a] >= c

    # 1. schedule (fold.hip "schedule"): effective tombstones, V_j, full_j, noop_j
    eff = {}
    for j, (_, _, e, t) in enumerate(chain):
        emap = {k: (a, c) for k, a, c in e}
        for x, (k, a, c) in enumerate(t or []):
            s = emap.get(k)
            eff[(j, x)] = not (s is not None and (s[0] != a or s[1] > c))
    V = list(vv0)
    Vs, full, noop, chg = [], [], [], {}
    for j, (aj, svv, e, t) in enumerate(chain):
        Vs.append(list(V))
        f = True
        if delta:
            if aj == R:
                err = True
            f = (V[aj] if aj < R else 0) == 0
        nop = False
        if not f:
            any_chg = False
            for i, (k, a, c) in enumerate(e):
                chg[(j, i)] = not has_dot(V, a, c)
                any_chg |= chg[(j, i)]
            nop = not any_chg and not any(eff[(j, x)] for x in range(len(t or [])))
        full.append(f)
        noop.append(nop)
        if not nop:
            V = [max(x, y) for x, y in zip(V, svv)]
    # 2. keep + tag: (key, tag, actor, counter); tag orders doc < entries < tombstones per step
    tup = [(k, 0, a, c) for k, a, c in ents]
    for j, (aj, svv, e, t) in enumerate(chain):
        if noop[j]:
            continue
        for i, (k, a, c) in enumerate(e):
            if full[j] or chg[(j, i)]:
                tup.append((k, (j + 1) * 2, a, c))
        if delta and not full[j]:
            for x, (k, a, c) in enumerate(t or []):
                if eff[(j, x)]:
                    tup.append((k, (j + 1) * 2 + 1, a, c))
    # 3. group by key in replay order
    tup.sort(key=lambda z: (z[0], z[1]))
    err_scan, out_scan = resolve_scan(tup, chain, full, Vs, R, delta)
    err_scan |= err  # panics of the schedule are the kernel's classify phase
    segs = {}
    for z in tup:
        segs.setdefault(z[0], []).append(z)
    # 4. event walk per key
    out = []
    for key in sorted(segs):
        ev = segs[key]
        p, pres, a, c = 0, False, 0, 0
        if ev[0][1] == 0:
            pres, a, c = True, ev[0][2], ev[0][3]
            p = 1
        jn = 0
        while True:
            ts = (ev[p][1] >> 1) - 1 if p < len(ev) else 64
            nf = next((j for j in range(jn, len(chain)) if full[j]), 64) if pres else 64
            je = min(ts, nf)
            if je >= 64:
                break
            is_e = is_t = False
            if ts == je and not ev[p][1] & 1:
                is_e, ea, ec = True, ev[p][2], ev[p][3]
                p += 1
            if delta and p < len(ev) and (ev[p][1] >> 1) - 1 == je:
                is_t, xa, xc = True, ev[p][2], ev[p][3]
                p += 1
            if full[je]:
                if is_e:
                    if pres or not has_dot(Vs[je], ea, ec):
                        pres, a, c = True, ea, ec
                elif pres and has_dot(chain[je][1], a, c):
                    pres = False
            else:
                if is_e:
                    pres, a, c = True, ea, ec
                if is_t and pres and not has_dot(Vs[je], xa, xc):
                    pres = False
            jn = je + 1
        if pres:
            out.append((key, a, c))
    assert err_scan == err
    if not err:
        assert out_scan == out
    return err, out, V


def rand_doc(rng, R, mode):
    U = rng.choice([6, 12, 40])

    def dots(p, amax):
        return sorted((k, rng.randrange(amax), rng.randint(1, 6)) for k in range(U) if rng.random() < p)

    amax = R + 2 if rng.random() < 0.15 else R  # sometimes actor == R (panic) or > R (never seen)
    vv0 = [rng.randint(0, 6) for _ in range(R)]
    if rng.random() < 0.3:
        vv0[rng.randrange(R)] = 0
    ents = dots(rng.uniform(0.0, 0.8), amax)
    chain = []
    for _ in range(rng.randint(0, 6)):
        aj = rng.randrange(amax)
        svv = [rng.randint(0, 8) for _ in range(R)]
        e = dots(rng.uniform(0.0, 0.6), amax)
        t = dots(rng.uniform(0.0, 0.4), amax) if mode == CRDT_FOLD_DELTA else []
        chain.append((aj, svv, e, t))
    return ents, vv0, chain


@pytest.mark.parametrize("mode", [CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
@pytest.mark.parametrize("seed", range(6))
def test_per_key_model_matches_oracle(mode, seed):
    rng = random.Random(1000 * seed + mode)
    checked = errs = 0
    for _ in range(150):
        R = rng.choice([1, 2, 3, 5])
        ents, vv0, chain = rand_doc(rng, R, mode)
        dst = AWSetBatch.from_docs(R, [(ents, vv0)])
        srcs = SrcBatch.from_lists(R, [[(a, v, e, t) for a, v, e, t in chain]])
        rc, want = oracle.fold(mode, dst, srcs)
        err, got, vv = model_fold(mode, ents, vv0, chain)
        assert err == (rc != 0), (ents, vv0, chain)
        if rc:
            errs += 1
            continue
        c = int(want.counts[0])
        o = int(want.offsets[0])
        exp = list(zip(want.keys[o:o + c].tolist(), want.actors[o:o + c].tolist(), want.counters[o:o + c].tolist()))
        assert got == exp, (ents, vv0, chain)
        assert vv == want.vv[:R].tolist()
        checked += 1
    assert checked > 50 and errs > 0


def kernel_steps(n, ent_sizes, tomb_sizes):
    """The fold kernel's step-of-tuple (csrc/fold.hip, fold_pipe_kernel): lane s
    marks s + 1 where source s's entries / tombstones end (only the last source
    ending at a position writes), then a max-scan of (region << 8 | mark) over
    the tuple positions, 64 per chunk with the previous chunk's last lane
    carried (the DPP row_shr / row_bcast scan is a plain prefix max here)."""
    ms = len(ent_sizes)
    E, X = sum(ent_sizes), sum(tomb_sizes)
    N = n + E + X
    mark = [0] * 256
    soff = list(itertools.accumulate(ent_sizes))  # lane s: end of source s's entries
    toff = list(itertools.accumulate(tomb_sizes))
    for s in range(ms):
        last = s + 1 == ms
        if soff[s] < E and (last or soff[s + 1] != soff[s]):
            mark[n + soff[s]] = s + 1
        if toff[s] < X and (last or toff[s + 1] != toff[s]):
            mark[n + E + toff[s]] = s + 1
    steps, carry = [], 0
    for c in range((N + 63) // 64):
        run = carry
        for lane in range(64):
            i = c * 64 + lane
            region = 2 if n + E <= i < N else (1 if n <= i < n + E else 0)
            run = max(run, (region << 8) | mark[i])
            if i < N:
                steps.append(run & 0xFF)
        carry = run
    return steps


@pytest.mark.parametrize("seed", range(6))
def test_step_of_tuple_marks(seed):
    """Every source tuple gets the index of the source holding it, empty sources
    (shared end positions) included; document entries get 0."""
    rng = random.Random(seed)
    for _ in range(300):
        ms = rng.randint(1, 64)
        n = rng.randint(0, 64)
        ent = [rng.choice([0, 0, 1, 2, 3, 8]) for _ in range(ms)]
        tomb = [rng.choice([0, 0, 0, 1, 2]) for _ in range(ms)]
        if n + sum(ent) + sum(tomb) > 256:
            continue
        want = [0] * n
        for s, k in enumerate(ent):
            want += [s] * k
        for s, k in enumerate(tomb):
            want += [s] * k
        assert kernel_steps(n, ent, tomb) == want


def slot_chain_fold(ents, vv0, chain):
    """fold.hip dense_awset_walk's lane-parallel rule for the AWSet fold
    (every step a full merge): per tuple t at row r (0 = the document, j + 1 =
    source j), add_t = document tuple or !HasDot(V_{r-1}, dot_t); drop_t =
    HasDot(svv_j, dot_t) for a step j in [r, the key's next row - 1).  The key
    survives iff some tuple has add and none from the last such row on has
    drop; the dot is the last tuple's.  Documents with actor == R take the
    step walk in the kernel (exact panics), so they are not modelled here."""
    R = len(vv0)
    V = list(vv0)
    Vs = []
    for _, svv, _, _ in chain:
        Vs.append(list(V))
        V = [max(x, y) for x, y in zip(V, svv)]
    rows = {}
    for k, a, c in ents:
        rows.setdefault(k, []).append((0, a, c))
    for j, (_, _, e, _) in enumerate(chain):
        for k, a, c in e:
            rows.setdefault(k, []).append((j + 1, a, c))
    ms = len(chain)
    out = []
    for k in sorted(rows):
        tl = rows[k]
        addw = dropw = 0
        for x, (r, a, c) in enumerate(tl):
            nr = tl[x + 1][0] if x + 1 < len(tl) else ms + 1
            cov = a < R
            add = r == 0 or not (cov and Vs[r - 1][a] >= c)
            drop = cov and any(chain[j][1][a] >= c for j in range(r, nr - 1))
            addw |= add << r
            dropw |= drop << r
        if addw and (dropw >> (addw.bit_length() - 1)) == 0:
            out.append((k, tl[-1][1], tl[-1][2]))
    return out, V


@pytest.mark.parametrize("seed", range(6))
def test_slot_chain_rule_matches_oracle(seed):
    rng = random.Random(7000 + seed)
    checked = 0
    for _ in range(300):
        R = rng.choice([1, 2, 3, 5])
        ents, vv0, chain = rand_doc(rng, R, CRDT_FOLD_AWSET)
        chain = chain[:15]
        acts = [a for _, a, _ in ents] + [a for _, _, e, _ in chain for _, a, _ in e]
        if R in acts:
            continue  # the kernel's step walk (exact panics)
        dst = AWSetBatch.from_docs(R, [(ents, vv0)])
        srcs = SrcBatch.from_lists(R, [[(a, v, e, t) for a, v, e, t in chain]])
        rc, want = oracle.fold(CRDT_FOLD_AWSET, dst, srcs)
        assert rc == 0
        got, vv = slot_chain_fold(ents, vv0, chain)
        c, o = int(want.counts[0]), int(want.offsets[0])
        exp = list(zip(want.keys[o:o + c].tolist(), want.actors[o:o + c].tolist(), want.counters[o:o + c].tolist()))
        assert got == exp, (ents, vv0, chain)
        assert vv == want.vv[:R].tolist()
        checked += 1
    assert checked > 150
