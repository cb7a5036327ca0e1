"""Host mirror of the reference's Go API, merging on the GPU.

Same types and method names as package crdt:
  Dot, VersionVector           crdt-misc.go:9-74
  AWSet                        awset.go:55-171
  AWSetDelta                   awset-delta_test.go:9-77
plus the batch entry points a caller with many documents uses:
  MergeBatch(dsts, srcs)                 one (*AWSet).Merge per pair
  FoldBatch(dsts, srcs_per_dst)          ordered (*AWSet).Merge sequences
  DeltaMergeBatch(dsts, srcs_per_dst)    ordered (*AWSetDelta).Merge sequences

``Merge`` / ``*Batch`` intern the string keys of the batch into u64 ids
(order-preserving, an exact bijection), pack structure-of-arrays buffers, run
the join/fold kernels through ``crdt_awset_join_batch`` /
``crdt_awset_fold_batch`` and unpack the result into the Go-shaped maps.  The
local ops (Add, Del, Clone, ...) are per-replica host state changes, as in the
reference; they are not part of the batched hot path.

Version vectors of unequal lengths:
  * a batch's version vectors are zero-padded to one width R (<= 64).  When
    every vector of a document has length R, the kernels flag HasDot/Counter
    at actor == R exactly where Go panics (crdt-misc.go:29,37).
  * a document with a shorter vector is replayed on the host before the
    launch (_replay_checks): every HasDot and Counter call of the reference,
    in order, on the unpadded vectors -- Counter(src.Actor)
    (awset-delta_test.go:53), MakeDeltaMergeData's HasDot (:85), phase 1
    (awset.go:133, awset-delta_test.go:137), phase 2 (awset.go:152,
    awset-delta_test.go:153).  A panic there raises CrdtError
    (CRDT_E_ACTOR_RANGE), nothing applied; the merged entries still come from
    the GPU.  R is chosen so that no actor of such a document equals R (the
    kernels' flag would otherwise fire where Go returns false).
  * the one input the padded layout cannot express: a dot with counter 0 at
    an actor between len(vv) and R, where Go's HasDot says false and the pad
    says true.  Counter-0 dots are unreachable (Add bumps first, awset.go:92),
    so such a batch is refused with CRDT_E_INVALID.
"""

from __future__ import annotations

from typing import Dict, List, NamedTuple, Optional, Sequence

from . import abi
from .batch import AWSetBatch, SrcBatch
from .engine import Engine


class Dot(NamedTuple):
    """crdt-misc.go:12-15."""

    Actor: int
    Counter: int

    def String(self) -> str:  # crdt-misc.go:17-19
        return "(%s %d)" % (chr(ord("A") + self.Actor), self.Counter)

    __str__ = String


class VersionVector(list):
    """crdt-misc.go:23; single-vector host helpers (the batched max runs in the kernels)."""

    def HasDot(self, d: Dot) -> bool:  # crdt-misc.go:28-34
        if len(self) < d.Actor:
            return False
        if d.Actor == len(self):
            raise abi.CrdtError(abi.CRDT_E_ACTOR_RANGE, "HasDot")
        return self[d.Actor] >= d.Counter

    def Counter(self, a: int) -> int:  # crdt-misc.go:36-41
        if len(self) < a:
            return 0
        if a == len(self):
            raise abi.CrdtError(abi.CRDT_E_ACTOR_RANGE, "Counter")
        return self[a]

    def Merge(self, src: Sequence[int]) -> None:  # crdt-misc.go:43-55
        for i, n in enumerate(src):
            if i < len(self):
                if self[i] < n:
                    self[i] = n
            else:
                self.append(n)

    def Clone(self) -> "VersionVector":  # crdt-misc.go:70-74
        return VersionVector(self)

    def String(self) -> str:  # crdt-misc.go:57-68
        return "[" + ", ".join("(%s %d)" % (chr(ord("A") + i), n) for i, n in enumerate(self)) + "]"

    __str__ = String


_engine: Optional[Engine] = None


def default_engine() -> Engine:
    global _engine
    if _engine is None:
        _engine = Engine(0)
    return _engine


class AWSet:
    """awset.go:55-59."""

    def __init__(self, Actor: int = 0, VersionVector_: Optional[Sequence[int]] = None,
                 Entries: Optional[Dict[str, Dot]] = None):
        self.Actor = Actor
        self.VersionVector = VersionVector(VersionVector_ or [])
        self.Entries: Dict[str, Dot] = dict(Entries or {})

    def SortedValues(self) -> List[str]:  # awset.go:61-70
        return sorted(self.Entries)

    def Reset(self) -> None:  # awset.go:72-75
        self.VersionVector = VersionVector([0])
        self.Entries = {}

    def Clone(self) -> "AWSet":  # awset.go:77-85
        return AWSet(self.Actor, list(self.VersionVector), self.Entries)

    def Has(self, k: str) -> bool:  # awset.go:87
        return k in self.Entries

    def Add(self, *keys: str) -> None:  # awset.go:89-94
        for k in keys:
            if self.Actor >= len(self.VersionVector):
                raise abi.CrdtError(abi.CRDT_E_ACTOR_RANGE, "Add")
            self.VersionVector[self.Actor] += 1
            self.Entries[k] = Dot(self.Actor, self.VersionVector[self.Actor])

    def Del(self, *keys: str) -> None:  # awset.go:96-101 (no clock bump)
        for k in keys:
            self.Entries.pop(k, None)

    def Merge(self, src: "AWSet") -> None:  # awset.go:103-105, on the GPU
        MergeBatch([self], [src])

    def String(self) -> str:  # awset.go:163-171
        s = self.VersionVector.String()
        for v in self.SortedValues():
            s += '\n  %s  "%s"' % (self.Entries[v], v)
        return s

    __str__ = String


class AWSetDelta(AWSet):
    """awset-delta_test.go:9-12."""

    def __init__(self, Actor: int = 0, VersionVector_: Optional[Sequence[int]] = None,
                 Entries: Optional[Dict[str, Dot]] = None, Deleted: Optional[Dict[str, Dot]] = None):
        super().__init__(Actor, VersionVector_, Entries)
        self.Deleted: Optional[Dict[str, Dot]] = dict(Deleted) if Deleted else None

    def Del(self, *keys: str) -> None:  # awset-delta_test.go:14-33
        if self.Actor >= len(self.VersionVector):
            raise abi.CrdtError(abi.CRDT_E_ACTOR_RANGE, "Del")
        self.VersionVector[self.Actor] += 1
        dot2 = Dot(self.Actor, self.VersionVector[self.Actor])
        for k in keys:
            if k in self.Entries:
                if self.Deleted is None:
                    self.Deleted = {}
                self.Deleted[k] = dot2
                del self.Entries[k]

    def Clone(self) -> "AWSetDelta":  # awset-delta_test.go:35-49
        return AWSetDelta(self.Actor, list(self.VersionVector), self.Entries, self.Deleted)

    def Merge(self, src: "AWSetDelta") -> None:  # awset-delta_test.go:51-65, on the GPU
        DeltaMergeBatch([self], [[src]])

    def gcDeleted(self, srcVersionVector) -> None:  # awset-delta_test.go:67-77: empty in the reference
        pass


# ---------------------------------------------------------------------------
# packing


def _intern(states) -> Dict[str, int]:
    keys = set()
    for s in states:
        keys.update(s.Entries)
        if isinstance(s, AWSetDelta) and s.Deleted:
            keys.update(s.Deleted)
    return {k: i for i, k in enumerate(sorted(keys))}


def _entries(m: Optional[Dict[str, Dot]], ids) -> list:
    return sorted((ids[k], d.Actor, d.Counter) for k, d in (m or {}).items())


def _pad(vv, R):
    return list(vv) + [0] * (R - len(vv))


def _width(states) -> int:
    R = max([len(s.VersionVector) for s in states] + [1])
    if R > abi.CRDT_MAX_R:
        raise abi.CrdtError(abi.CRDT_E_INVALID, "version vector longer than %d" % abi.CRDT_MAX_R)
    return R


def _unpack(dsts, out, names, R, widths):
    for d, dst in enumerate(dsts):
        o, n = int(out.offsets[d]), int(out.counts[d])
        keys = out.keys[o:o + n].tolist()
        acts = out.actors[o:o + n].tolist()
        cnts = out.counters[o:o + n].tolist()
        dst.Entries = {names[k]: Dot(a, c) for k, a, c in zip(keys, acts, cnts)}
        dst.VersionVector = VersionVector(out.vv[d * R:d * R + widths[d]].tolist())


class _GoPanic(Exception):
    pass


class _Check:
    """HasDot / Counter as Go evaluates them on the unpadded vectors
    (crdt-misc.go:28-41), noting where the zero-padded width R answers
    differently (a counter-0 dot at len(vv) < actor < R)."""

    def __init__(self, R):
        self.R, self.pad_differs = R, False

    def has(self, vv, d: Dot) -> bool:
        n = len(vv)
        if n < d.Actor:
            if d.Actor < self.R and d.Counter == 0:
                self.pad_differs = True
            return False
        if d.Actor == n:
            raise _GoPanic
        return vv[d.Actor] >= d.Counter

    @staticmethod
    def counter(vv, a: int) -> int:
        n = len(vv)
        if n < a:
            return 0
        if a == n:
            raise _GoPanic
        return vv[a]


def _replay_checks(mode, dst, srcs, R) -> Optional[str]:
    """Replay dst.Merge(src) for src in srcs, in order, on maps with the
    reference's rules -- (*AWSet).merge awset.go:107-161, (*AWSetDelta).Merge
    awset-delta_test.go:51-65, MakeDeltaMergeData :79-105, deltaMerge :107-166
    -- only to find whether Go panics ("panic") or the padded layout would
    differ ("pad"); None otherwise.  Whether Go panics does not depend on its
    random map order: every call site runs unless an earlier one panicked."""
    ck = _Check(R)
    V = list(dst.VersionVector)
    E = dict(dst.Entries)
    try:
        for s in srcs:
            full = mode != abi.CRDT_FOLD_DELTA or ck.counter(V, s.Actor) <= 0
            if full:
                changed, dele = s.Entries, {}
            else:
                changed = {k: d for k, d in s.Entries.items() if not ck.has(V, d)}
                dele = {}
                for k, x in (getattr(s, "Deleted", None) or {}).items():
                    m = s.Entries.get(k)
                    if m is None or not (m.Actor != x.Actor or m.Counter > x.Counter):
                        dele[k] = x
                if not changed and not dele:
                    continue  # awset-delta_test.go:60: no deltaMerge, no VersionVector.Merge
            for k, sd in changed.items():
                if k in E or not ck.has(V, sd):
                    E[k] = sd
            if full:
                for k in [k for k in E if k not in s.Entries]:
                    if ck.has(s.VersionVector, E[k]):
                        del E[k]
            else:
                for k, x in dele.items():
                    if k in E and not ck.has(V, x):
                        del E[k]
            sv = list(s.VersionVector)
            V = [max(x, y) for x, y in zip(V, sv)] + V[len(sv):] + sv[len(V):]
    except _GoPanic:
        return "panic"
    return "pad" if ck.pad_differs else None


def _doc_actors(mode, states):
    a = set()
    for i, s in enumerate(states):
        a.update(d.Actor for d in s.Entries.values())
        a.update(d.Actor for d in (getattr(s, "Deleted", None) or {}).values())
        if i and mode == abi.CRDT_FOLD_DELTA:
            a.add(s.Actor)
    return a


def _ragged_checks(mode, docs, what) -> int:
    """The padded width R of a batch (docs[i] = [dst, src...]) and the host
    checks of its documents with a vector shorter than R (module docstring)."""
    R = _width([s for doc in docs for s in doc])
    short = lambda doc, w: any(len(s.VersionVector) < w for s in doc)  # noqa: E731
    for w in range(R, abi.CRDT_MAX_R + 1):
        if not any(short(doc, w) and w in _doc_actors(mode, doc) for doc in docs):
            break
    else:
        raise abi.CrdtError(abi.CRDT_E_INVALID, "%s: every padded width collides with an actor" % what)
    for doc in docs:
        if short(doc, w):
            r = _replay_checks(mode, doc[0], doc[1:], w)
            if r == "panic":
                raise abi.CrdtError(abi.CRDT_E_ACTOR_RANGE, "%s: HasDot/Counter at actor == len(vv)" % what)
            if r == "pad":
                raise abi.CrdtError(abi.CRDT_E_INVALID, "%s: counter-0 dot beyond a shorter version vector" % what)
    return w


def _join_panics(dst: "AWSet", src: "AWSet") -> bool:
    """Would dst.Merge(src) panic in Go at a HasDot with actor == len(vv)?"""
    return _replay_checks(abi.CRDT_FOLD_AWSET, dst, [src], abi.CRDT_MAX_R + 1) == "panic"


def MergeBatch(dsts: Sequence[AWSet], srcs: Sequence[AWSet], engine: Optional[Engine] = None) -> None:
    """dsts[i].Merge(srcs[i]) for every i, as one batched GPU join (dsts must be distinct)."""
    if len(dsts) != len(srcs):
        raise ValueError("MergeBatch: length mismatch")
    if not dsts:
        return
    states = list(dsts) + list(srcs)
    R = _ragged_checks(abi.CRDT_FOLD_AWSET, [[a, b] for a, b in zip(dsts, srcs)], "MergeBatch")
    ids = _intern(states)
    names = {i: k for k, i in ids.items()}
    db = AWSetBatch.from_docs(R, [(_entries(s.Entries, ids), _pad(s.VersionVector, R)) for s in dsts])
    sb = AWSetBatch.from_docs(R, [(_entries(s.Entries, ids), _pad(s.VersionVector, R)) for s in srcs])
    out = (engine or default_engine()).join(db, sb)
    widths = [max(len(a.VersionVector), len(b.VersionVector)) for a, b in zip(dsts, srcs)]
    _unpack(dsts, out, names, R, widths)


def _fold(mode, dsts, srcs_per_dst, engine):
    if len(dsts) != len(srcs_per_dst):
        raise ValueError("length mismatch")
    if not dsts:
        return
    states = list(dsts) + [s for lst in srcs_per_dst for s in lst]
    R = _ragged_checks(mode, [[d] + list(lst) for d, lst in zip(dsts, srcs_per_dst)],
                       "DeltaMergeBatch" if mode == abi.CRDT_FOLD_DELTA else "FoldBatch")
    ids = _intern(states)
    names = {i: k for k, i in ids.items()}
    db = AWSetBatch.from_docs(R, [(_entries(s.Entries, ids), _pad(s.VersionVector, R)) for s in dsts])
    per_doc = [[(s.Actor, _pad(s.VersionVector, R), _entries(s.Entries, ids),
                 _entries(getattr(s, "Deleted", None), ids)) for s in lst] for lst in srcs_per_dst]
    sb = SrcBatch.from_lists(R, per_doc)
    out = (engine or default_engine()).fold(mode, db, sb)
    widths = [_fold_width(mode, d, lst) for d, lst in zip(dsts, srcs_per_dst)]
    _unpack(dsts, out, names, R, widths)


def _fold_width(mode, dst, srcs) -> int:
    """len(dst.VersionVector) after the fold, replayed on the VVs alone.  A
    delta step that brings nothing (awset-delta_test.go:60) skips
    VersionVector.Merge, so a longer source VV must not lengthen dst there; a
    step merges iff Counter(src.Actor) == 0 (full merge, :53) or
    MakeDeltaMergeData finds a changed entry or an effective tombstone
    (:79-105) -- both decided by the VV before the step and the source alone."""
    n = len(dst.VersionVector)
    if mode != abi.CRDT_FOLD_DELTA:
        return max([n] + [len(s.VersionVector) for s in srcs])
    V = list(dst.VersionVector)
    for s in srcs:
        if (V[s.Actor] if s.Actor < len(V) else 0) != 0:
            changed = any(not (d.Actor < len(V) and V[d.Actor] >= d.Counter) for d in s.Entries.values())
            ents = s.Entries
            eff = any(not (k in ents and (ents[k].Actor != d.Actor or ents[k].Counter > d.Counter))
                      for k, d in (getattr(s, "Deleted", None) or {}).items())
            if not changed and not eff:
                continue
        sv = list(s.VersionVector)
        V = [max(x, y) for x, y in zip(V, sv)] + V[len(sv):] + sv[len(V):]
    return len(V)


def FoldBatch(dsts: Sequence[AWSet], srcs_per_dst: Sequence[Sequence[AWSet]], engine: Optional[Engine] = None):
    """for each i, for src in srcs_per_dst[i] in order: dsts[i].Merge(src)."""
    _fold(abi.CRDT_FOLD_AWSET, dsts, srcs_per_dst, engine)


def DeltaMergeBatch(dsts: Sequence[AWSetDelta], srcs_per_dst: Sequence[Sequence[AWSetDelta]],
                    engine: Optional[Engine] = None):
    """for each i, for src in srcs_per_dst[i] in order: dsts[i].Merge(src) (AWSetDelta semantics)."""
    _fold(abi.CRDT_FOLD_DELTA, dsts, srcs_per_dst, engine)


def ApplyBatch(states: Sequence[AWSet], calls_per_state: Sequence[Sequence[tuple]],
               engine: Optional[Engine] = None) -> None:
    """Local ops on many replicas in one GPU call (crdt_awset_apply_batch).

    calls_per_state[i] is state i's call script, applied in order:
      ("Add", k1, k2, ...)        (*AWSet).Add          awset.go:89-94
      ("Del", k1, ...)            Del of the state's own type: (*AWSetDelta).Del
                                  (awset-delta_test.go:14-33) for an AWSetDelta,
                                  (*AWSet).Del (awset.go:96-101) otherwise
      ("AWSet.Del", k1, ...)      the embedded (*AWSet).Del of an AWSetDelta
    A call that bumps the clock with Actor >= len(VersionVector) is Go's index
    panic: CrdtError(CRDT_E_ACTOR_RANGE), nothing applied.  Each state's script
    holds at most CRDT_MAX_OPS_PER_DOC ops (one per key, plus one per delta Del)."""
    from .batch import OpBatch, TombBatch

    if len(states) != len(calls_per_state):
        raise ValueError("ApplyBatch: length mismatch")
    if not states:
        return
    R = _width(states)
    per_ops, tombs = [], []
    for s, calls in zip(states, calls_per_state):
        ops = []
        for call in calls:
            name, keys = call[0], call[1:]
            delta_del = name == "Del" and isinstance(s, AWSetDelta)
            if (name == "Add" and keys) or delta_del:  # clock bump: vv[actor]++ panics past the end
                if s.Actor >= len(s.VersionVector):
                    raise abi.CrdtError(abi.CRDT_E_ACTOR_RANGE, "ApplyBatch: %s with actor %d" % (name, s.Actor))
            if name == "Add":
                ops += [(abi.CRDT_OP_ADD, k) for k in keys]
            elif delta_del:
                ops.append((abi.CRDT_OP_DELTA_DEL, None))
                ops += [(abi.CRDT_OP_DELTA_DEL_KEY, k) for k in keys]
            elif name in ("Del", "AWSet.Del"):
                ops += [(abi.CRDT_OP_DEL, k) for k in keys]
            else:
                raise ValueError("ApplyBatch: unknown call %r" % (name,))
        per_ops.append(ops)
    # keys interned per batch (order-preserving over states, tombstones and op keys)
    names_all = set()
    for s, ops in zip(states, per_ops):
        names_all.update(s.Entries)
        names_all.update(getattr(s, "Deleted", None) or {})
        names_all.update(k for _, k in ops if k is not None)
    ids = {k: i for i, k in enumerate(sorted(names_all))}
    names = {i: k for k, i in ids.items()}
    st = AWSetBatch.from_docs(R, [(_entries(s.Entries, ids), _pad(s.VersionVector, R)) for s in states])
    tb = TombBatch.from_lists([_entries(getattr(s, "Deleted", None), ids) for s in states])
    ob = OpBatch.from_lists([[(k, ids[key] if key is not None else 0) for k, key in ops] for ops in per_ops],
                            [s.Actor for s in states])
    out, tout = (engine or default_engine()).apply(st, ob, tb)
    _unpack(states, out, names, R, [len(s.VersionVector) for s in states])
    for d, s in enumerate(states):
        if isinstance(s, AWSetDelta):
            dele = {names[k]: Dot(a, c) for k, a, c in tout.doc(d)}
            s.Deleted = dele if (dele or s.Deleted is not None) else None  # nil until the first record
