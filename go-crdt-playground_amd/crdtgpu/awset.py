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

Differences from the Go code, all at inputs where Go panics or is ambiguous:
  * a batch's version vectors are zero-padded to the longest one (R <= 64).
    The kernels flag HasDot at actor == R; for a shorter vector the panic at
    actor == len(vv) is found on the host before the launch -- exactly for
    MergeBatch (the HasDot calls of awset.go:133 and :152 are replayed on the
    keys alone).  Folds over vectors of unequal lengths read the pad instead
    of panicking; equal-length vectors (every reference test) are exact.
  * where Go panics (actor == len(vv)), the merge raises CrdtError
    (CRDT_E_ACTOR_RANGE) and leaves the destination untouched.
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


def _join_panics(dst: "AWSet", src: "AWSet") -> bool:
    """Would dst.Merge(src) panic in Go at a HasDot with actor == len(vv)?  The
    reference evaluates dstVV.HasDot(s) for every src-only key (awset.go:133)
    and srcVV.HasDot(d) for every dst-only key (:152)."""
    ld, ls = len(dst.VersionVector), len(src.VersionVector)
    if any(k not in dst.Entries and s.Actor == ld for k, s in src.Entries.items()):
        return True
    return any(k not in src.Entries and d.Actor == ls for k, d in dst.Entries.items())


def MergeBatch(dsts: Sequence[AWSet], srcs: Sequence[AWSet], engine: Optional[Engine] = None) -> None:
    """dsts[i].Merge(srcs[i]) for every i, as one batched GPU join (dsts must be distinct)."""
    if len(dsts) != len(srcs):
        raise ValueError("MergeBatch: length mismatch")
    if not dsts:
        return
    states = list(dsts) + list(srcs)
    R = _width(states)
    for a, b in zip(dsts, srcs):  # vectors shorter than R: their panic point is below the kernels' actor == R
        if (len(a.VersionVector) < R or len(b.VersionVector) < R) and _join_panics(a, b):
            raise abi.CrdtError(abi.CRDT_E_ACTOR_RANGE, "MergeBatch: HasDot at actor == len(vv)")
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
    ids = _intern(states)
    names = {i: k for k, i in ids.items()}
    R = _width(states)
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
