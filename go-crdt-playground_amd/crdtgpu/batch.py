"""SoA batch containers matching include/crdtgpu.h.

A batch's arrays are either numpy arrays (host: the synchronous ``*_batch``
entry points) or torch tensors on a HIP device (the ``*_async`` entry points,
inputs resident in HBM).  Device tensors use torch.int32 / torch.int64, whose
bits are the ABI's u32 / u64.
"""

from __future__ import annotations

import ctypes

import numpy as np

from .abi import CAWSetBatch, CAWSetOut, COpBatch, CSrcBatch, CTombBatch, CTombOut

U32, U64 = np.uint32, np.uint64


def _is_torch(a) -> bool:
    return a is not None and type(a).__module__.startswith("torch")


def ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags.c_contiguous:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    if not a.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return a.data_ptr()


def _np(a, dtype):
    if a is None:
        return None
    if _is_torch(a):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(a).view(dtype) if a.dtype.itemsize == np.dtype(dtype).itemsize else \
        np.ascontiguousarray(a, dtype=dtype)


def _torch(a, device):
    import torch

    if a is None:
        return None
    if _is_torch(a):
        return a.to(device)
    sdt = {1: (np.uint8, torch.uint8), 4: (np.int32, torch.int32), 8: (np.int64, torch.int64)}[a.dtype.itemsize]
    return torch.from_numpy(np.ascontiguousarray(a).view(sdt[0])).to(device)


class AWSetBatch:
    """n_docs AWSet states: doc d owns slots [offsets[d], offsets[d+1]), live = counts[d]."""

    def __init__(self, R, offsets, keys, actors, counters, vv, counts=None):
        self.R = int(R)
        self.offsets, self.keys, self.actors, self.counters, self.vv, self.counts = (
            offsets, keys, actors, counters, vv, counts)

    @property
    def n_docs(self) -> int:
        return int(self.offsets.shape[0]) - 1

    def c(self) -> CAWSetBatch:
        return CAWSetBatch(self.n_docs, self.R, ptr(self.offsets), ptr(self.counts), ptr(self.keys),
                           ptr(self.actors), ptr(self.counters), ptr(self.vv))

    def numpy(self) -> "AWSetBatch":
        return AWSetBatch(self.R, _np(self.offsets, U32), _np(self.keys, U64), _np(self.actors, U32),
                          _np(self.counters, U64), _np(self.vv, U64), _np(self.counts, U32))

    def to(self, device) -> "AWSetBatch":
        return AWSetBatch(self.R, *(_torch(a, device) for a in (self.offsets, self.keys, self.actors,
                                                                  self.counters, self.vv)),
                          counts=_torch(self.counts, device))

    # -- host helpers ---------------------------------------------------
    @staticmethod
    def from_docs(R, docs, slack=0) -> "AWSetBatch":
        """docs: list of (entries [(key, actor, counter)] sorted by key, vv [R])."""
        n = len(docs)
        counts = np.array([len(e) for e, _ in docs], dtype=U32)
        caps = counts + U32(slack)
        offsets = np.zeros(n + 1, dtype=U32)
        np.cumsum(caps, out=offsets[1:])
        total = int(offsets[-1])
        keys = np.zeros(total, dtype=U64)
        actors = np.zeros(total, dtype=U32)
        counters = np.zeros(total, dtype=U64)
        vv = np.zeros(n * R, dtype=U64)
        for d, (ents, v) in enumerate(docs):
            o = int(offsets[d])
            for i, (k, a, c) in enumerate(ents):
                keys[o + i], actors[o + i], counters[o + i] = k, a, c
            vv[d * R:(d + 1) * R] = v
        return AWSetBatch(R, offsets, keys, actors, counters, vv, counts if slack else None)

    def live(self, d) -> int:
        if self.counts is not None:
            return int(self.counts[d])
        return int(self.offsets[d + 1]) - int(self.offsets[d])

    def doc(self, d):
        """(entries [(key, actor, counter)], vv list) of doc d (host batch)."""
        o, n = int(self.offsets[d]), self.live(d)
        ents = list(zip(self.keys[o:o + n].tolist(), self.actors[o:o + n].tolist(), self.counters[o:o + n].tolist()))
        return ents, self.vv[d * self.R:(d + 1) * self.R].tolist()

    def live_slots(self) -> int:
        if self.counts is not None:
            return int(np.asarray(_np(self.counts, U32), dtype=np.uint64).sum())
        o = _np(self.offsets, U32)
        return int(o[-1]) - int(o[0])


def pinned_zeros(n, dtype):
    """A zeroed numpy array in page-locked host memory (crdt_host_alloc), freed
    with the array.  The *_batch calls stage inputs that lie in one such block
    with one copy, and write packed outputs that lie in such blocks from the
    gather kernel (api.cpp, fetch_outputs)."""
    import weakref

    from . import abi

    lib = abi.lib()
    nbytes = max(int(n), 1) * np.dtype(dtype).itemsize
    p = ctypes.c_void_p()
    rc = lib.crdt_host_alloc(nbytes, ctypes.byref(p))
    if rc != 0:
        raise MemoryError("crdt_host_alloc(%d): %d" % (nbytes, rc))
    buf = (ctypes.c_char * nbytes).from_address(p.value)
    arr = np.frombuffer(buf, dtype=dtype, count=max(int(n), 1))
    arr[:] = 0
    weakref.finalize(buf, lib.crdt_host_free, ctypes.c_void_p(p.value))
    return arr


class OutBuffers:
    """Output of a join/fold: n_docs docs, `slots` capacity, numpy or torch.
    shared_keys: another OutBuffers whose key column this one uses (the two
    outputs of an exchange hold the same keys at the same slots,
    crdt_awset_exchange_async).  pinned: host arrays in page-locked memory."""

    def __init__(self, n_docs, R, slots, device=None, shared_keys=None, pinned=False):
        self.R, self.n_docs, self.slots = int(R), int(n_docs), int(slots)
        if device is None:
            z = pinned_zeros if pinned else (lambda n, dt: np.zeros(n, dtype=dt))
            self.offsets = z(n_docs + 1, U32)
            self.counts = z(n_docs, U32)[:n_docs]
            self.keys = z(max(slots, 1), U64)
            self.actors = z(max(slots, 1), U32)
            self.counters = z(max(slots, 1), U64)
            self.vv = z(max(n_docs * R, 1), U64)
        else:
            import torch

            e = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=device)  # noqa: E731
            self.offsets = e(n_docs + 1, torch.int32)[: n_docs + 1]
            self.counts = e(n_docs, torch.int32)[:n_docs]
            self.keys = e(slots if shared_keys is None else 0, torch.int64)
            self.actors = e(slots, torch.int32)
            self.counters = e(slots, torch.int64)
            self.vv = e(n_docs * R, torch.int64)
        if shared_keys is not None:
            assert shared_keys.slots >= self.slots
            self.keys = shared_keys.keys

    def c(self) -> CAWSetOut:
        return CAWSetOut(ptr(self.offsets), ptr(self.counts), ptr(self.keys), ptr(self.actors), ptr(self.counters),
                         ptr(self.vv))

    def as_batch(self) -> AWSetBatch:
        return AWSetBatch(self.R, self.offsets, self.keys, self.actors, self.counters, self.vv, counts=self.counts)


class SrcBatch:
    """Ordered sources folded into each doc (AWSet or AWSetDelta states)."""

    def __init__(self, R, doc_srcs, src_actor, vv, entry_off, keys, actors, counters,
                 tomb_off=None, tkeys=None, tactors=None, tcounters=None):
        self.R = int(R)
        self.doc_srcs, self.src_actor, self.vv, self.entry_off = doc_srcs, src_actor, vv, entry_off
        self.keys, self.actors, self.counters = keys, actors, counters
        self.tomb_off, self.tkeys, self.tactors, self.tcounters = tomb_off, tkeys, tactors, tcounters

    @property
    def n_docs(self) -> int:
        return int(self.doc_srcs.shape[0]) - 1

    @property
    def n_srcs(self) -> int:
        return int(self.src_actor.shape[0])

    def c(self) -> CSrcBatch:
        return CSrcBatch(self.n_docs, self.R, ptr(self.doc_srcs), ptr(self.src_actor), ptr(self.vv),
                         ptr(self.entry_off), ptr(self.keys), ptr(self.actors), ptr(self.counters),
                         ptr(self.tomb_off), ptr(self.tkeys), ptr(self.tactors), ptr(self.tcounters))

    _FIELDS = (("doc_srcs", U32), ("src_actor", U32), ("vv", U64), ("entry_off", U32), ("keys", U64),
               ("actors", U32), ("counters", U64), ("tomb_off", U32), ("tkeys", U64), ("tactors", U32),
               ("tcounters", U64))

    def to(self, device) -> "SrcBatch":
        return SrcBatch(self.R, *(_torch(getattr(self, f), device) for f, _ in self._FIELDS))

    def numpy(self) -> "SrcBatch":
        return SrcBatch(self.R, *(_np(getattr(self, f), dt) for f, dt in self._FIELDS))

    @staticmethod
    def from_lists(R, per_doc) -> "SrcBatch":
        """per_doc[d] = list of sources (actor, vv, entries [(k,a,c)], tombstones [(k,a,c)] or None)."""
        srcs = [s for lst in per_doc for s in lst]
        doc_srcs = np.zeros(len(per_doc) + 1, dtype=U32)
        np.cumsum([len(lst) for lst in per_doc], out=doc_srcs[1:])
        ns = len(srcs)
        src_actor = np.array([s[0] for s in srcs], dtype=U32).reshape(ns)
        vv = np.zeros(max(ns * R, 1), dtype=U64)
        entry_off = np.zeros(ns + 1, dtype=U32)
        tomb_off = np.zeros(ns + 1, dtype=U32)
        for i, s in enumerate(srcs):
            vv[i * R:(i + 1) * R] = s[1]
            entry_off[i + 1] = entry_off[i] + len(s[2])
            tomb_off[i + 1] = tomb_off[i] + len(s[3] or [])
        def flat(idx, off):
            n = int(off[-1])
            k, a, c = np.zeros(max(n, 1), U64), np.zeros(max(n, 1), U32), np.zeros(max(n, 1), U64)
            for i, s in enumerate(srcs):
                for j, (kk, aa, cc) in enumerate(s[idx] or []):
                    k[off[i] + j], a[off[i] + j], c[off[i] + j] = kk, aa, cc
            return k, a, c
        keys, actors, counters = flat(2, entry_off)
        tkeys, tactors, tcounters = flat(3, tomb_off)
        return SrcBatch(R, doc_srcs, src_actor, vv, entry_off, keys, actors, counters,
                        tomb_off, tkeys, tactors, tcounters)

    def out_slots(self, dst: AWSetBatch) -> int:
        eo = _np(self.entry_off, U32)
        return int(_np(dst.offsets, U32)[-1]) + int(eo[-1])


class SrcBuffers(SrcBatch):
    """Device (torch) or host (numpy) storage for n_srcs sources of fixed
    entry / tombstone slot counts (what the workload generators fill)."""

    def __init__(self, R, n_docs, n_srcs, entry_slots, tomb_slots, device=None):
        if device is None:
            z = lambda n, dt: np.zeros(max(n, 1), dtype=dt)  # noqa: E731
            i32, i64 = U32, U64
        else:
            import torch

            z = lambda n, dt: torch.zeros(max(n, 1), dtype=dt, device=device)  # noqa: E731
            i32, i64 = torch.int32, torch.int64
        super().__init__(R, z(n_docs + 1, i32)[: n_docs + 1], z(n_srcs, i32)[:n_srcs], z(n_srcs * R, i64),
                         z(n_srcs + 1, i32)[: n_srcs + 1], z(entry_slots, i64), z(entry_slots, i32),
                         z(entry_slots, i64), z(n_srcs + 1, i32)[: n_srcs + 1], z(tomb_slots, i64),
                         z(tomb_slots, i32), z(tomb_slots, i64))


class OpBatch:
    """Per doc an ordered list of local ops (include/crdtgpu.h, CRDT_OP_*) and
    the doc's replica actor."""

    def __init__(self, op_off, kind, keys, doc_actor):
        self.op_off, self.kind, self.keys, self.doc_actor = op_off, kind, keys, doc_actor

    @property
    def n_docs(self) -> int:
        return int(self.op_off.shape[0]) - 1

    def c(self) -> COpBatch:
        return COpBatch(self.n_docs, ptr(self.op_off), ptr(self.kind), ptr(self.keys), ptr(self.doc_actor))

    def numpy(self) -> "OpBatch":
        return OpBatch(_np(self.op_off, U32), _np(self.kind, np.uint8), _np(self.keys, U64),
                       _np(self.doc_actor, U32))

    def to(self, device) -> "OpBatch":
        return OpBatch(*(_torch(a, device) for a in (self.op_off, self.kind, self.keys, self.doc_actor)))

    @staticmethod
    def from_lists(per_doc, actors) -> "OpBatch":
        """per_doc[d] = [(kind, key)], actors[d] = the doc's replica actor."""
        op_off = np.zeros(len(per_doc) + 1, dtype=U32)
        np.cumsum([len(x) for x in per_doc], out=op_off[1:])
        n = int(op_off[-1])
        kind = np.zeros(max(n, 1), dtype=np.uint8)
        keys = np.zeros(max(n, 1), dtype=U64)
        i = 0
        for lst in per_doc:
            for k, key in lst:
                kind[i], keys[i] = k, key
                i += 1
        return OpBatch(op_off, kind, keys, np.asarray(actors, dtype=U32).reshape(len(per_doc)))


class TombBatch:
    """AWSetDelta.Deleted of each doc: sorted (key, actor, counter) per doc."""

    def __init__(self, offsets, keys, actors, counters, counts=None):
        self.offsets, self.keys, self.actors, self.counters, self.counts = offsets, keys, actors, counters, counts

    @property
    def n_docs(self) -> int:
        return int(self.offsets.shape[0]) - 1

    def c(self) -> CTombBatch:
        return CTombBatch(ptr(self.offsets), ptr(self.counts), ptr(self.keys), ptr(self.actors), ptr(self.counters))

    def numpy(self) -> "TombBatch":
        return TombBatch(_np(self.offsets, U32), _np(self.keys, U64), _np(self.actors, U32), _np(self.counters, U64),
                         _np(self.counts, U32))

    def to(self, device) -> "TombBatch":
        return TombBatch(*(_torch(a, device) for a in (self.offsets, self.keys, self.actors, self.counters)),
                         counts=_torch(self.counts, device))

    @staticmethod
    def from_lists(per_doc) -> "TombBatch":
        offsets = np.zeros(len(per_doc) + 1, dtype=U32)
        np.cumsum([len(x) for x in per_doc], out=offsets[1:])
        n = int(offsets[-1])
        k, a, c = np.zeros(max(n, 1), U64), np.zeros(max(n, 1), U32), np.zeros(max(n, 1), U64)
        i = 0
        for lst in per_doc:
            for kk, aa, cc in lst:
                k[i], a[i], c[i] = kk, aa, cc
                i += 1
        return TombBatch(offsets, k, a, c)

    def doc(self, d):
        o = int(self.offsets[d])
        n = int(self.counts[d]) if self.counts is not None else int(self.offsets[d + 1]) - o
        return list(zip(self.keys[o:o + n].tolist(), self.actors[o:o + n].tolist(), self.counters[o:o + n].tolist()))


class TombBuffers(TombBatch):
    """Output tombstones of an apply call (numpy, or torch on `device`)."""

    def __init__(self, n_docs, slots, device=None):
        if device is None:
            super().__init__(np.zeros(n_docs + 1, U32), np.zeros(max(slots, 1), U64), np.zeros(max(slots, 1), U32),
                             np.zeros(max(slots, 1), U64), np.zeros(max(n_docs, 1), U32)[:n_docs])
        else:
            import torch

            e = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=device)  # noqa: E731
            super().__init__(e(n_docs + 1, torch.int32)[: n_docs + 1], e(slots, torch.int64), e(slots, torch.int32),
                             e(slots, torch.int64), e(n_docs, torch.int32)[:n_docs])

    def c_out(self) -> CTombOut:
        return CTombOut(ptr(self.offsets), ptr(self.counts), ptr(self.keys), ptr(self.actors), ptr(self.counters))


def c_ref(x):
    return ctypes.byref(x)
