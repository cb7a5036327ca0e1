"""Engine: one crdt_ctx (one per host thread), the batched merge entry points."""

from __future__ import annotations

import ctypes

from . import abi
from .abi import check
from .batch import AWSetBatch, OpBatch, OutBuffers, SrcBatch, TombBatch, TombBuffers, ptr


def _c(x):
    """ctypes struct of a batch/output (or the struct itself, prebuilt by the caller
    to keep per-launch host work at a few ctypes calls)."""
    return x.c() if hasattr(x, "c") else x


def _stream(stream):
    if stream is None:
        return None
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


class Engine:
    def __init__(self, device: int = 0):
        self._lib = abi.lib()
        h = ctypes.c_void_p()
        check(self._lib.crdt_ctx_create(int(device), ctypes.byref(h)), "crdt_ctx_create")
        self._ctx = h
        self.device = device

    def close(self):
        if self._ctx:
            self._lib.crdt_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- workspace / errors ------------------------------------------------
    def reserve(self, max_docs: int, max_fold_slots: int = 0):
        check(self._lib.crdt_ctx_reserve(self._ctx, int(max_docs), int(max_fold_slots)), "crdt_ctx_reserve")

    def set_max_doc_entries(self, n: int = 0xFFFFFFFF):
        check(self._lib.crdt_ctx_set_max_doc_entries(self._ctx, int(n)), "crdt_ctx_set_max_doc_entries")

    def set_option(self, name: str, value: int):
        check(self._lib.crdt_ctx_set_option(self._ctx, name.encode(), int(value)), "crdt_ctx_set_option")

    def sync(self, stream=None):
        check(self._lib.crdt_ctx_sync(self._ctx, _stream(stream)), "crdt_ctx_sync")

    def clock_probe(self) -> float:
        """Shader clock in MHz under an all-CU integer load (crdt_clock_probe)."""
        g = ctypes.c_double()
        check(self._lib.crdt_clock_probe(self._ctx, ctypes.byref(g)), "crdt_clock_probe")
        return g.value

    def bw_probe(self, kind: int, a, b, nbytes: int, reps: int = 10) -> float:
        """GB/s of a streaming read / write / copy over device buffers a, b (crdt_bw_probe)."""
        g = ctypes.c_double()
        pa = a.data_ptr() if a is not None else None
        check(self._lib.crdt_bw_probe(self._ctx, int(kind), pa, b.data_ptr(), int(nbytes), int(reps), ctypes.byref(g)),
              "crdt_bw_probe")
        return g.value

    # -- device-resident, asynchronous -------------------------------------
    def join_async(self, dst: AWSetBatch, src: AWSetBatch, out: OutBuffers, stream=None):
        d, s, o = _c(dst), _c(src), _c(out)
        check(self._lib.crdt_awset_join_async(self._ctx, ctypes.byref(d), ctypes.byref(s), ctypes.byref(o),
                                              _stream(stream)), "crdt_awset_join_async")

    def exchange_async(self, a: AWSetBatch, b: AWSetBatch, out_ab: OutBuffers, out_ba: OutBuffers, stream=None):
        ca, cb, o1, o2 = _c(a), _c(b), _c(out_ab), _c(out_ba)
        check(self._lib.crdt_awset_exchange_async(self._ctx, ctypes.byref(ca), ctypes.byref(cb), ctypes.byref(o1),
                                                  ctypes.byref(o2), _stream(stream)), "crdt_awset_exchange_async")

    def fold_async(self, mode: int, dst: AWSetBatch, srcs: SrcBatch, out: OutBuffers, stream=None):
        d, s, o = _c(dst), _c(srcs), _c(out)
        check(self._lib.crdt_awset_fold_async(self._ctx, int(mode), ctypes.byref(d), ctypes.byref(s),
                                              ctypes.byref(o), _stream(stream)), "crdt_awset_fold_async")

    def vv_max_async(self, dst, src, n: int, stream=None):
        check(self._lib.crdt_vv_max_async(self._ctx, ptr(dst), ptr(src), int(n), _stream(stream)),
              "crdt_vv_max_async")

    def causal_context_async(self, vv, n_docs: int, R: int, out, stream=None):
        check(self._lib.crdt_causal_context_async(self._ctx, ptr(vv), int(n_docs), int(R), ptr(out),
                                                  _stream(stream)), "crdt_causal_context_async")

    def apply_async(self, state: AWSetBatch, ops: OpBatch, out: OutBuffers, tombs: TombBatch = None,
                    tomb_out: TombBuffers = None, stream=None):
        """Device-resident batched Add / Del / AWSetDelta.Del (crdt_awset_apply_async)."""
        cs, co, cout = _c(state), _c(ops), _c(out)
        ct = _c(tombs) if tombs is not None else None
        cto = tomb_out.c_out() if tomb_out is not None else None
        check(self._lib.crdt_awset_apply_async(self._ctx, ctypes.byref(cs), ctypes.byref(ct) if ct else None,
                                               ctypes.byref(co), ctypes.byref(cout),
                                               ctypes.byref(cto) if cto else None, _stream(stream)),
              "crdt_awset_apply_async")

    def sort_async(self, batch: AWSetBatch, n_slots: int, out: OutBuffers, stream=None):
        """Ingest sort: each doc's live entries ordered by key (crdt_awset_sort_async)."""
        cb, co = _c(batch), _c(out)
        check(self._lib.crdt_awset_sort_async(self._ctx, ctypes.byref(cb), int(n_slots), ctypes.byref(co),
                                              _stream(stream)), "crdt_awset_sort_async")

    def sort(self, batch: AWSetBatch) -> OutBuffers:
        """Host buffers: the batch with each doc's live entries sorted by key."""
        b = batch.numpy()
        out = OutBuffers(b.n_docs, b.R, int(b.offsets[-1]))
        cb, co = b.c(), out.c()
        check(self._lib.crdt_awset_sort_batch(self._ctx, ctypes.byref(cb), ctypes.byref(co)), "crdt_awset_sort_batch")
        return out

    def tombstone_gc_async(self, tombs: TombBatch, R: int, stable_vv, out: TombBuffers, stream=None):
        """Opt-in GC: drop each doc's tombstones its stable clock covers (crdt_tombstone_gc_async)."""
        ct, co = _c(tombs), out.c_out()
        check(self._lib.crdt_tombstone_gc_async(self._ctx, ctypes.byref(ct), tombs.n_docs, int(R), ptr(stable_vv),
                                                ctypes.byref(co), _stream(stream)), "crdt_tombstone_gc_async")

    def vv_min_async(self, dst, src, n: int, stream=None):
        check(self._lib.crdt_vv_min_async(self._ctx, ptr(dst), ptr(src), int(n), _stream(stream)),
              "crdt_vv_min_async")

    # -- multi-GPU: global causal context over RCCL ------------------------
    def comm_init(self, n_ranks: int, rank: int, uid: bytes):
        """One process per GPU: join the communicator of `uid` (crdt_comm_unique_id on rank 0)."""
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        check(self._lib.crdt_comm_init(self._ctx, int(n_ranks), int(rank), buf), "crdt_comm_init")

    def context_allreduce_async(self, vv_R, R: int, stream=None):
        """In-place u64 max of this rank's R-vector with every other rank's (RCCL)."""
        check(self._lib.crdt_context_allreduce_async(self._ctx, ptr(vv_R), int(R), _stream(stream)),
              "crdt_context_allreduce_async")

    def gen_pair_async(self, seed: int, n_docs: int, a: OutBuffers, b: OutBuffers, stream=None):
        ca, cb = a.c(), b.c()
        check(self._lib.crdt_gen_pair_async(self._ctx, int(seed), int(n_docs), ctypes.byref(ca), ctypes.byref(cb),
                                            _stream(stream)), "crdt_gen_pair_async")

    def gen_delta_async(self, seed: int, n_docs: int, R: int, M: int, dst: OutBuffers, srcs: SrcBatch, stream=None):
        cd, cs = dst.c(), srcs.c()
        check(self._lib.crdt_gen_delta_async(self._ctx, int(seed), int(n_docs), int(R), int(M), ctypes.byref(cd),
                                             ctypes.byref(cs), _stream(stream)), "crdt_gen_delta_async")

    def gen_replicas_async(self, seed: int, n_docs: int, P: int, E: int, dst: OutBuffers, srcs: SrcBatch,
                           stream=None):
        cd, cs = dst.c(), srcs.c()
        check(self._lib.crdt_gen_replicas_async(self._ctx, int(seed), int(n_docs), int(P), int(E), ctypes.byref(cd),
                                                ctypes.byref(cs), _stream(stream)), "crdt_gen_replicas_async")

    def gen_zipf_async(self, seed: int, n_docs: int, offsets, a: OutBuffers, b: OutBuffers, stream=None):
        ca, cb = a.c(), b.c()
        check(self._lib.crdt_gen_zipf_async(self._ctx, int(seed), int(n_docs), ptr(offsets), ctypes.byref(ca),
                                            ctypes.byref(cb), _stream(stream)), "crdt_gen_zipf_async")

    # -- host buffers, synchronous ----------------------------------------
    def join(self, dst: AWSetBatch, src: AWSetBatch, pinned: bool = False) -> OutBuffers:
        """Host buffers; pinned: the output in page-locked memory (crdt_host_alloc)."""
        dst, src = dst.numpy(), src.numpy()
        out = OutBuffers(dst.n_docs, dst.R, int(dst.offsets[-1]) + int(src.offsets[-1]), pinned=pinned)
        d, s, o = dst.c(), src.c(), out.c()
        check(self._lib.crdt_awset_join_batch(self._ctx, ctypes.byref(d), ctypes.byref(s), ctypes.byref(o)),
              "crdt_awset_join_batch")
        return out

    def exchange(self, a: AWSetBatch, b: AWSetBatch, shared_keys: bool = False, pinned: bool = False):
        """Host buffers: (a <- b, b <- a); shared_keys: both outputs use one key column;
        pinned: the outputs in page-locked memory (crdt_host_alloc)."""
        a, b = a.numpy(), b.numpy()
        slots = int(a.offsets[-1]) + int(b.offsets[-1])
        o1 = OutBuffers(a.n_docs, a.R, slots, pinned=pinned)
        o2 = OutBuffers(a.n_docs, a.R, slots, shared_keys=o1 if shared_keys else None, pinned=pinned)
        ca, cb, c1, c2 = a.c(), b.c(), o1.c(), o2.c()
        check(self._lib.crdt_awset_exchange_batch(self._ctx, ctypes.byref(ca), ctypes.byref(cb), ctypes.byref(c1),
                                                  ctypes.byref(c2)), "crdt_awset_exchange_batch")
        return o1, o2

    def apply(self, state: AWSetBatch, ops: OpBatch, tombs: TombBatch = None, with_tombs: bool = True):
        """Host buffers: (entries out, tombstones out or None) after each doc's ops."""
        state, ops = state.numpy(), ops.numpy()
        tombs = tombs.numpy() if tombs is not None else None
        nops = int(ops.op_off[-1])
        out = OutBuffers(state.n_docs, state.R, int(state.offsets[-1]) + nops)
        tout = TombBuffers(state.n_docs, (int(tombs.offsets[-1]) if tombs is not None else 0) + nops) \
            if with_tombs else None
        cs, co, cout = state.c(), ops.c(), out.c()
        ct = tombs.c() if tombs is not None else None
        cto = tout.c_out() if tout is not None else None
        check(self._lib.crdt_awset_apply_batch(self._ctx, ctypes.byref(cs), ctypes.byref(ct) if ct else None,
                                               ctypes.byref(co), ctypes.byref(cout),
                                               ctypes.byref(cto) if cto else None), "crdt_awset_apply_batch")
        return out, tout

    def fold(self, mode: int, dst: AWSetBatch, srcs: SrcBatch, pinned: bool = False) -> OutBuffers:
        dst, srcs = dst.numpy(), srcs.numpy()
        out = OutBuffers(dst.n_docs, dst.R, srcs.out_slots(dst), pinned=pinned)
        d, s, o = dst.c(), srcs.c(), out.c()
        check(self._lib.crdt_awset_fold_batch(self._ctx, int(mode), ctypes.byref(d), ctypes.byref(s),
                                              ctypes.byref(o)), "crdt_awset_fold_batch")
        return out


def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id (rank 0 makes it, every rank passes it to comm_init)."""
    buf = ctypes.create_string_buffer(128)
    check(abi.lib().crdt_comm_unique_id(buf), "crdt_comm_unique_id")
    return buf.raw


def global_context_allreduce(engines, vvs, R: int):
    """One process, one Engine per GPU: every vvs[i] (device R-vector on engine i's
    GPU) becomes the elementwise u64 max over all of them; returns it as a list."""
    n = len(engines)
    ctxs = (ctypes.c_void_p * n)(*[e._ctx for e in engines])
    ptrs = (ctypes.c_void_p * n)(*[ptr(v) for v in vvs])
    out = (ctypes.c_uint64 * int(R))()
    check(abi.lib().crdt_global_context_allreduce(ctxs, n, ptrs, int(R), ctypes.cast(out, ctypes.c_void_p)),
          "crdt_global_context_allreduce")
    return [int(x) for x in out]


def format_doc(batch: AWSetBatch, d: int, names=None) -> str:
    """Go's (AWSet).String() of doc d of a host batch (crdt_awset_format); names[id] = key string."""
    b = batch.numpy()
    cb = b.c()
    arr = None
    if names is not None:
        enc = [n.encode() if isinstance(n, str) else bytes(n) for n in names]
        arr = (ctypes.c_char_p * len(enc))(*enc)
    n = ctypes.c_size_t(0)
    check(abi.lib().crdt_awset_format(ctypes.byref(cb), int(d), arr, None, 0, ctypes.byref(n)), "crdt_awset_format")
    buf = ctypes.create_string_buffer(n.value + 1)
    check(abi.lib().crdt_awset_format(ctypes.byref(cb), int(d), arr, buf, n.value + 1, ctypes.byref(n)),
          "crdt_awset_format")
    return buf.raw[: n.value].decode("utf-8", errors="surrogateescape")


def dump_batch(batch: AWSetBatch) -> bytes:
    """Self-checking binary image of a host batch (crdt_batch_dump)."""
    b = batch.numpy()
    cb = b.c()
    n = ctypes.c_size_t(0)
    check(abi.lib().crdt_batch_dump(ctypes.byref(cb), None, 0, ctypes.byref(n)), "crdt_batch_dump")
    buf = ctypes.create_string_buffer(n.value)
    check(abi.lib().crdt_batch_dump(ctypes.byref(cb), buf, n.value, ctypes.byref(n)), "crdt_batch_dump")
    return buf.raw


def load_batch(image: bytes) -> AWSetBatch:
    """Inverse of dump_batch: a compact host batch (crdt_batch_info + crdt_batch_undump)."""
    import numpy as np

    nd, R, ne = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_uint64(0)
    buf = ctypes.create_string_buffer(bytes(image), len(image))
    check(abi.lib().crdt_batch_info(buf, len(image), ctypes.byref(nd), ctypes.byref(R), ctypes.byref(ne)),
          "crdt_batch_info")
    out = OutBuffers(nd.value, R.value, ne.value)
    co = out.c()
    check(abi.lib().crdt_batch_undump(buf, len(image), ctypes.byref(co)), "crdt_batch_undump")
    return AWSetBatch(R.value, out.offsets, out.keys, out.actors, out.counters, out.vv,
                      counts=out.counts if nd.value else np.zeros(0, np.uint32))


def zipf_sizes(seed: int, n_docs: int):
    """Document sizes of the "zipf" workload (host computation, no GPU)."""
    import numpy as np

    out = np.zeros(max(n_docs, 1), dtype=np.uint32)
    check(abi.lib().crdt_gen_zipf_sizes(int(seed), int(n_docs), out.ctypes.data), "crdt_gen_zipf_sizes")
    return out[:n_docs]


def validate(batch: AWSetBatch) -> int:
    b = batch.numpy().c()
    return abi.lib().crdt_validate_batch(ctypes.byref(b))


def validate_src(srcs: SrcBatch) -> int:
    s = srcs.numpy().c()
    return abi.lib().crdt_validate_src_batch(ctypes.byref(s))


def validate_tombs(tombs, n_docs: int) -> int:
    t = tombs.numpy().c()
    return abi.lib().crdt_validate_tomb_batch(ctypes.byref(t), n_docs)
