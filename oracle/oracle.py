"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the C oracle (awset_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, as the checker.  It takes the same SoA batches as the product
(the ctypes struct layouts are imported from the product's ABI mirror; the
product never imports the oracle).
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "go-crdt-playground_amd"))

from crdtgpu.abi import CAWSetBatch, CAWSetOut, COpBatch, CSrcBatch, CTombBatch, CTombOut  # noqa: E402
from crdtgpu.batch import AWSetBatch, OpBatch, OutBuffers, SrcBatch, TombBatch, TombBuffers  # noqa: E402

LIB = os.path.join(HERE, "build", "liboracle.so")
MAPLIB = os.path.join(HERE, "build", "libawsetmap.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or not os.path.exists(MAPLIB):
        subprocess.check_call(["make", "-s", "-C", HERE, "all"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        _lib.oracle_awset_join.restype = ctypes.c_int
        _lib.oracle_awset_join.argtypes = [P(CAWSetBatch), P(CAWSetBatch), P(CAWSetOut)]
        _lib.oracle_awset_fold.restype = ctypes.c_int
        _lib.oracle_awset_fold.argtypes = [ctypes.c_int, P(CAWSetBatch), P(CSrcBatch), P(CAWSetOut)]
        _lib.oracle_awset_apply.restype = ctypes.c_int
        _lib.oracle_awset_apply.argtypes = [P(CAWSetBatch), P(CTombBatch), P(COpBatch), P(CAWSetOut), P(CTombOut)]
        _lib.oracle_tomb_gc.restype = ctypes.c_int
        _lib.oracle_tomb_gc.argtypes = [P(CTombBatch), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, P(CTombOut)]
        _lib.oracle_causal_context.restype = None
        _lib.oracle_causal_context.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    return _lib


def join(dst: AWSetBatch, src: AWSetBatch):
    """(status, OutBuffers) of out[d] = dst[d] <- src[d]."""
    dst, src = dst.numpy(), src.numpy()
    out = OutBuffers(dst.n_docs, dst.R, int(dst.offsets[-1]) + int(src.offsets[-1]))
    d, s, o = dst.c(), src.c(), out.c()
    rc = lib().oracle_awset_join(ctypes.byref(d), ctypes.byref(s), ctypes.byref(o))
    return rc, out


def fold(mode: int, dst: AWSetBatch, srcs: SrcBatch):
    dst, srcs = dst.numpy(), srcs.numpy()
    out = OutBuffers(dst.n_docs, dst.R, srcs.out_slots(dst))
    d, s, o = dst.c(), srcs.c(), out.c()
    rc = lib().oracle_awset_fold(int(mode), ctypes.byref(d), ctypes.byref(s), ctypes.byref(o))
    return rc, out


def apply(state: AWSetBatch, ops: OpBatch, tombs: TombBatch = None, with_tombs: bool = True):
    """(status, entries out, tombstones out or None) after each doc's local ops
    (awset.go:89-101, awset-delta_test.go:14-33), same layout as crdt_awset_apply_*."""
    state, ops = state.numpy(), ops.numpy()
    tombs = tombs.numpy() if tombs is not None else None
    nops = int(ops.op_off[-1])
    out = OutBuffers(state.n_docs, state.R, int(state.offsets[-1]) + nops)
    tout = TombBuffers(state.n_docs, (int(tombs.offsets[-1]) if tombs is not None else 0) + nops) if with_tombs else None
    cs, co, cout = state.c(), ops.c(), out.c()
    ct = tombs.c() if tombs is not None else None
    cto = tout.c_out() if tout is not None else None
    rc = lib().oracle_awset_apply(ctypes.byref(cs), ctypes.byref(ct) if ct else None, ctypes.byref(co),
                                  ctypes.byref(cout), ctypes.byref(cto) if cto else None)
    return rc, out, tout


def tomb_gc(tombs: TombBatch, R: int, stable: np.ndarray):
    """(status, TombBuffers): tombstones not covered by each doc's stable clock."""
    tombs = tombs.numpy()
    n = tombs.n_docs
    out = TombBuffers(n, int(tombs.offsets[-1]))
    st = np.ascontiguousarray(stable, dtype=np.uint64)
    ct, co = tombs.c(), out.c_out()
    rc = lib().oracle_tomb_gc(ctypes.byref(ct), n, int(R), st.ctypes.data, ctypes.byref(co))
    return rc, out


def causal_context(vv: np.ndarray, n_docs: int, R: int) -> np.ndarray:
    vv = np.ascontiguousarray(vv, dtype=np.uint64)
    out = np.zeros(R, dtype=np.uint64)
    lib().oracle_causal_context(vv.ctypes.data, n_docs, R, out.ctypes.data)
    return out


# ---- the map[string]Dot restatement (awset_map.cpp): second oracle + CPU baseline

_maplib = None


def maplib():
    global _maplib
    if _maplib is None:
        build()
        _maplib = ctypes.CDLL(MAPLIB)
        P = ctypes.POINTER
        m = _maplib
        m.awmap_join.restype = ctypes.c_int
        m.awmap_join.argtypes = [P(CAWSetBatch), P(CAWSetBatch), P(CAWSetOut)]
        m.awmap_fold.restype = ctypes.c_int
        m.awmap_fold.argtypes = [ctypes.c_int, P(CAWSetBatch), P(CSrcBatch), P(CAWSetOut)]
        m.awmap_bench_join.restype = ctypes.c_double
        m.awmap_bench_join.argtypes = [P(CAWSetBatch), P(CAWSetBatch), ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                       P(ctypes.c_uint64)]
        m.awmap_bench_fold.restype = ctypes.c_double
        m.awmap_bench_fold.argtypes = [ctypes.c_int, P(CAWSetBatch), P(CSrcBatch), ctypes.c_int, ctypes.c_double,
                                       P(ctypes.c_uint64)]
    return _maplib


def map_join(dst: AWSetBatch, src: AWSetBatch):
    """As join(), through the hash-map restatement."""
    dst, src = dst.numpy(), src.numpy()
    out = OutBuffers(dst.n_docs, dst.R, int(dst.offsets[-1]) + int(src.offsets[-1]))
    d, s, o = dst.c(), src.c(), out.c()
    rc = maplib().awmap_join(ctypes.byref(d), ctypes.byref(s), ctypes.byref(o))
    return rc, out


def map_fold(mode: int, dst: AWSetBatch, srcs: SrcBatch):
    """As fold(), through the hash-map restatement."""
    dst, srcs = dst.numpy(), srcs.numpy()
    out = OutBuffers(dst.n_docs, dst.R, srcs.out_slots(dst))
    d, s, o = dst.c(), srcs.c(), out.c()
    rc = maplib().awmap_fold(int(mode), ctypes.byref(d), ctypes.byref(s), ctypes.byref(o))
    return rc, out


def map_bench_join(a: AWSetBatch, b: AWSetBatch, both_dirs: bool, threads: int, budget_s: float):
    """(merges, timed seconds) of repeated map merges a <- b (and b <- a), maps cloned untimed per pass."""
    a, b = a.numpy(), b.numpy()
    ca, cb = a.c(), b.c()
    m = ctypes.c_uint64(0)
    t = maplib().awmap_bench_join(ctypes.byref(ca), ctypes.byref(cb), int(both_dirs), int(threads), float(budget_s),
                                  ctypes.byref(m))
    if t < 0:
        raise RuntimeError("map baseline: a merge panicked (actor == len(VV))")
    return int(m.value), t


def map_bench_fold(mode: int, dst: AWSetBatch, srcs: SrcBatch, threads: int, budget_s: float):
    """(merges, timed seconds) of repeated ordered map folds, dst maps cloned untimed per pass."""
    dst, srcs = dst.numpy(), srcs.numpy()
    cd, cs = dst.c(), srcs.c()
    m = ctypes.c_uint64(0)
    t = maplib().awmap_bench_fold(int(mode), ctypes.byref(cd), ctypes.byref(cs), int(threads), float(budget_s),
                                  ctypes.byref(m))
    if t < 0:
        raise RuntimeError("map baseline: a merge panicked (actor == len(VV))")
    return int(m.value), t


def cpu_threads() -> int:
    """Host threads a baseline may use: the affinity set, capped by OMP_NUM_THREADS when set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)
