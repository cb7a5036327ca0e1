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

from crdtgpu.abi import CAWSetBatch, CAWSetOut, CSrcBatch  # noqa: E402
from crdtgpu.batch import AWSetBatch, OutBuffers, SrcBatch  # noqa: E402

LIB = os.path.join(HERE, "build", "liboracle.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", HERE, "build/liboracle.so"])
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


def causal_context(vv: np.ndarray, n_docs: int, R: int) -> np.ndarray:
    vv = np.ascontiguousarray(vv, dtype=np.uint64)
    out = np.zeros(R, dtype=np.uint64)
    lib().oracle_causal_context(vv.ctypes.data, n_docs, R, out.ctypes.data)
    return out
