"""ctypes mirror of include/crdtgpu.h and the loader of libcrdtgpu.so.

The library is the product: there is no fallback.  If it is missing or fails
to load, importing this module raises -- a GPU box must never silently run a
CPU path.
"""

from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# CRDTGPU_LIB: a diagnostic build of the same library (tools/libcrdtgpu_stamps.so)
LIB_PATH = os.environ.get("CRDTGPU_LIB") or os.path.join(HERE, "libcrdtgpu.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "crdtgpu.h")

CRDT_OK = 0
CRDT_E_INVALID = -1
CRDT_E_ACTOR_RANGE = -2
CRDT_E_UNSORTED = -3
CRDT_E_CAPACITY = -4
CRDT_E_HIP = -5
CRDT_E_NOMEM = -6
CRDT_E_WORKSPACE = -7
CRDT_E_RCCL = -8
CRDT_E_DUP_KEY = -9
CRDT_COMM_ID_BYTES = 128
CRDT_MAX_R = 64
CRDT_FOLD_AWSET = 0
CRDT_FOLD_DELTA = 1
CRDT_OP_ADD = 0
CRDT_OP_DEL = 1
CRDT_OP_DELTA_DEL = 2
CRDT_OP_DELTA_DEL_KEY = 3
CRDT_MAX_OPS_PER_DOC = 256
CRDT_PROBE_READ = 0
CRDT_PROBE_WRITE = 1
CRDT_PROBE_COPY = 2
CRDT_PROBE_WRITE_PLAIN = 3
CRDT_PROBE_COPY_PLAIN = 4
CRDT_PROBE_MIX = 5
CRDT_PROBE_MIX_PLAIN = 6

_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64


class CAWSetBatch(ctypes.Structure):
    _fields_ = [
        ("n_docs", _u32), ("R", _u32),
        ("offsets", _vp), ("counts", _vp), ("keys", _vp), ("actors", _vp), ("counters", _vp), ("vv", _vp),
    ]


class CAWSetOut(ctypes.Structure):
    _fields_ = [("offsets", _vp), ("counts", _vp), ("keys", _vp), ("actors", _vp), ("counters", _vp), ("vv", _vp)]


class CSrcBatch(ctypes.Structure):
    _fields_ = [
        ("n_docs", _u32), ("R", _u32),
        ("doc_srcs", _vp), ("src_actor", _vp), ("vv", _vp), ("entry_off", _vp),
        ("keys", _vp), ("actors", _vp), ("counters", _vp),
        ("tomb_off", _vp), ("tkeys", _vp), ("tactors", _vp), ("tcounters", _vp),
    ]


class COpBatch(ctypes.Structure):
    _fields_ = [("n_docs", _u32), ("op_off", _vp), ("kind", _vp), ("keys", _vp), ("doc_actor", _vp)]


class CTombBatch(ctypes.Structure):
    _fields_ = [("offsets", _vp), ("counts", _vp), ("keys", _vp), ("actors", _vp), ("counters", _vp)]


class CTombOut(ctypes.Structure):
    _fields_ = [("offsets", _vp), ("counts", _vp), ("keys", _vp), ("actors", _vp), ("counters", _vp)]


class CrdtError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = "%s (code %d)" % (strerror(code) if _lib is not None else "crdtgpu error", code)
        super().__init__(what + ": " + msg if what else msg)


def header_functions(path: str = HEADER_PATH):
    """Names of the functions include/crdtgpu.h declares."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(crdt_\w+)\s*\(", text, flags=re.M)))


def hip_runtimes_mapped():
    """Distinct libamdhip64 files mapped into this process."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    out.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return sorted(out)


def _load():
    # PyTorch (the host's device-memory / stream / RCCL plumbing) bundles its
    # own HIP runtime with the same soname (libamdhip64.so.7).  Loading torch
    # first makes our NEEDED entry bind to that already-loaded runtime, so torch
    # streams and allocations are native handles for this library; loading us
    # first would put two HIP/HSA runtimes in one process.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("libcrdtgpu.so not built at %s: run `python -c 'import __graft_entry__ as g; g.build()'`"
                          % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    rts = hip_runtimes_mapped()
    if len(rts) > 1:
        raise ImportError("two HIP runtimes mapped into one process: %s" % rts)
    for name, (res, args) in signatures().items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def signatures():
    """name -> (restype, argtypes) of every entry point the package binds
    (include/crdtgpu.h; tests/test_abi.py checks the argument counts)."""
    P = ctypes.POINTER
    return {
        "crdt_abi_version": (ctypes.c_int, []),
        "crdt_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "crdt_ctx_create": (ctypes.c_int, [ctypes.c_int, P(_vp)]),
        "crdt_ctx_destroy": (None, [_vp]),
        "crdt_ctx_reserve": (ctypes.c_int, [_vp, _u32, _u64]),
        "crdt_ctx_sync": (ctypes.c_int, [_vp, _vp]),
        "crdt_ctx_set_max_doc_entries": (ctypes.c_int, [_vp, _u32]),
        "crdt_ctx_set_option": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int64]),
        "crdt_awset_join_async": (ctypes.c_int, [_vp, P(CAWSetBatch), P(CAWSetBatch), P(CAWSetOut), _vp]),
        "crdt_awset_exchange_async": (ctypes.c_int, [_vp, P(CAWSetBatch), P(CAWSetBatch), P(CAWSetOut),
                                                     P(CAWSetOut), _vp]),
        "crdt_awset_exchange_batch": (ctypes.c_int, [_vp, P(CAWSetBatch), P(CAWSetBatch), P(CAWSetOut), P(CAWSetOut)]),
        "crdt_awset_fold_async": (ctypes.c_int, [_vp, ctypes.c_int, P(CAWSetBatch), P(CSrcBatch), P(CAWSetOut), _vp]),
        "crdt_vv_max_async": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_size_t, _vp]),
        "crdt_causal_context_async": (ctypes.c_int, [_vp, _vp, _u32, _u32, _vp, _vp]),
        "crdt_gen_pair_async": (ctypes.c_int, [_vp, _u64, _u32, P(CAWSetOut), P(CAWSetOut), _vp]),
        "crdt_gen_delta_async": (ctypes.c_int, [_vp, _u64, _u32, _u32, _u32, P(CAWSetOut), P(CSrcBatch), _vp]),
        "crdt_gen_zipf_sizes": (ctypes.c_int, [_u64, _u32, _vp]),
        "crdt_gen_zipf_async": (ctypes.c_int, [_vp, _u64, _u32, _vp, P(CAWSetOut), P(CAWSetOut), _vp]),
        "crdt_gen_replicas_async": (ctypes.c_int, [_vp, _u64, _u32, _u32, _u32, P(CAWSetOut), P(CSrcBatch), _vp]),
        "crdt_awset_join_batch": (ctypes.c_int, [_vp, P(CAWSetBatch), P(CAWSetBatch), P(CAWSetOut)]),
        "crdt_awset_fold_batch": (ctypes.c_int, [_vp, ctypes.c_int, P(CAWSetBatch), P(CSrcBatch), P(CAWSetOut)]),
        "crdt_bw_probe": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, ctypes.c_size_t, ctypes.c_int,
                                         P(ctypes.c_double)]),
        "crdt_host_alloc": (ctypes.c_int, [ctypes.c_size_t, P(_vp)]),
        "crdt_host_free": (None, [_vp]),
        "crdt_clock_probe": (ctypes.c_int, [_vp, P(ctypes.c_double)]),
        "crdt_validate_batch": (ctypes.c_int, [P(CAWSetBatch)]),
        "crdt_validate_src_batch": (ctypes.c_int, [P(CSrcBatch)]),
        "crdt_validate_tomb_batch": (ctypes.c_int, [P(CTombBatch), _u32]),
        "crdt_awset_apply_async": (ctypes.c_int, [_vp, P(CAWSetBatch), P(CTombBatch), P(COpBatch), P(CAWSetOut),
                                                  P(CTombOut), _vp]),
        "crdt_awset_apply_batch": (ctypes.c_int, [_vp, P(CAWSetBatch), P(CTombBatch), P(COpBatch), P(CAWSetOut),
                                                  P(CTombOut)]),
        "crdt_awset_sort_async": (ctypes.c_int, [_vp, P(CAWSetBatch), _u32, P(CAWSetOut), _vp]),
        "crdt_awset_sort_batch": (ctypes.c_int, [_vp, P(CAWSetBatch), P(CAWSetOut)]),
        "crdt_tombstone_gc_async": (ctypes.c_int, [_vp, P(CTombBatch), _u32, _u32, _vp, P(CTombOut), _vp]),
        "crdt_vv_min_async": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_size_t, _vp]),
        "crdt_awset_format": (ctypes.c_int, [P(CAWSetBatch), _u32, _vp, _vp, ctypes.c_size_t,
                                             P(ctypes.c_size_t)]),
        "crdt_batch_dump": (ctypes.c_int, [P(CAWSetBatch), _vp, ctypes.c_size_t, P(ctypes.c_size_t)]),
        "crdt_batch_info": (ctypes.c_int, [_vp, ctypes.c_size_t, P(_u32), P(_u32), P(_u64)]),
        "crdt_batch_undump": (ctypes.c_int, [_vp, ctypes.c_size_t, P(CAWSetOut)]),
        "crdt_global_context_allreduce": (ctypes.c_int, [P(_vp), ctypes.c_int, P(_vp), _u32, _vp]),
        "crdt_comm_unique_id": (ctypes.c_int, [_vp]),
        "crdt_comm_init": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp]),
        "crdt_context_allreduce_async": (ctypes.c_int, [_vp, _vp, _u32, _vp]),
    }


_lib = None
_lib = _load()


def lib():
    return _lib


def strerror(code: int) -> str:
    return _lib.crdt_strerror(code).decode()


def check(code: int, what: str = "") -> None:
    if code != CRDT_OK:
        raise CrdtError(code, what)
