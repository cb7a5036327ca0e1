"""crdtgpu -- MI355X batched AWSet / AWSetDelta merge engine (Python host side).

Everything here drives libcrdtgpu.so (HIP kernels for gfx950 behind the C ABI
of include/crdtgpu.h).  Importing fails loudly when the library is missing.
"""

from .abi import (CRDT_E_ACTOR_RANGE, CRDT_E_CAPACITY, CRDT_E_DUP_KEY, CRDT_E_HIP, CRDT_E_INVALID, CRDT_E_NOMEM,  # noqa: F401
                  CRDT_E_RCCL, CRDT_E_UNSORTED, CRDT_E_WORKSPACE, CRDT_FOLD_AWSET, CRDT_FOLD_DELTA, CRDT_MAX_OPS_PER_DOC, CRDT_MAX_R, CRDT_OK,
                  CRDT_OP_ADD, CRDT_OP_DEL, CRDT_OP_DELTA_DEL, CRDT_OP_DELTA_DEL_KEY,
                  CrdtError, LIB_PATH, header_functions, lib, strerror)
from .batch import AWSetBatch, OpBatch, OutBuffers, SrcBatch, SrcBuffers, TombBatch, TombBuffers  # noqa: F401
from .engine import (Engine, comm_unique_id, dump_batch, format_doc, global_context_allreduce,  # noqa: F401
                     load_batch, validate, validate_src)
