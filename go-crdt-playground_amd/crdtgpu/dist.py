"""Multi-GPU plumbing: documents shard across ranks with no data-path
exchange; the only collective is the global causal-context summary -- the
elementwise u64 max of every rank's per-GPU summary (crdt_causal_context_async).

Two transports for it:
  * the engine's own RCCL communicator, the C-ABI path a Go/C caller binds
    (crdt_comm_unique_id on rank 0, the id shared once over torch.distributed,
    crdt_comm_init on every rank, then crdt_context_allreduce_async per step):
    engine_comm_handshake();
  * torch.distributed itself (u64_max_allreduce), for host-side (gloo) runs.
"""

from __future__ import annotations

SIGN = -(1 << 63)


def u64_max_allreduce(dist, t, group=None):
    """all_reduce(MAX) of u64 values held in an int64 tensor.

    torch.distributed has no unsigned 64-bit MAX, so the sign bit is flipped
    (x ^ 2^63 maps u64 order onto int64 order), reduced as int64, and flipped
    back: exact for every u64."""
    import torch

    flip = torch.tensor(SIGN, dtype=torch.int64, device=t.device)
    x = t ^ flip
    dist.all_reduce(x, op=dist.ReduceOp.MAX, group=group)
    return x ^ flip


def shard(n_docs_total: int, world: int, rank: int):
    """Contiguous document range [lo, hi) of `rank` (balanced to within one doc)."""
    base, extra = divmod(n_docs_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def engine_comm_handshake(dist, world: int, rank: int, init, make_id=None) -> bytes:
    """Set up the engine's own RCCL communicator across the ranks of `dist`.

    Rank 0 makes the communicator id (crdt_comm_unique_id), the id travels to
    every rank over torch.distributed once (an object broadcast: any backend,
    gloo included), and every rank then calls init(world, rank, id) --
    Engine.comm_init, i.e. crdt_comm_init.  Returns the id."""
    if make_id is None:
        from .engine import comm_unique_id as make_id
    box = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    uid = bytes(box[0])
    init(world, rank, uid)
    return uid
