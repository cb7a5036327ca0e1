"""Multi-GPU plumbing: documents shard across ranks with no data-path
exchange; the only collective is the global causal-context summary -- the
elementwise u64 max of every rank's per-GPU summary (crdt_causal_context_async)
-- all-reduced over torch.distributed (RCCL on ROCm, gloo on CPU for tests).
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
