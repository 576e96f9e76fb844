"""Multi-GPU plumbing: one process per GPU, independent QP shards.

Every QP is independent, so the data path has no collective: rank r owns global
indices [r*B, (r+1)*B) and generates them locally from (seed, global index).
Collectives are used only for the benchmark bookkeeping (barrier, max of the
timed region, status counts) and, optionally, to gather GRFs to rank 0 with
point-to-point sends (one direct xGMI link per sender) when a single consumer
needs the whole batch.
"""
from __future__ import annotations

import os


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(rank: int, world: int, per_rank: int):
    """Global index range owned by `rank` (weak scaling: per_rank QPs each)."""
    first = rank * per_rank
    return first, first + per_rank


def split_range(rank: int, world: int, total: int):
    """Global index range owned by `rank` when a fixed total is split (strong scaling)."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def max_over_ranks(value: float, dist, device=None) -> float:
    import torch

    if dist is None:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, dist, device=None):
    import torch

    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(t)
    return [float(v) for v in t.tolist()]


def gather_to_rank0(tensor, dist, world: int, rank: int, counts=None):
    """Gather per-rank result tensors (leading dim = that rank's QP count) to rank 0.

    One grouped point-to-point exchange (batch_isend_irecv = ncclGroupStart / ncclSend x
    (N-1) / ncclRecv x (N-1) / ncclGroupEnd on RCCL): every sender uses its own direct xGMI
    link to rank 0, nothing is relayed around a ring.  `counts[r]` = rows
    owned by rank r (default: all equal).  Returns the concatenation on rank 0, None elsewhere.
    """
    import torch

    if dist is None or world == 1:
        return tensor
    if counts is None:
        counts = [tensor.shape[0]] * world
    if rank == 0:
        bufs = [tensor] + [torch.empty((counts[src],) + tuple(tensor.shape[1:]), dtype=tensor.dtype,
                                       device=tensor.device) for src in range(1, world)]
        ops = [dist.P2POp(dist.irecv, bufs[src], src) for src in range(1, world)]
    else:
        ops = [dist.P2POp(dist.isend, tensor, 0)]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    return torch.cat(bufs, dim=0) if rank == 0 else None
