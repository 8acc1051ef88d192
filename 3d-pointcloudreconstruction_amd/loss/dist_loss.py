"""Batch-sharded Chamfer/EMD loss over several GPUs (one process per GPU).

The reference is single-GPU (train.py:5); SURVEY.md section 8e adds exactly
one exchange: every rank evaluates the hot path on its own shard of the batch
(no halo, no data-path collective) and ONE all-reduce of the loss partial sums
(a few bytes, RCCL over xGMI with the "nccl" backend) makes the global value.

``global_chamfer_loss`` returns a scalar whose VALUE is the loss of the whole
global batch and whose GRADIENT w.r.t. the local predictions is that of the
global loss (each local distance weighted 1/(global count)).  Under DDP, whose
gradient all-reduce averages over ranks, use ``local=True`` instead (the
per-rank mean), which yields the same averaged gradient with equal shards.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int):
    """Contiguous near-equal [start, stop) slice of `total` items for `rank`."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _reduce(t: torch.Tensor, group=None) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def global_chamfer_loss(dist1: torch.Tensor, dist2: torch.Tensor, group=None, local: bool = False):
    """mean(dist1) + mean(dist2) over the GLOBAL batch (loss/loss.py:36)."""
    sums = torch.stack([dist1.sum(), dist2.sum()])
    counts = torch.tensor([dist1.numel(), dist2.numel()], dtype=sums.dtype, device=sums.device)
    if local:
        return sums[0] / counts[0] + sums[1] / counts[1]
    packed = _reduce(torch.cat([sums.detach(), counts]), group)
    g_sums, g_counts = packed[:2], packed[2:]
    differentiable = sums[0] / g_counts[0] + sums[1] / g_counts[1]
    value = g_sums[0] / g_counts[0] + g_sums[1] / g_counts[1]
    return differentiable + (value - differentiable).detach()


def global_emd_loss(dist: torch.Tensor, group=None, local: bool = False):
    """mean over points and batch of sqrt(dist) (loss/loss.py:25) over the GLOBAL batch."""
    s = torch.sqrt(dist)
    rows = s.mean(1)
    if local:
        return rows.mean()
    packed = _reduce(torch.stack([rows.sum().detach(),
                                  torch.tensor(float(rows.numel()), device=s.device)]), group)
    differentiable = rows.sum() / packed[1]
    value = packed[0] / packed[1]
    return differentiable + (value - differentiable).detach()
