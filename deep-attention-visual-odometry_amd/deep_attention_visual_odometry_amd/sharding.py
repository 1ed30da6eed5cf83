"""Multi-GPU data parallelism for batches of independent BA problems.

SURVEY.md 8(e): problems share nothing, so a global batch is cut into
contiguous per-rank slabs, each rank solves its slab on its own GPU with no
communication, and ONE all-gather (RCCL over xGMI with the "nccl" backend)
assembles the converged parameters (and the per-problem status words) on
every rank.  Inputs are never scattered: each rank generates or loads only its
own slab (``make_scenes(..., first_index=shard.start)``).
"""
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class Shard:
    start: int
    stop: int

    @property
    def size(self) -> int:
        return self.stop - self.start


def shard_range(global_batch: int, world_size: int, rank: int) -> Shard:
    """Contiguous slab of rank ``rank``; the first ``global_batch % world_size`` ranks get one extra."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    base, extra = divmod(global_batch, world_size)
    start = rank * base + min(rank, extra)
    return Shard(start, start + base + (1 if rank < extra else 0))


def gather_rows(local: torch.Tensor, global_batch: int, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """All-gather per-rank row slabs (possibly of unequal size) into the (global_batch, ...) tensor,
    in global problem order.  One collective when the slabs are equal (the benchmark case)."""
    world = dist.get_world_size(group)
    sizes = [shard_range(global_batch, world, r).size for r in range(world)]
    width = max(sizes)
    if local.shape[0] != sizes[dist.get_rank(group)]:
        raise ValueError("local slab size does not match shard_range")
    if all(s == width for s in sizes):
        out = torch.empty((global_batch,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    padded = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    padded[: local.shape[0]] = local
    buf = torch.empty((world * width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(buf, padded, group=group)
    return torch.cat([buf[r * width: r * width + sizes[r]] for r in range(world)])


def gather_packed(x: torch.Tensor, status: torch.Tensor, global_batch: int,
                  group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """ONE all-gather for a solve's outputs: x (n, P) float32 and status (n, S) int32 travel
    as one (n, P + S) float32 buffer (status bit-cast, not converted), split again after."""
    if x.dtype != torch.float32 or status.dtype != torch.int32:
        raise TypeError("gather_packed expects float32 parameters and int32 status words")
    p = x.shape[-1]
    packed = torch.cat([x.reshape(x.shape[0], p), status.reshape(status.shape[0], -1).view(torch.float32)], dim=1)
    out = gather_rows(packed, global_batch, group)
    return out[:, :p].contiguous(), out[:, p:].contiguous().view(torch.int32)


def solve_sharded(solve_slab: Callable[[Shard], Tuple[torch.Tensor, torch.Tensor]], global_batch: int,
                  group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Run ``solve_slab(shard) -> (x (n, P), status (n, 4))`` on this rank's slab, then all-gather
    both in one collective (float32 parameters) or two (other dtypes)."""
    shard = shard_range(global_batch, dist.get_world_size(group), dist.get_rank(group))
    x, status = solve_slab(shard)
    if x.dtype == torch.float32 and status.dtype == torch.int32:
        return gather_packed(x, status, global_batch, group)
    return gather_rows(x, global_batch, group), gather_rows(status, global_batch, group)
