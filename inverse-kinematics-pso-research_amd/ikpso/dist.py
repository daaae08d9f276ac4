"""Multi-GPU sharding of a batch of independent swarms.

One process per GPU.  Swarms are independent, so a batch shards by contiguous
swarm ranges with no data-path collective; generator seeds are derived from
the GLOBAL swarm index, so every swarm's result is identical whatever the
world size.  The only exchange is one all-gather of the per-swarm results
(D angles + fitness + residual) at the end, over RCCL ("nccl" backend) on the
GPUs or gloo on the CPU.
"""
from __future__ import annotations

from typing import Tuple


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """[first, first + count) of `total` swarms for `rank` of `world`;
    the first total % world ranks get one extra swarm."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(int(total), int(world))
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def pack_results(angles, fitness, residual):
    """[B, D+2] rows: angles, fitness, residual -- one contiguous payload."""
    import torch

    cols = [angles, fitness[:, None]]
    cols.append(residual[:, None] if residual is not None else torch.zeros_like(fitness)[:, None])
    return torch.cat(cols, dim=1).contiguous()


def gather_rows(local, total: int, world: int, group=None, force: bool = False):
    """All-gather per-rank row blocks (possibly uneven) into [total, cols] on every rank.
    With one rank the rows are returned as they are, unless `force` (tests: drive
    the collective through a world-1 process group)."""
    import torch
    import torch.distributed as dist

    if world == 1 and not force:
        return local
    cols = local.shape[1]
    counts = [shard_range(total, world, r)[1] for r in range(world)]
    cap = max(counts)
    buf = torch.zeros((cap, cols), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    if dist.get_backend(group) == "gloo":  # host tensors (CPU runs, or a GPU rehearsal over gloo)
        host = buf.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        out = torch.cat(parts, dim=0).to(local.device)
    else:
        out = torch.empty((cap * world, cols), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, buf, group=group)
    return torch.cat([out[r * cap: r * cap + counts[r]] for r in range(world)], dim=0)
