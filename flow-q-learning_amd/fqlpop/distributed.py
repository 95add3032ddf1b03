"""Multi-GPU plumbing for the population (one process per GPU, torch.distributed).

The alpha-population is embarrassingly parallel: members are
sharded across ranks with NO collective in the update itself.  RCCL (the
"nccl" backend on ROCm, over xGMI) is used only to
  * broadcast the shared offline dataset from rank 0 once (``broadcast_dataset``),
  * gather evaluation scores so every rank takes the same halving decision
    (``gather_scores``),
  * reduce the timed region's wall time to its max over ranks (``max_over_ranks``).
The same functions run on the gloo backend with CPU tensors (tests).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

DATA_KEYS = ("observations", "actions", "rewards", "masks", "next_observations")


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard(items, rank: int, world_size: int):
    """Round-robin assignment of population members to ranks (member i -> rank i % W)."""
    return list(items)[rank::world_size]


def broadcast_dataset(data: dict | None, shapes: dict, device: torch.device, src: int = 0) -> dict:
    """Rank ``src`` holds ``data`` (numpy arrays); every rank returns torch tensors
    on ``device`` with the same contents (one broadcast per field)."""
    rank, ws = world()
    out = {}
    for k in DATA_KEYS:
        if rank == src:
            t = torch.from_numpy(np.ascontiguousarray(data[k], dtype=np.float32)).to(device)
        else:
            t = torch.empty(shapes[k], dtype=torch.float32, device=device)
        if ws > 1:
            dist.broadcast(t, src=src)
        out[k] = t
    return out


def gather_scores(local: dict) -> dict:
    """Union of every rank's {candidate: score} (all_gather_object)."""
    rank, ws = world()
    if ws == 1:
        return dict(local)
    parts = [None] * ws
    dist.all_gather_object(parts, dict(local))
    merged = {}
    for p in parts:
        merged.update(p)
    return merged


def max_over_ranks(value: float, device: torch.device | None = None) -> float:
    rank, ws = world()
    if ws == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
