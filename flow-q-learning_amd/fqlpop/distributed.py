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
    # gloo (ranks sharing a device, CPU tests) moves host tensors; RCCL moves device tensors
    stage = torch.device("cpu") if ws > 1 and dist.get_backend() == "gloo" else device
    out = {}
    for k in DATA_KEYS:
        if rank == src:
            t = torch.from_numpy(np.ascontiguousarray(data[k], dtype=np.float32)).to(stage)
        else:
            t = torch.empty(shapes[k], dtype=torch.float32, device=stage)
        if ws > 1:
            dist.broadcast(t, src=src)
        out[k] = t.to(device)
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


# ------------------------------------------------------------------ halving
# A population sharded over ranks (BASELINE configs 4 and 5): every
# rank holds the same HPO strategy and takes the same decisions from the gathered
# scores, trains only the members it owns, and hands members to other ranks when
# pruning leaves the shards uneven.  Everything below is a pure function of the
# (identical) strategy state, so all ranks compute the same owners and moves
# without exchanging them.

def config_key(cfg):
    """Total order on ExperimentConfig-like records (alpha, then seed; None first),
    the order every rank iterates candidates in."""
    def k(v):
        return (0, 0.0) if v is None else (1, float(v))
    return (k(getattr(cfg, "alpha", None)), k(getattr(cfg, "seed", None)))


def ordered(configs):
    return sorted(configs, key=config_key)


def assign_owners(configs, world_size: int) -> dict:
    """Round-robin over the ordered candidates: config -> rank."""
    return {c: i % world_size for i, c in enumerate(ordered(configs))}


def shard_capacity(n_configs: int, world_size: int) -> int:
    """Population slots a rank needs: its initial share, which pruning and
    rebalancing never exceed."""
    return max(1, -(-n_configs // world_size))


def rebalance_plan(live, owner: dict, world_size: int) -> list:
    """Moves (config, src, dst) that even out the live members per rank (max - min
    <= 1), moving the fewest members: while uneven, the last live config (in
    ``ordered`` order) of the most loaded rank goes to the least loaded one (lowest
    rank id on ties)."""
    shards = {r: [c for c in ordered(live) if owner[c] == r] for r in range(world_size)}
    moves = []
    while True:
        hi = max(range(world_size), key=lambda r: (len(shards[r]), -r))
        lo = min(range(world_size), key=lambda r: (len(shards[r]), r))
        if len(shards[hi]) - len(shards[lo]) <= 1:
            return moves
        c = shards[hi].pop()
        shards[lo].append(c)
        moves.append((c, hi, lo))


def place_new(new_configs, live, owner: dict, world_size: int) -> dict:
    """Owners for configs a strategy adds: each goes to the currently least loaded rank."""
    load = {r: sum(1 for c in live if owner.get(c) == r) for r in range(world_size)}
    out = {}
    for c in ordered(new_configs):
        r = min(range(world_size), key=lambda q: (load[q], q))
        out[c] = r
        load[r] += 1
    return out


def broadcast_object(obj, src: int = 0):
    """``obj`` of rank ``src`` on every rank."""
    rank, ws = world()
    if ws == 1:
        return obj
    box = [obj if rank == src else None]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def send_object(obj, dst: int) -> None:
    dist.send_object_list([obj], dst=dst)


def recv_object(src: int):
    box = [None]
    dist.recv_object_list(box, src=src)
    return box[0]


def gather_objects(obj, dst: int = 0):
    """List of every rank's ``obj`` on rank ``dst`` (None elsewhere)."""
    rank, ws = world()
    if ws == 1:
        return [obj]
    out = [None] * ws if rank == dst else None
    dist.gather_object(obj, out, dst=dst)
    return out


def eval_round_seed(base_seed: int, round_index: int) -> int:
    """Seed of the world-model evaluation of round ``round_index``: a function of
    the run seed and the round only, so a member's scores do not depend on the
    sharding or the world size (Trainer and DistributedTrainer alike)."""
    return int(np.random.default_rng([int(base_seed) & 0xFFFFFFFF, int(round_index)]).integers(0, 2**31 - 1))


def member_eval_seed(base_seed: int, round_index: int, cfg) -> int:
    """Seed of one candidate's own evaluation in round ``round_index`` (tasks without
    a batched world-model evaluation): a function of the run seed, the round and the
    candidate's (alpha, seed), so it does not depend on which rank owns the member."""
    (fa, a), (fs, s) = config_key(cfg)
    a_bits = int(np.array([a], dtype=np.float64).view(np.uint64)[0])
    words = [int(base_seed) & 0xFFFFFFFF, int(round_index), fa, a_bits & 0xFFFFFFFF, a_bits >> 32, fs,
             int(s) & 0xFFFFFFFF]
    return int(np.random.default_rng(words).integers(0, 2**31 - 1))
