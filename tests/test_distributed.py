"""World-size-2 gloo tests of the multi-GPU plumbing (fqlpop/distributed.py):
member sharding, dataset broadcast, score gathering for halving decisions and
the max-over-ranks timer, all on CPU tensors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "flow-q-learning_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fqlpop import distributed as D
    from bench import population_values
    from hpo.successive_halving import SuccessiveHalving
    from trainer.config import ExperimentConfig

    alphas, seeds = population_values(16 * world)
    mine = D.shard(list(zip(alphas, seeds)), rank, world)
    rng = np.random.default_rng(0)
    data = None
    shapes = {"observations": (100, 28), "actions": (100, 5), "rewards": (100,), "masks": (100,),
              "next_observations": (100, 28)}
    if rank == 0:
        data = {k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()}
    got = D.broadcast_dataset(data, shapes, torch.device("cpu"))
    checksum = float(sum(t.double().sum() for t in got.values()))
    # each rank scores its own members; every rank must reach the same halving decision
    configs = [ExperimentConfig(seed=s, alpha=a) for a, s in zip(alphas, seeds)]
    local = {c: (c.seed % 97) / 97.0 for c in D.shard(configs, rank, world)}
    scores = D.gather_scores(local)
    sh = SuccessiveHalving(set(configs), total_evaluations=8, fraction=0.5, history_length=1)
    for c, v in scores.items():
        sh.update(c, v)
    sh.performed_evaluations = sh.halving_milestones[0]
    kept = sorted(c.seed for c in sh.sample())
    tmax = D.max_over_ranks(1.0 + rank)
    q.put((rank, [m[1] for m in mine], checksum, kept, tmax, len(scores)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world_size_2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, m0, c0, k0, t0, n0), (r1, m1, c1, k1, t1, n1) = out
    assert set(m0).isdisjoint(m1) and len(m0) == len(m1) == 16
    assert c0 == c1                # identical broadcast dataset
    assert k0 == k1 and len(k0) == 16  # same halving decision on both ranks (32 -> 16)
    assert t0 == t1 == 2.0 and n0 == n1 == 32


def _cfgs(n):
    from trainer.config import ExperimentConfig
    return [ExperimentConfig(seed=1000 + i, alpha=float(3 + 7 * (i % 5))) for i in range(n)]


def test_owner_assignment_and_rebalance_plan():
    """Owners are dealt round-robin over the ordered candidates; after any pruning the
    plan evens the shards (max - min <= 1) with the fewest moves, identically on
    every rank (a pure function of the configs)."""
    import itertools
    import random as pyrandom
    from fqlpop import distributed as D
    for n, world in itertools.product((1, 5, 16, 64), (1, 2, 3, 8)):
        cfgs = _cfgs(n)
        owner = D.assign_owners(cfgs, world)
        counts = [sum(1 for c in cfgs if owner[c] == r) for r in range(world)]
        assert max(counts) - min(counts) <= 1 and max(counts) == D.shard_capacity(n, world)
        assert D.assign_owners(list(reversed(cfgs)), world) == owner  # order-independent
        rng = pyrandom.Random(n * 31 + world)
        for _ in range(5):
            live = rng.sample(cfgs, rng.randint(1, n))
            own = dict(owner)
            moves = D.rebalance_plan(live, own, world)
            assert moves == D.rebalance_plan(list(reversed(live)), dict(owner), world)
            before = [sum(1 for c in live if own[c] == r) for r in range(world)]
            for c, src, dst in moves:
                assert own[c] == src and src != dst
                own[c] = dst
            after = [sum(1 for c in live if own[c] == r) for r in range(world)]
            assert max(after) - min(after) <= 1 and max(after) <= D.shard_capacity(n, world)
            # fewest moves: every member above the balanced share moves once, no more
            share = -(-len(live) // world)
            assert len(moves) <= sum(max(0, b - share) for b in before) + world
            assert len({c for c, _, _ in moves}) == len(moves)


def test_eval_round_seed_depends_on_seed_and_round_only():
    from fqlpop import distributed as D
    s = [D.eval_round_seed(0, r) for r in range(8)]
    assert len(set(s)) == 8 and s == [D.eval_round_seed(0, r) for r in range(8)]
    assert D.eval_round_seed(1, 0) != s[0]
    assert all(0 <= v < 2**31 - 1 for v in s)


def _move_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "flow-q-learning_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fqlpop import distributed as D
    cfgs = _cfgs(6)
    owner = D.assign_owners(cfgs, world)
    # rank 1 keeps all of its 3, rank 0 loses 2: one move from rank 1 to rank 0
    live = [c for c in D.ordered(cfgs) if owner[c] == 1] + [D.ordered(cfgs)[0]]
    got = {}
    for c, src, dst in D.rebalance_plan(live, owner, world):
        if rank == src:
            D.send_object({"cfg": c, "params": np.full(1000, src, np.float32), "step": 7}, dst)
        elif rank == dst:
            got[c] = D.recv_object(src)
    seed = D.broadcast_object(12345 if rank == 0 else None)
    parts = D.gather_objects({rank: sorted(str(c) for c in got)}, dst=0)
    q.put((rank, {str(c): (float(v["params"].sum()), v["step"], v["cfg"] == c) for c, v in got.items()}, seed,
           parts))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_member_move_and_object_collectives():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_move_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got0, seed0, parts0 = out[0]
    got1, seed1, parts1 = out[1]
    assert seed0 == seed1 == 12345
    assert len(got0) == 1 and not got1
    (s, step, same), = got0.values()
    assert s == 1000.0 and step == 7 and same   # the state rank 1 sent
    assert parts1 is None and len(parts0) == 2
