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
