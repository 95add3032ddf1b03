"""The sharded population trainer (trainer/distributed_trainer.py) on the GPU:
two ranks (gloo for the collectives, both processes on cuda:0 -- this box has
one GPU) against one rank.  Every member's scores, the strategy's decisions and
every surviving member's parameters must be bit-identical, with and without a
member moving between ranks after pruning."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
H = 512  # the rollout evaluator is built for the 512-wide actor


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank, world, port, save_dir, strategy_kind, plain=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "flow-q-learning_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from fqlpop import distributed as D
    from hpo.strategy import HpoStrategy
    from hpo.successive_halving import SuccessiveHalving
    from task.offline_task_simulated import OfflineTaskWithSimulatedEvaluations
    from trainer.config import AgentConfig, ExperimentConfig, TrainerConfig
    from trainer.distributed_trainer import DistributedTrainer
    from trainer.trainer import Trainer

    class KeepEven(HpoStrategy):
        """After two evaluations keep the candidates at even positions of the
        ordered list: on 2 ranks all of them start on rank 0, so one must move."""
        def __init__(self, population):
            super().__init__(population, 0)
            self.n_eval = {}

        def update(self, candidate, performance):
            self.n_eval[candidate] = self.n_eval.get(candidate, 0) + 1

        def sample(self):
            if self.n_eval and min(self.n_eval.values()) >= 2:
                self.population = set(D.ordered(self.population)[0::2][:3])
            return self.population

    class DropAndRevive(HpoStrategy):
        """After the first evaluation keep the candidates at even positions of the ordered
        list (on 2 ranks: rank 1 retires all of its members, rank 0 gives one survivor to
        rank 1), after the second bring every candidate back: a retired member resumes on
        the rank that holds its state, or is sent to the rank place_new picks."""
        def __init__(self, population):
            super().__init__(population, 0)
            self.all = set(population)
            self.n_eval = {}

        def update(self, candidate, performance):
            self.n_eval[candidate] = self.n_eval.get(candidate, 0) + 1

        def sample(self):
            rounds = max(self.n_eval.values()) if self.n_eval else 0
            self.population = set(D.ordered(self.all)[0::2]) if rounds == 1 else set(self.all)
            return self.population

    task = OfflineTaskWithSimulatedEvaluations(n_rows=20_000, n_val_rows=2_000, num_evaluation_envs=16,
                                               max_episode_steps=25)
    agent = AgentConfig(actor_hidden_dims=(H,) * 4, value_hidden_dims=(H,) * 4, batch_size=64)
    cfg = TrainerConfig(agent=agent, steps=40, eval_interval=10, log_interval=10, save_directory=save_dir)
    configs = {ExperimentConfig(alpha=a, seed=s) for a, s in [(3.0, 1), (10.0, 2), (30.0, 3), (100.0, 4),
                                                               (300.0, 5), (1000.0, 6)]}
    if strategy_kind == "halving":
        strategy = SuccessiveHalving(configs, total_evaluations=12, fraction=0.5, history_length=1)
    elif strategy_kind == "revive":
        strategy = DropAndRevive(configs)
    else:
        strategy = KeepEven(configs)
    tr = Trainer(task, strategy, cfg) if plain else DistributedTrainer(task, strategy, cfg)
    tr.train(max_evaluations=100)
    state = tr.state_dict()
    from fql.utils.serialization import params_of
    live = {c: e for c, e in tr.experiments.items() if c in tr.candidates}  # Trainer keeps stopped ones too
    params = {str(c): np.concatenate([v.ravel() for net in params_of(e.agent.to_state_dict()).values()
                                      for v in net.values()]) for c, e in live.items()}
    steps = {str(c): e.current_step for c, e in live.items()}
    scores = {str(c): list(v) for c, v in getattr(strategy, "candidate_scores", {}).items()}
    out = dict(rank=rank, candidates=sorted(str(c) for c in tr.candidates), params=params, steps=steps,
               scores=scores, n_state=None if state is None else len(state["experiments"]),
               owners={str(c): r for c, r in getattr(tr, "owner", {}).items() if c in tr.candidates})
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return out


def _worker(rank, world, port, save_dir, kind, q):
    try:
        q.put(_run(rank, world, port, save_dir, kind))
    except BaseException as e:  # report instead of hanging the parent
        q.put(dict(rank=rank, error=repr(e)))
        raise


def _two_ranks(tmp_path, kind):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path / "w2"), kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for o in outs:
        assert "error" not in o, o
    assert all(p.exitcode == 0 for p in procs)
    return sorted(outs, key=lambda o: o["rank"])


@pytest.mark.parametrize("kind", ["halving", "keep_even", "revive"])
def test_two_ranks_match_one_rank(tmp_path, kind):
    """The baseline is the plain single-process Trainer (what tune_alpha runs at
    WORLD_SIZE=1); DistributedTrainer at one rank must agree with it too."""
    one = _run(0, 1, 0, str(tmp_path / "w1"), kind, plain=True)
    one_d = _run(0, 1, 0, str(tmp_path / "w1d"), kind)
    assert one_d["candidates"] == one["candidates"] and one_d["scores"] == one["scores"]
    for c, p in one_d["params"].items():
        np.testing.assert_array_equal(p, one["params"][c])
    r0, r1 = _two_ranks(tmp_path, kind)
    # the same decisions and scores on every rank, equal to the one-rank run
    assert r0["candidates"] == r1["candidates"] == one["candidates"]
    # halving: 6 -> 3 at the 3-evaluation milestone; keep_even: 6 -> 3 -> 2; revive: 6 -> 3 -> 6
    assert len(one["candidates"]) == {"halving": 3, "keep_even": 2, "revive": 6}[kind]
    assert r0["scores"] == r1["scores"] == one["scores"]
    # the survivors are split over the ranks (evened out after pruning) ...
    assert set(r0["params"]).isdisjoint(r1["params"])
    assert sorted(list(r0["params"]) + list(r1["params"])) == sorted(one["params"])
    assert abs(len(r0["params"]) - len(r1["params"])) <= 1
    if kind == "keep_even":  # all three survivors started on rank 0: one moved to rank 1
        assert len(r1["params"]) >= 1
    # ... and each one is bit-identical to the one-rank run
    for part in (r0, r1):
        for c, p in part["params"].items():
            assert part["steps"][c] == one["steps"][c] == 40
            np.testing.assert_array_equal(p, one["params"][c])
    # rank 0 returns the whole trainer state (every experiment ever created)
    assert r0["n_state"] == one["n_state"] == 6 and r1["n_state"] is None
