"""A seeded evaluation leaves the process-wide random / np.random streams alone.

The reference's ``Experiment.evaluate`` passes no seed (reference trainer/experiment.py:121),
so its ``evaluate_actor_fn`` never re-seeds the global streams (evaluator/evaluation.py:41-43)
that ``task.sample`` draws batches from and that the trainer checkpoints (np_rng_state).  Our
Trainer seeds each evaluation by (run seed, round, candidate) for world-size independence; the
evaluation must then not leak that seed into the global streams, or every rank would end a
round with a global state set by the last member it happened to evaluate."""
import random

import numpy as np

from trainer.experiment import Experiment


class _Env:
    """Two envs that finish after 3 steps with success 1."""

    def reset(self, seed=None):
        self.t = 0
        return np.zeros((2, 3), np.float32), {}

    def step(self, actions):
        self.t += 1
        done = np.full(2, self.t >= 3)
        return np.zeros((2, 3), np.float32), 0.0, done, np.zeros(2, bool), [{"success": 1.0}] * 2


class _Agent:
    population = None

    def sample_actions(self, observations, seed, temperature=0):
        return np.random.default_rng(seed % 2**32).uniform(-1, 1, (len(observations), 2))


class _Logger:
    def __init__(self):
        self.rows = []

    def log(self, info, step, group):
        self.rows.append((group, step, dict(info)))


class _Stub:
    def __init__(self):
        self.task, self.agent, self.logger, self.current_step = _Env(), _Agent(), _Logger(), 7


def _global_state():
    return random.getstate(), np.random.get_state()


def test_seeded_evaluation_keeps_the_global_streams():
    random.seed(123)
    np.random.seed(456)
    before = _global_state()
    score = Experiment.evaluate(_Stub(), None, seed=99)
    after = _global_state()
    assert score == 1.0
    assert before[0] == after[0]
    assert all(np.array_equal(a, b) if isinstance(a, np.ndarray) else a == b for a, b in zip(before[1], after[1]))


def test_seeded_evaluation_is_reproducible_and_independent_of_the_global_streams():
    def run(global_seed):
        random.seed(global_seed)
        np.random.seed(global_seed)
        stub = _Stub()
        Experiment.evaluate(stub, None, seed=5)
        return stub.logger.rows

    assert run(1) == run(2)


def test_unseeded_evaluation_draws_from_np_random_as_the_reference():
    # seed None: the actor seed comes from np.random (reference evaluator/evaluation.py:12-20,
    # 34-36), so the global stream advances, and nothing re-seeds it
    np.random.seed(0)
    Experiment.evaluate(_Stub(), None)
    drawn = np.random.get_state()[2]
    np.random.seed(0)
    np.random.randint(0, 2**32)
    assert drawn == np.random.get_state()[2]
