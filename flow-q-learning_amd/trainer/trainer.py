"""Population trainer (reference trainer/trainer.py:11-120).

Same surface and bookkeeping as the reference ``Trainer`` (candidates,
untrained/finished candidates, strategy updates, pruning, resumable
``state_dict``), but every evaluation round trains its candidates TOGETHER:
one HBM-resident population, one set of member-batched HIP launches per
update (the reference trains members one after the other).

Deliberate fix: the strategy is updated with the
candidate's ExperimentConfig, not the Experiment object (the reference passes
``self.experiments[config]`` at trainer/trainer.py:86, which breaks
SuccessiveHalving because ``sample()`` then returns Experiments).

Determinism across world sizes: candidates are visited in ``D.ordered`` order
(the reference iterates a set), and the evaluation of round r is seeded by
``D.eval_round_seed(seed, r)`` (world-model rollouts of the whole round) or
``D.member_eval_seed(seed, r, config)`` (per-experiment evaluation), never by the
global np.random stream.  So ``Trainer`` and ``DistributedTrainer`` at any world
size score every member identically and take the same decisions.
"""
from __future__ import annotations

import random
import time

import numpy as np

from fqlpop import Population, PopulationConfig
from fqlpop import distributed as D
from hpo.strategy import HpoStrategy
from task.task import Task
from trainer.config import TrainerConfig
from trainer.experiment import Experiment, agent_config_for, train_population
from dataclasses import asdict


class Trainer:
    def __init__(self, task: Task, strategy: HpoStrategy, config: TrainerConfig, state_dict: dict | None = None,
                 device: int = 0):
        self.task = task
        self.strategy = strategy
        self.config = config
        self.experiments = {}
        self.member_of = {}
        # strategy.sample() is called once on a fresh start (trainer/trainer.py:37-40 of the
        # reference): the same set sizes the population and becomes the candidates, so a
        # strategy whose sample() is stateful or random places the configs it returned
        sampled = None if state_dict else strategy.sample()
        initial = list(state_dict["experiments"]) if state_dict else list(sampled)
        self.population = self._make_population(initial, device)
        if state_dict is not None:
            for cfg, exp_state in state_dict["experiments"].items():
                self.create_experiment(cfg, state_dict=exp_state)
            self.candidates = state_dict["candidates"]
            self.untrained_candidates = state_dict["untrained_candidates"]
            self.finished_candidates = state_dict["finished_candidates"]
            random.setstate(state_dict["random_rng_state"])
            np.random.set_state(state_dict["np_rng_state"])
            self.round_index = int(state_dict.get("round_index", 0))
        else:
            self.round_index = 0
            self.untrained_candidates = []
            self.finished_candidates = []
            self.candidates = sampled
            for cfg in self.candidates:
                self.create_experiment(cfg)

    # ----------------------------------------------------------- population
    def _make_population(self, configs, device):
        example = self.task.sample("train", 1)
        alphas, seeds = [], []
        for cfg in configs:
            acfg, _ = agent_config_for(self.config, cfg)
            alphas.append(acfg.alpha)
            seeds.append(acfg.seed if cfg.seed is None else cfg.seed)
        acfg, _ = agent_config_for(self.config, configs[0])
        pcfg = PopulationConfig.from_agent_config(asdict(acfg), example["observations"].shape[-1],
                                                  example["actions"].shape[-1])
        pop = Population(pcfg, alphas, seeds, device=device)
        dd = self.task.device_datasets()
        if dd is not None:
            pop.set_dataset(dd["train"], "train")
            pop.set_dataset(dd["val"], "val")
        self._free_slots = list(range(len(configs)))
        return pop

    def _slot_for(self, cfg) -> int:
        if cfg in self.member_of:
            return self.member_of[cfg]
        if not self._free_slots:
            raise RuntimeError("population is full: every slot holds a candidate")
        slot = self._free_slots.pop(0)
        acfg, _ = agent_config_for(self.config, cfg)
        self.population.set_member(slot, acfg.alpha, acfg.seed if cfg.seed is None else cfg.seed, reinit=True)
        self.member_of[cfg] = slot
        return slot

    def create_experiment(self, experiment_config, **kwargs) -> Experiment:
        slot = self._slot_for(experiment_config)
        exp = Experiment(self.task, self.config, experiment_config, population=self.population, member=slot,
                         **kwargs)
        self.experiments[experiment_config] = exp
        return exp

    def state_dict(self) -> dict:
        return {
            "experiments": {cfg: exp.state_dict() for cfg, exp in self.experiments.items()},
            "candidates": self.candidates,
            "random_rng_state": random.getstate(),
            "np_rng_state": np.random.get_state(),
            "untrained_candidates": self.untrained_candidates,
            "finished_candidates": self.finished_candidates,
            "round_index": self.round_index,
        }

    # ---------------------------------------------------------------- train
    def _train_round(self, configs):
        """eval_interval updates of every config, in lock-step groups by step."""
        groups = {}
        for cfg in configs:
            exp = self.experiments[cfg]
            groups.setdefault(exp.current_step, []).append(exp)
        for step, exps in groups.items():
            n = min(self.config.eval_interval, self.config.steps - step)
            if exps[0].on_device:
                train_population(exps, n)
            else:
                for e in exps:
                    e.train(self.config.eval_interval)

    def _evaluate_round(self, configs) -> dict:
        """World-model tasks: every candidate of the round in one GPU rollout
        (slot -> eval info); other tasks evaluate per experiment."""
        if not hasattr(self.task, "evaluate_members"):
            return {}
        members = [self.member_of[cfg] for cfg in configs if cfg in self.member_of]
        if not members:
            return {}
        return self.task.evaluate_members(self.population, members,
                                          D.eval_round_seed(self.config.seed, self.round_index))

    def _score(self, cfg, round_eval: dict) -> float:
        """The candidate's evaluation of this round: the round's world-model result, or
        its own evaluation seeded by (run seed, round, candidate)."""
        info = round_eval.get(self.member_of.get(cfg))
        seed = None if info is not None else D.member_eval_seed(self.config.seed, self.round_index, cfg)
        return self.experiments[cfg].evaluate(info, seed=seed)

    def train(self, max_evaluations: int) -> None:
        while max_evaluations > 0:
            queue = list(self.untrained_candidates) if self.untrained_candidates else D.ordered(self.candidates)
            this_round, deferred = queue[:max_evaluations], queue[max_evaluations:]
            start = time.perf_counter()
            self._train_round(this_round)
            round_eval = self._evaluate_round(this_round)
            for cfg in this_round:
                exp = self.experiments[cfg]
                if exp.current_step == exp.steps and cfg not in self.finished_candidates:
                    exp.save_agent()
                    self.finished_candidates.append(cfg)
                self.strategy.update(cfg, self._score(cfg, round_eval))
                max_evaluations -= 1
            self.round_index += 1
            print(f"Elapsed time: {time.perf_counter() - start:.6f} seconds ({len(this_round)} candidates)")
            if deferred:
                self.untrained_candidates = deferred
                break
            self.untrained_candidates = []
            if all(cfg in self.finished_candidates for cfg in self.candidates):
                break
            new_candidates = self.strategy.sample()
            for cfg in new_candidates:
                if cfg not in self.experiments:
                    self.create_experiment(cfg)
            for cfg in self.candidates:
                if cfg not in new_candidates:
                    self.experiments[cfg].stop()
            self.candidates = new_candidates
        for exp in self.experiments.values():
            exp.stop()
