"""Population trainer sharded over ranks: one process per GPU (BASELINE configs 4
and 5).

The reference trains its population serially in one process
(trainer/trainer.py:69-120).  Here every rank runs the same control flow as
``Trainer.train`` over the SAME strategy state, but trains and evaluates only
the members it owns:

* owners: the ordered candidates dealt round-robin over the ranks
  (``fqlpop.distributed.assign_owners``); each rank's ``Population`` holds its
  share (``shard_capacity`` slots);
* after each round the per-member (score, finished) pairs are all-gathered
  (``gather_scores``; RCCL over xGMI on GPUs, gloo on CPU) and every rank feeds
  ALL of them to its strategy in the same order, so every rank's
  ``strategy.sample()`` returns the same survivors -- no decision is broadcast;
* pruned members are retired by their owner; when pruning leaves the shards
  uneven, ``rebalance_plan`` moves the fewest members (their full
  ``Experiment.state_dict``: parameters, Adam moments and count, logger state,
  step) from the most to the least loaded rank by point-to-point sends.  The
  device sampler is keyed by (seed, alpha, update count), not by slot or rank,
  so a moved member continues exactly as it would have in place;
* the evaluation of round r is seeded by ``eval_round_seed(config.seed, r)``
  (world-model rollouts) or ``member_eval_seed(config.seed, r, config)``
  (``Trainer._score``), so a member's scores -- and therefore every decision --
  are the same for every world size and equal to the single-process Trainer's.

``state_dict()`` is collective: rank 0 returns the reference-shaped trainer
state (every experiment ever created, candidates, RNG states), the other ranks
None; any world size resumes from it.
"""
from __future__ import annotations

import random
import time

import numpy as np

from fqlpop import distributed as D
from hpo.strategy import HpoStrategy
from task.task import Task
from trainer.config import TrainerConfig
from trainer.trainer import Trainer


class DistributedTrainer(Trainer):
    def __init__(self, task: Task, strategy: HpoStrategy, config: TrainerConfig, state_dict: dict | None = None,
                 device: int = 0):
        self.rank, self.world_size = D.world()
        self.task = task
        self.strategy = strategy
        self.config = config
        self.experiments = {}   # this rank's live experiments
        self.member_of = {}
        self.retired = {}       # config -> state dict of members this rank stopped (pruned or moved in from a checkpoint)
        if state_dict is not None:
            self.candidates = state_dict["candidates"]
            self.untrained_candidates = list(state_dict["untrained_candidates"])
            self.finished_candidates = list(state_dict["finished_candidates"])
            self.round_index = int(state_dict.get("round_index", 0))
            saved = state_dict["experiments"]
            random.setstate(state_dict["random_rng_state"])
            np.random.set_state(state_dict["np_rng_state"])
        else:
            self.candidates = strategy.sample()
            self.untrained_candidates = []
            self.finished_candidates = []
            self.round_index = 0
            saved = {}
        live = D.ordered(self.candidates)
        self.owner = D.assign_owners(live, self.world_size)
        local = [c for c in live if self.owner[c] == self.rank]
        cap = D.shard_capacity(len(live), self.world_size)
        # slots beyond this rank's share are placeholders until a member is created there
        self.population = self._make_population((local + live * cap)[:cap], device)
        for cfg in local:
            self.create_experiment(cfg, state_dict=saved.get(cfg))
        if self.rank == 0:  # experiments that are no longer candidates: re-emitted by rank 0's state_dict
            self.retired = {c: s for c, s in saved.items() if c not in self.owner}
        # holder[c]: the rank that keeps the state of a stopped experiment c (the same map on
        # every rank), so that a strategy that brings c back (SuccessiveHalving ranks every
        # candidate it has scores for, hpo/successive_halving.py:83-97) resumes it, not a
        # fresh one
        self.holder = {c: 0 for c in saved if c not in self.owner}

    # ------------------------------------------------------------ members
    def _release(self, cfg) -> dict:
        """Stop a local experiment and free its slot; returns its state dict."""
        exp = self.experiments.pop(cfg)
        state = exp.state_dict()
        exp.stop()
        slot = self.member_of.pop(cfg)
        self._free_slots.append(slot)
        return state

    def _rebalance(self, live) -> None:
        for cfg, src, dst in D.rebalance_plan(live, self.owner, self.world_size):
            if self.rank == src:
                D.send_object(self._release(cfg), dst)
            elif self.rank == dst:
                self.create_experiment(cfg, state_dict=D.recv_object(src))
            self.owner[cfg] = dst

    # -------------------------------------------------------------- state
    def state_dict(self) -> dict | None:
        """Collective: every rank contributes its members; rank 0 returns the merged state."""
        mine = {cfg: exp.state_dict() for cfg, exp in self.experiments.items()}
        mine.update(self.retired)
        parts = D.gather_objects(mine, dst=0)
        if self.rank != 0:
            return None
        experiments = {}
        for p in parts:
            experiments.update(p)
        return {
            "experiments": experiments,
            "candidates": self.candidates,
            "random_rng_state": random.getstate(),
            "np_rng_state": np.random.get_state(),
            "untrained_candidates": self.untrained_candidates,
            "finished_candidates": self.finished_candidates,
            "round_index": self.round_index,
        }

    # -------------------------------------------------------------- train
    def train(self, max_evaluations: int) -> None:
        while max_evaluations > 0:
            queue = list(self.untrained_candidates) if self.untrained_candidates else D.ordered(self.candidates)
            this_round, deferred = queue[:max_evaluations], queue[max_evaluations:]
            local = [c for c in this_round if self.owner.get(c) == self.rank]
            start = time.perf_counter()
            self._train_round(local)
            round_eval = self._evaluate_round(local)
            results = {}
            for cfg in local:
                exp = self.experiments[cfg]
                done = exp.current_step == exp.steps
                if done and cfg not in self.finished_candidates:
                    exp.save_agent()
                results[cfg] = (self._score(cfg, round_eval), done)
            merged = D.gather_scores(results)
            for cfg in this_round:  # the same order on every rank: identical strategy state
                score, done = merged[cfg]
                if done and cfg not in self.finished_candidates:
                    self.finished_candidates.append(cfg)
                self.strategy.update(cfg, score)
                max_evaluations -= 1
            self.round_index += 1
            if self.rank == 0:
                print(f"Elapsed time: {time.perf_counter() - start:.6f} seconds ({len(this_round)} candidates, "
                      f"{self.world_size} ranks)")
            if deferred:
                self.untrained_candidates = deferred
                break
            self.untrained_candidates = []
            if all(cfg in self.finished_candidates for cfg in self.candidates):
                break
            new_candidates = self.strategy.sample()
            for cfg in D.ordered(self.candidates):
                if cfg not in new_candidates:
                    src = self.owner.pop(cfg)
                    self.holder[cfg] = src
                    if src == self.rank:
                        self.retired[cfg] = self._release(cfg)
            live = D.ordered(new_candidates)
            for cfg, r in D.place_new([c for c in live if c not in self.owner], live, self.owner,
                                      self.world_size).items():
                self.owner[cfg] = r
                src = self.holder.pop(cfg, None)
                if src is None:  # a new candidate
                    if r == self.rank:
                        self.create_experiment(cfg)
                elif src == r:   # a stopped candidate brought back on the rank that holds it
                    if r == self.rank:
                        self.create_experiment(cfg, state_dict=self.retired.pop(cfg))
                elif self.rank == src:
                    D.send_object(self.retired.pop(cfg), r)
                elif self.rank == r:
                    self.create_experiment(cfg, state_dict=D.recv_object(src))
            self._rebalance(live)
            self.candidates = new_candidates
        for exp in self.experiments.values():
            exp.stop()
