"""Successive halving over evaluation milestones (reference
hpo/successive_halving.py:10-115).

With N candidates, prune fraction f and history length h over E total
evaluations: eta = 1/(1-f), T = int((E - h)(1 - f)), R = floor(log N / log eta)
rounds, milestones = [int(T * eta**-r) + h for r < R].  At a milestone (and once
at least h scores exist) the population shrinks to the best
max(1, int(n - n f)) candidates by the mean of their last h scores.
"""
from __future__ import annotations

import math
from collections import defaultdict
from typing import List

from hpo.strategy import HpoStrategy


class SuccessiveHalving(HpoStrategy):
    def __init__(self, population, total_evaluations: int, fraction: float = 0.5,
                 history_length: int = 1, state_dict: dict | None = None) -> None:
        super().__init__(population, total_evaluations, state_dict)
        self.fraction = fraction
        self.history_length = history_length
        self.candidate_scores = defaultdict(list)
        self.performed_evaluations = 0
        self.halving_milestones = self.compute_halving_milestones()
        if state_dict is not None:
            self.candidate_scores = defaultdict(list, state_dict["candidate_scores"])
            self.performed_evaluations = state_dict["performed_evaluations"]

    def state_dict(self) -> dict:
        sd = super().state_dict()
        sd["candidate_scores"] = dict(self.candidate_scores)
        sd["performed_evaluations"] = self.performed_evaluations
        return sd

    def update(self, candidate, performance: float) -> None:
        history = self.candidate_scores[candidate]
        history.append(performance)
        if len(history) > self.performed_evaluations:
            self.performed_evaluations = len(history)

    def _mean_recent(self, scores):
        return sum(scores[-self.history_length:]) / self.history_length

    def sample(self):
        at_milestone = self.performed_evaluations in self.halving_milestones
        if not at_milestone or self.performed_evaluations < self.history_length:
            return self.population
        n = len(self.population)
        if n <= 1:
            return self.population
        keep = max(1, int(n - n * self.fraction))
        ranked = sorted(self.candidate_scores.items(), key=lambda kv: self._mean_recent(kv[1]),
                        reverse=True)
        self.population = {cand for cand, _ in ranked[:keep]}
        return self.population

    def compute_halving_milestones(self) -> List[int]:
        n = len(self.population)
        eta = 1.0 / (1.0 - self.fraction)
        horizon = int((self.total_evaluations - self.history_length) * (1.0 - self.fraction))
        rounds = int(math.floor(math.log(n) / math.log(eta)))
        return [int(horizon * eta ** -r) + self.history_length for r in range(rounds)]
