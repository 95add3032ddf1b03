"""HPO strategy interface (reference hpo/strategy.py:7-58).

A strategy owns a population of ExperimentConfig candidates, is told each
evaluation score through ``update`` and decides the surviving candidates in
``sample``.  ``state_dict`` makes it resumable.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Iterable, Set

from trainer.config import ExperimentConfig


class HpoStrategy(ABC):
    def __init__(self, population: Iterable[ExperimentConfig], total_evaluations: int,
                 state_dict: dict | None = None):
        self.population = population
        self.total_evaluations = total_evaluations
        if state_dict is not None:
            self.population = state_dict["population"]

    def state_dict(self) -> dict:
        return {"population": self.population}

    @abstractmethod
    def update(self, candidate: ExperimentConfig, performance: float) -> None:
        """Record one evaluation score of ``candidate``."""

    @abstractmethod
    def sample(self) -> Set[ExperimentConfig]:
        """Return the candidates to keep training."""
