"""Keep-everyone strategy (reference hpo/identity.py:7-15); tune_alpha.py uses it."""
from __future__ import annotations

from hpo.strategy import HpoStrategy


class Identity(HpoStrategy):
    def update(self, candidate, performance: float) -> None:
        return None

    def sample(self):
        return self.population
