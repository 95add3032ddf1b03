"""Task interface (reference task/task.py:5-45): minibatch sampling for
training plus a vectorised environment for evaluation."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Literal


class Task(ABC):
    @abstractmethod
    def sample(self, dataset: Literal["train", "val"], batch_size: int):
        """A dict minibatch (observations, actions, rewards, masks, next_observations)."""

    @abstractmethod
    def reset(self, seed: int | None = None):
        """Reset every evaluation environment; returns (observations, infos)."""

    @abstractmethod
    def step(self, actions):
        """Step every evaluation environment; returns (obs, rewards, terminated, truncated, infos)."""

    @abstractmethod
    def close(self):
        """Release the evaluation environments."""

    def device_datasets(self):
        """Optional: {"train": dict, "val": dict} of full row-major arrays that the
        population engine copies to HBM once and samples on device."""
        return None
