"""Offline task on synthetic transitions of a given shape (no OGBench / MuJoCo in
this environment).

* Dataset: SURVEY.md 8(d) recipe -- obs ~ N(0,1), act ~ U(-1+1e-5, 1-1e-5),
  next_obs = obs + 0.05 N(0,1), reward in {-1, 0} with P(0) = 0.05,
  mask = 1 - (reward == 0), terminals every 1000th row.
* Evaluation env: a vectorised toy reaching task standing in for the MuJoCo
  evaluation of reference task/offline_task_real.py:45-95 (same reset/step
  contract: per-env termination, the `invalid` flag after an env is done,
  `success` in the final info).  MuJoCo evaluation itself is out of scope.
"""
from __future__ import annotations

from typing import Literal

import numpy as np

from task.task import Task

SHAPES = {  # obs_dim, action_dim (cube-single / antsoccer)
    "cube": (28, 5),
    "antsoccer": (42, 8),
}


def env_shape(env_name: str):
    for key, shape in SHAPES.items():
        if env_name.startswith(key):
            return shape
    return SHAPES["cube"]


def make_synthetic_dataset(n_rows: int, obs_dim: int, action_dim: int, seed: int = 0) -> dict:
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((n_rows, obs_dim), dtype=np.float32)
    act = rng.uniform(-1 + 1e-5, 1 - 1e-5, (n_rows, action_dim)).astype(np.float32)
    nxt = obs + np.float32(0.05) * rng.standard_normal((n_rows, obs_dim), dtype=np.float32)
    rew = np.where(rng.uniform(size=n_rows) < 0.05, 0.0, -1.0).astype(np.float32)
    term = np.zeros(n_rows, np.float32)
    term[999::1000] = 1.0
    return {"observations": obs, "actions": act, "rewards": rew,
            "masks": (1.0 - (rew == 0.0)).astype(np.float32), "next_observations": nxt,
            "terminals": term}


class OfflineTaskSynthetic(Task):
    def __init__(self, env_name: str = "cube-single-play-singletask-task2-v0", n_rows: int = 100_000,
                 n_val_rows: int = 10_000, num_evaluation_envs: int = 8, max_episode_steps: int = 50,
                 seed: int = 0):
        self.env_name = env_name
        self.obs_dim, self.action_dim = env_shape(env_name)
        self.train_dataset = make_synthetic_dataset(n_rows, self.obs_dim, self.action_dim, seed)
        self.val_dataset = make_synthetic_dataset(n_val_rows, self.obs_dim, self.action_dim, seed + 1)
        self.num_envs = num_evaluation_envs
        self.max_episode_steps = max_episode_steps
        self._rng = np.random.default_rng(seed + 2)
        self._state = None

    # ---------------------------------------------------------------- data
    def sample(self, dataset: Literal["train", "val"], batch_size: int):
        data = self.train_dataset if dataset == "train" else self.val_dataset
        idx = np.random.randint(data["observations"].shape[0], size=batch_size)
        return {k: v[idx] for k, v in data.items()}

    def device_datasets(self):
        keys = ("observations", "actions", "rewards", "masks", "next_observations")
        return {"train": {k: self.train_dataset[k] for k in keys},
                "val": {k: self.val_dataset[k] for k in keys}}

    # ----------------------------------------------------------------- env
    def reset(self, seed: int | None = None):
        rng = np.random.default_rng(seed) if seed is not None else self._rng
        self._state = rng.standard_normal((self.num_envs, self.obs_dim)).astype(np.float32)
        self._t = 0
        self.invalidate = [False] * self.num_envs
        return self._state.copy(), [{} for _ in range(self.num_envs)]

    def step(self, actions):
        actions = np.clip(np.asarray(actions, np.float32), -1, 1)
        A = self.action_dim
        self._state[:, :A] = 0.9 * self._state[:, :A] + 0.3 * actions
        self._t += 1
        dist = np.linalg.norm(self._state[:, :A], axis=1)
        success = dist < 0.25 * np.sqrt(A)
        terminated = success.copy()
        truncated = np.full(self.num_envs, self._t >= self.max_episode_steps)
        rewards = np.where(success, 0.0, -1.0)
        infos = []
        for i in range(self.num_envs):
            info = {"success": float(success[i])}
            if self.invalidate[i]:
                info["invalid"] = True
            if terminated[i] or truncated[i]:
                self.invalidate[i] = True
            infos.append(info)
        return self._state.copy(), rewards, terminated, truncated, infos

    def close(self):
        self._state = None
