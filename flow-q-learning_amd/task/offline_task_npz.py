"""Offline task over a local OGBench-style ``.npz`` dataset.

Reads ``<data_directory>/<dataset>.npz`` (and ``-val.npz``) with
``numpy.load(allow_pickle=False)``; actions are clipped to +-(1-1e-5) and
masks = 1 - terminals-of-success as in [EXT] fql envs/env_utils.  Evaluation
environments (MuJoCo) are out of scope: reset/step raise.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from task.task import Task


def load_npz_dataset(path: Path) -> dict:
    with np.load(path, allow_pickle=False) as f:
        data = {k: f[k] for k in f.files}
    obs = data["observations"].astype(np.float32)
    act = np.clip(data["actions"].astype(np.float32), -1 + 1e-5, 1 - 1e-5)
    term = data.get("terminals", np.zeros(len(obs), np.float32)).astype(np.float32)
    if "next_observations" in data:
        nxt = data["next_observations"].astype(np.float32)
    else:  # consecutive rows within an episode
        nxt = np.concatenate([obs[1:], obs[-1:]], 0)
    rew = data.get("rewards", np.zeros(len(obs), np.float32)).astype(np.float32)
    masks = data.get("masks", 1.0 - (rew == 0.0)).astype(np.float32)
    return {"observations": obs, "actions": act, "rewards": rew, "masks": masks,
            "next_observations": nxt, "terminals": term}


class OfflineTaskNpz(Task):
    def __init__(self, env_name: str, data_directory: Path):
        base = env_name.replace("-singletask", "").rsplit("-task", 1)[0]
        d = Path(data_directory)
        self.train_dataset = load_npz_dataset(d / f"{base}.npz")
        val = d / f"{base}-val.npz"
        self.val_dataset = load_npz_dataset(val) if val.exists() else self.train_dataset

    def sample(self, dataset, batch_size: int):
        data = self.train_dataset if dataset == "train" else self.val_dataset
        idx = np.random.randint(data["observations"].shape[0], size=batch_size)
        return {k: v[idx] for k, v in data.items()}

    def device_datasets(self):
        keys = ("observations", "actions", "rewards", "masks", "next_observations")
        return {"train": {k: self.train_dataset[k] for k in keys},
                "val": {k: self.val_dataset[k] for k in keys}}

    def reset(self, seed=None):
        raise NotImplementedError("MuJoCo evaluation environments are out of scope")

    def step(self, actions):
        raise NotImplementedError("MuJoCo evaluation environments are out of scope")

    def close(self):
        pass
