"""Offline task over a local OGBench-style ``.npz`` dataset.

Replaces the dataset half of ``task/offline_task_real.py:26-36``, i.e.
[EXT] ``fql.envs.env_utils.make_env_and_datasets`` -> ``ogbench.make_env_and_datasets``
(``ogbench.utils.load_dataset`` + ``relabel_dataset`` for singletask datasets), for
files that are already on disk.  Reads ``<data_directory>/<dataset>.npz`` (and
``-val.npz``) with ``numpy.load(allow_pickle=False)``:

* ``rewards`` and ``masks`` must be in the file.  OGBench computes them for the
  singletask datasets by relabelling with the MuJoCo environment (``relabel_dataset``),
  which is absent here, so a raw OGBench file (observations / actions / terminals only)
  is refused instead of trained with invented zeros (masks = 0 would switch
  bootstrapping off for every transition).
* Without ``next_observations`` the file is in OGBench's raw layout (one row per state;
  ``terminals`` = 1 on the last state of each trajectory) and the transitions are built
  as ``load_dataset(compact_dataset=False)`` does: rows whose terminal flag is 0 are
  the transitions, ``next_observations`` is the following row, and the terminal rows
  themselves are dropped (so no transition crosses an episode boundary); ``terminals``
  becomes 1 on each trajectory's last transition.  ``rewards`` / ``masks`` are then
  per raw row and are filtered the same way.  With ``next_observations`` every field
  is already one row per transition and is used as is.
* actions are clipped to +-(1 - 1e-5) ([EXT] env_utils ``action_clip_eps``).

Evaluation environments (MuJoCo) are out of scope: reset/step raise.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from task.task import Task

ACTION_CLIP_EPS = 1e-5


def load_npz_dataset(path: Path) -> dict:
    with np.load(path, allow_pickle=False) as f:
        data = {k: f[k] for k in f.files}
    missing = [k for k in ("observations", "actions", "rewards", "masks") if k not in data]
    if missing:
        raise ValueError(
            f"{path}: missing {missing}.  OGBench singletask rewards/masks come from relabelling the "
            "dataset with the MuJoCo environment (ogbench relabel_dataset), which is not available "
            "here; export a relabelled file that holds them")
    obs = data["observations"].astype(np.float32)
    n = len(obs)
    act = np.clip(data["actions"].astype(np.float32), -1 + ACTION_CLIP_EPS, 1 - ACTION_CLIP_EPS)
    rew = data["rewards"].astype(np.float32).reshape(-1)
    masks = data["masks"].astype(np.float32).reshape(-1)
    if "terminals" in data:
        term = data["terminals"].astype(np.float32).reshape(-1)
    elif "next_observations" in data:
        term = np.zeros(n, np.float32)
    else:
        raise ValueError(f"{path}: raw OGBench layout (no next_observations) needs terminals")
    for k, v in (("actions", act), ("rewards", rew), ("masks", masks), ("terminals", term)):
        if len(v) != n:
            raise ValueError(f"{path}: {k} has {len(v)} rows, observations {n}")
    if "next_observations" in data:
        nxt = data["next_observations"].astype(np.float32)
        if nxt.shape != obs.shape:
            raise ValueError(f"{path}: next_observations shape {nxt.shape} != observations {obs.shape}")
    else:
        if n == 0 or term[-1] != 1.0:
            raise ValueError(f"{path}: the last raw row must end a trajectory (terminals[-1] = 1)")
        ob_mask = term == 0.0
        next_ob_mask = np.concatenate([[False], ob_mask[:-1]])
        nxt = obs[next_ob_mask]
        new_term = np.concatenate([term[1:], [1.0]]).astype(np.float32)
        obs, act, rew, masks, term = obs[ob_mask], act[ob_mask], rew[ob_mask], masks[ob_mask], new_term[ob_mask]
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
