"""Offline task evaluated in a learned world model (reference
task/offline_task_simulated.py:13-111), with the evaluation on the GPU.

Training data: a dict dataset (synthetic of the env's shape by default, or a
local OGBench ``.npz`` through task.offline_task_npz).  Evaluation: the
reference steps ``num_evaluation_envs`` copies of the state predictor and the
termination predictor from real-env resets, one Python-driven jit call per
step (evaluator/evaluation.py:75-114).  Here

* ``evaluate_members`` rolls every requested population member in ONE device
  launch (``Population.rollout`` -> ``fqlpop_rollout``) and returns the
  success rate per member (BASELINE config 5);
* ``reset`` / ``step`` keep the reference's per-step Task contract for the
  generic ``evaluate_agent`` loop, each step running the env model on the
  GPU (``fqlpop_envmodel_step``).

Initial observations: the reference resets MuJoCo envs (absent here); this
task draws episode starts of the training dataset, rows 0, 1000, 2000, ...
as utils/data_loader.py:14-19 (InitialObservationLoader) does.

Env model source, in order: explicit ``env_model=(sp_tree, tp_tree)``; the
reference's files ``<save_directory>/<env_name>/env_models/{model}.pt`` +
``{model}_config.yaml`` and ``termination_predictor.*`` (utils/envmodel.py:10-49;
flax msgpack read by envmodel.flax_msgpack, yaml with SafeLoader); otherwise
a seeded synthetic model of the default shape.
"""
from __future__ import annotations

from pathlib import Path
from typing import Literal

import numpy as np
import yaml

import envmodel as em
from task.offline_task_synthetic import env_shape, make_synthetic_dataset
from task.task import Task


def load_reference_env_model(save_directory: Path, env_name: str, model: str):
    """(sp_tree, tp_tree) from the reference's save layout (utils/envmodel.py:10-49)."""
    d = Path(save_directory) / env_name / "env_models"
    trees = []
    for name in (model, "termination_predictor"):
        cfg_path, pt_path = d / f"{name}_config.yaml", d / f"{name}.pt"
        if not cfg_path.exists() or not pt_path.exists():
            raise FileNotFoundError(f"env model {name} not found under {d}")
        with open(cfg_path) as f:
            yaml.load(f, Loader=yaml.SafeLoader)  # hidden dims are re-derived from the shapes
        tree = em.load_flax_msgpack(pt_path)
        trees.append(tree)
    return trees[0], trees[1]


class OfflineTaskWithSimulatedEvaluations(Task):
    def __init__(self, env_name: str = "cube-single-play-singletask-task2-v0", model: str = "multistep",
                 save_directory: Path | None = None, dataset: dict | None = None, val_dataset: dict | None = None,
                 n_rows: int = 100_000, n_val_rows: int = 10_000, num_evaluation_envs: int = 50,
                 max_episode_steps: int = 1000, env_model=None, seed: int = 0):
        self.env_name = env_name
        self.model = model
        self.max_episode_steps = int(max_episode_steps)
        self.num_envs = int(num_evaluation_envs)
        obs_dim, action_dim = env_shape(env_name)
        if dataset is None:
            dataset = make_synthetic_dataset(n_rows, obs_dim, action_dim, seed)
            val_dataset = make_synthetic_dataset(n_val_rows, obs_dim, action_dim, seed + 1)
        self.train_dataset = dataset
        self.val_dataset = val_dataset if val_dataset is not None else dataset
        self.obs_dim = self.train_dataset["observations"].shape[-1]
        self.action_dim = self.train_dataset["actions"].shape[-1]
        if env_model is None and save_directory is not None:
            env_model = load_reference_env_model(save_directory, env_name, model)
        if env_model is None:
            spec = em.EnvModelSpec(self.obs_dim, self.action_dim)
            env_model = (em.init_state_predictor(spec, seed), em.init_termination_predictor(spec, seed + 1))
        self.sp_tree, self.tp_tree = env_model
        self.spec = em.spec_from_trees(self.sp_tree, self.tp_tree)
        self.initial_observations = self.train_dataset["observations"][::1000]
        self._population = None
        self.current_observations = None
        self.episode_steps = 0
        self.invalidate = []

    # ---------------------------------------------------------------- data
    def sample(self, dataset: Literal["train", "val"], batch_size: int):
        data = self.train_dataset if dataset == "train" else self.val_dataset
        idx = np.random.randint(data["observations"].shape[0], size=batch_size)
        return {k: v[idx] for k, v in data.items()}

    def device_datasets(self):
        keys = ("observations", "actions", "rewards", "masks", "next_observations")
        return {"train": {k: self.train_dataset[k] for k in keys},
                "val": {k: self.val_dataset[k] for k in keys}}

    # ---------------------------------------------------- device env model
    def attach(self, population) -> None:
        """Upload the env model into a population's handle (once per handle)."""
        if self._population is population:
            return
        population.set_env_model(em.flatten_state_predictor(self.spec, self.sp_tree),
                                 em.flatten_termination_predictor(self.spec, self.tp_tree),
                                 self.spec.sp_hidden, self.spec.tp_hidden)
        self._population = population

    def reset_observations(self, seed: int | None = None) -> np.ndarray:
        rng = np.random.default_rng(seed)
        idx = rng.integers(0, self.initial_observations.shape[0], size=self.num_envs)
        return self.initial_observations[idx].astype(np.float32)

    def evaluate_members(self, population, members, seed: int = 0) -> dict:
        """Success rate of each member in ``members`` (population slots): every
        member's episodes in one GPU launch.  Restores the active mask."""
        self.attach(population)
        saved = population.active.copy()
        mask = np.zeros(population.n, dtype=bool)
        mask[list(members)] = True
        population.set_active(mask)
        try:
            success, lengths = population.rollout(self.reset_observations(seed), self.max_episode_steps, seed=seed)
        finally:
            population.set_active(saved)
        ids = [int(i) for i in np.nonzero(mask)[0]]
        return {m: {"success": float(success[k].mean()), "episode_length": float(lengths[k].mean())}
                for k, m in enumerate(ids)}

    # ------------------------------------------- reference per-step contract
    def reset(self, seed: int | None = None):
        self.current_observations = self.reset_observations(seed)
        self.episode_steps = 0
        self.invalidate = [False] * self.num_envs
        return self.current_observations.copy(), [{} for _ in range(self.num_envs)]

    def step(self, actions):
        if self._population is None:
            raise RuntimeError("attach(population) first: the env model runs on the population's GPU")
        nxt, logits = self._population.envmodel_step(self.current_observations, np.clip(actions, -1, 1))
        terminations = logits > 0
        reward = np.where(terminations, 0, -1)
        self.current_observations = nxt
        self.episode_steps += 1
        truncations = np.full(terminations.shape, self.episode_steps >= self.max_episode_steps)
        infos = [{"success": bool(s)} for s in terminations]
        for i in range(self.num_envs):
            if self.invalidate[i]:
                infos[i]["invalid"] = True
            if terminations[i] or truncations[i]:
                self.invalidate[i] = True
        return nxt.copy(), reward, terminations, truncations, infos

    def close(self):
        self._population = None
