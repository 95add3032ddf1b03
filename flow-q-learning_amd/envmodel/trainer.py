"""Env-model trainers on the GPU.

Same surface as the reference's ``StatePredictorTrainer``
(envmodel/state_predictor_trainer.py:22-170) and ``TerminationPredictorTrainer``
(envmodel/termination_predictor_trainer.py:21-171): ``train_step(state, batch)``,
``eval_step(state, batch)``, ``train()``, the cosine-decayed Adam of their
``__init__``, val logs every 100 steps over ``val_batches`` batches.  The step
itself is ``fqlpop_emtrain_*`` (include/fqlpop.h): one fused HIP launch for
forward + loss + backward of the 16-row blocks and one for the Adam update.
There is no CPU path: a missing libfqlpop.so raises.

Differences to the reference, by necessity:

* models are specified by ``EnvModelSpec`` + a parameter tree (flax is absent);
  the tree and flat-vector order are flax's (``envmodel.sp_leaf_names``);
* ``train()`` samples minibatches on the device from the loader's dataset
  (uniform with replacement, like ``Dataset.sample``) instead of the global
  numpy stream, when the loader exposes ``dataset``; otherwise it uploads
  ``loader.sample(B)`` every step;
* the dropout mask of the termination trainer is one fixed mask, as in the
  reference (it passes the same ``self.rng`` every step), but drawn by Philox.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

import envmodel as em

DEFAULT_FOCAL_ALPHA, DEFAULT_FOCAL_GAMMA, DEFAULT_DROPOUT = 0.25, 2.0, 0.1
SP_LOG_KEYS = ("loss", "next_observation_loss", "termination_loss", "true_termination_loss",
               "false_termination_loss")
TP_TRAIN_LOG_KEYS = ("loss", "true_loss", "false_loss")
TP_EVAL_LOG_KEYS = ("loss", "true_loss", "false_loss", "accuracy", "precision", "recall")
MULTISTEP_EPISODE_LENGTH = 1000  # utils/data_loader.py:30 reshapes the dataset into 1000-step episodes


@dataclass
class EnvModelTrainerConfig:
    """envmodel/config.py:5-20 (TrainerConfig)."""
    seed: int = 0
    steps: int = 2000
    env_name: str = "cube-single-play-singletask-task2-v0"
    model: str = "baseline"
    true_termination_weight: float = 30.0
    termination_weight: float = 1.0
    reconstruction_weight: float = 1.0
    model_config: dict = field(default_factory=dict)
    init_learning_rate: float = 1e-3
    batch_size: int = 256
    sequence_length: int = 256
    val_batches: int = 20
    data_directory: Path = Path("data/")
    save_directory: Path = Path("exp/")


def unflatten(names, shapes, flat: np.ndarray) -> dict:
    tree, o = {}, 0
    for (mod, leaf), shp in zip(names, shapes):
        n = int(np.prod(shp))
        tree.setdefault(mod, {})[leaf] = flat[o:o + n].reshape(shp).copy()
        o += n
    return tree


def _leaf_shapes(names, dims, ln_dim=None):
    shapes = []
    for mod, leaf in names:
        if mod.startswith("Dense_"):
            i = int(mod.split("_")[1])
            shapes.append((dims[i], dims[i + 1]) if leaf == "kernel" else (dims[i + 1],))
        else:
            shapes.append((ln_dim,))
    return shapes


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, np.float32))


class _GpuEnvModelTrainer:
    kind = None

    def __init__(self, spec: em.EnvModelSpec, params: dict, train_loader, val_loader, config: EnvModelTrainerConfig,
                 logger=None, device: int = 0, tp_params: dict | None = None, focal_alpha=DEFAULT_FOCAL_ALPHA,
                 focal_gamma=DEFAULT_FOCAL_GAMMA, dropout_rate=DEFAULT_DROPOUT):
        from fqlpop._lib import EM_MULTISTEP, EmTrainConfig, check, fptr, load_library
        self._lib, self._check, self._fptr = load_library(), check, fptr
        self.spec, self.config, self.logger = spec, config, logger
        self.train_loader, self.val_loader = train_loader, val_loader
        # the multistep model (train_env_model.py:46-66) trains the same cell through a scan
        self._ms = self.kind == 0 and getattr(config, "model", "baseline") == "multistep"
        self._T = int(config.sequence_length) if self._ms else 1
        c = EmTrainConfig()
        c.kind = EM_MULTISTEP if self._ms else self.kind
        c.sequence_length = self._T
        c.episode_length = int(getattr(train_loader, "episode_length", MULTISTEP_EPISODE_LENGTH)) if self._ms else 0
        c.obs_dim, c.action_dim = spec.obs_dim, spec.action_dim
        hid = spec.sp_hidden if self.kind == 0 else spec.tp_hidden
        c.num_hidden = len(hid)
        for i, hdim in enumerate(hid):
            c.hidden_dims[i] = int(hdim)
        c.batch_size, c.steps = int(config.batch_size), int(config.steps)
        c.init_lr = float(config.init_learning_rate)
        c.termination_weight = float(config.termination_weight) if self.kind == 0 else 0.0
        c.true_termination_weight = float(config.true_termination_weight)
        c.focal_alpha, c.focal_gamma, c.dropout_rate = float(focal_alpha), float(focal_gamma), float(dropout_rate)
        c.seed = int(config.seed) & 0xFFFFFFFFFFFFFFFF
        c.tp_num_hidden = len(spec.tp_hidden)
        for i, hdim in enumerate(spec.tp_hidden):
            c.tp_hidden_dims[i] = int(hdim)
        self._cfg = c
        if self.kind == 0:
            self._names = em.sp_leaf_names(spec)
            self._shapes = _leaf_shapes(self._names, spec.sp_dims(), spec.obs_dim + spec.action_dim)
            flat = em.flatten_state_predictor(spec, params)
        else:
            self._names = em.tp_leaf_names(spec)
            self._shapes = _leaf_shapes(self._names, spec.tp_dims())
            flat = em.flatten_termination_predictor(spec, params)
        n = ctypes.c_int64()
        check(self._lib.fqlpop_emtrain_param_count(ctypes.byref(c), ctypes.byref(n)))
        if n.value != flat.size:
            raise ValueError(f"parameter count {flat.size} != {n.value}")
        self.n_params = n.value
        h = ctypes.c_void_p()
        flat = _f32(flat)
        check(self._lib.fqlpop_emtrain_create(ctypes.byref(c), fptr(flat), flat.size, int(device), ctypes.byref(h)))
        self._h = h
        if self.kind == 0 and c.termination_weight > 0:
            if tp_params is None:
                raise ValueError("termination_weight > 0 needs the trained termination predictor (tp_params)")
            tflat = _f32(em.flatten_termination_predictor(spec, tp_params))
            check(self._lib.fqlpop_emtrain_set_frozen_termination(h, fptr(tflat), tflat.size))
        ds = getattr(train_loader, "dataset", None) if train_loader is not None else None
        self._device_sampling = isinstance(ds, dict) and "observations" in ds
        if self._device_sampling:
            self._set_dataset(ds)

    # ------------------------------------------------------------- plumbing
    def _set_dataset(self, ds: dict):
        # rows (a multistep loader holds [episodes][episode_length][..]: flattened back to rows)
        D, A = self.spec.obs_dim, self.spec.action_dim
        obs = _f32(ds["observations"]).reshape(-1, D)
        act = _f32(ds["actions"]).reshape(-1, A) if "actions" in ds else np.zeros((len(obs), A), np.float32)
        arrs = [obs, np.ascontiguousarray(act), _f32(ds["rewards"]).reshape(-1),
                _f32(ds["next_observations"]).reshape(-1, D)]
        self._check(self._lib.fqlpop_emtrain_set_dataset(self._h, *[self._fptr(a) for a in arrs], len(arrs[0])))

    def _batch_ptrs(self, batch: dict):
        B = self.config.batch_size
        arrs = [_f32(batch["observations"]),
                _f32(batch.get("actions", np.zeros(np.shape(batch["observations"])[:-1] + (self.spec.action_dim,)))),
                _f32(batch["rewards"]), _f32(batch["next_observations"])]
        if arrs[0].shape[0] != B:
            raise ValueError(f"batch has {arrs[0].shape[0]} rows, batch_size is {B}")
        if self._ms and (arrs[0].ndim != 3 or arrs[0].shape[1] != self._T):
            raise ValueError(f"multistep batches are [B, {self._T}, ..], got {arrs[0].shape}")
        return arrs

    def _logs(self, v: np.ndarray, keys) -> dict:
        return {k: float(v[i]) for i, k in enumerate(keys)}

    # --------------------------------------------------------- reference API
    def train_step(self, state=None, batch: dict | None = None, keep_mask: np.ndarray | None = None):
        """One update on a host batch; returns (state, logs) like the reference's jitted step."""
        arrs = self._batch_ptrs(batch)
        km = None
        if keep_mask is not None:
            km = np.ascontiguousarray(np.asarray(keep_mask, np.uint8))
        self._check(self._lib.fqlpop_emtrain_step_injected(
            self._h, *[self._fptr(a) for a in arrs],
            km.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if km is not None else None))
        return self, self.read_logs()

    def eval_step(self, state=None, batch: dict | None = None) -> dict:
        arrs = self._batch_ptrs(batch)
        out = np.zeros(8, np.float32)
        self._check(self._lib.fqlpop_emtrain_eval(self._h, *[self._fptr(a) for a in arrs], self._fptr(out)))
        return self._logs(out, self._eval_keys())

    def steps(self, n: int):
        """n updates on device-sampled batches (asynchronous)."""
        if not self._device_sampling:
            raise RuntimeError("device sampling needs a loader exposing its dataset dict")
        self._check(self._lib.fqlpop_emtrain_step(self._h, int(n)))

    def read_logs(self) -> dict:
        out = np.zeros(8, np.float32)
        self._check(self._lib.fqlpop_emtrain_read_logs(self._h, self._fptr(out)))
        return self._logs(out, self._train_keys())

    def learning_rate(self, step: int) -> float:
        """optax.cosine_decay_schedule(init_learning_rate, steps)(step)."""
        c = min(step, self.config.steps)
        return self.config.init_learning_rate * 0.5 * (1.0 + np.cos(np.pi * c / self.config.steps))

    def sync(self):
        self._check(self._lib.fqlpop_emtrain_sync(self._h))

    @property
    def count(self) -> int:
        c = ctypes.c_int64()
        self._check(self._lib.fqlpop_emtrain_get_count(self._h, ctypes.byref(c)))
        return c.value

    def flat(self, which: int = 0) -> np.ndarray:
        out = np.zeros(self.n_params, np.float32)
        self._check(self._lib.fqlpop_emtrain_get_params(self._h, int(which), self._fptr(out), self.n_params))
        return out

    @property
    def params(self) -> dict:
        return unflatten(self._names, self._shapes, self.flat(0))

    def _val(self, step: int):
        if self.val_loader is None:
            return
        logs = [self.eval_step(None, self.val_loader.sample(self.config.batch_size))
                for _ in range(self.config.val_batches)]
        if self.logger:
            for k in logs[0]:
                self.logger.log({f"val/{k}": float(np.mean([lg[k] for lg in logs]))}, step=step)

    def train(self) -> None:
        """The reference loop (state_predictor_trainer.py:119-170): val every 100
        steps, one update per step, a final val pass."""
        for step in range(self.config.steps):
            if step % 100 == 0:
                self._val(step)
            if self._device_sampling:
                self.steps(1)
                logs = self.read_logs() if self.logger else None
            else:
                _, logs = self.train_step(None, self.train_loader.sample(self.config.batch_size))
            if self.logger:
                self.logger.log({"train/learning_rate": self.learning_rate(step),
                                 **{f"train/{k}": v for k, v in logs.items()}}, step=step)
        # the reference logs the final pass at the last loop index (step = steps - 1,
        # state_predictor_trainer.py:160-175), so the val curves line up when overlaid
        self._val(self.config.steps - 1)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fqlpop_emtrain_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StatePredictorTrainer(_GpuEnvModelTrainer):
    """envmodel/state_predictor_trainer.py:22-170: the baseline model, or the multistep
    model (envmodel/multistep.py) when ``config.model == "multistep"`` -- then batches
    are [B, sequence_length, ..] windows and ``params`` is the scanned cell's tree."""
    kind = 0

    def _train_keys(self):
        return SP_LOG_KEYS if self._cfg.termination_weight > 0 else SP_LOG_KEYS[:2]

    _eval_keys = _train_keys


class TerminationPredictorTrainer(_GpuEnvModelTrainer):
    """envmodel/termination_predictor_trainer.py:21-171 (focal loss, dropout)."""
    kind = 1

    def _train_keys(self):
        return TP_TRAIN_LOG_KEYS

    def _eval_keys(self):
        return TP_EVAL_LOG_KEYS
