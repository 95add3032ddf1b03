"""World-model (env-model) parameters for the on-GPU rollout evaluator.

Host-side bookkeeping only -- the networks run in ``rollout_kernel`` behind
``fqlpop_set_env_model`` / ``fqlpop_rollout`` / ``fqlpop_envmodel_step``
(include/fqlpop.h).  Shapes follow the reference:

* ``BaselineStatePredictor`` (envmodel/baseline.py:17-37): LayerNorm over
  concat(s, a), Dense + ReLU per hidden dim, Dense(obs_dim) + s.  The
  ``multistep`` model scans the same cell (envmodel/multistep.py:10-54); its
  parameters are ``params["ScanCell_0"]["cell"]`` (utils/envmodel.py:46-49).
* ``TerminationPredictor`` (envmodel/termination_predictor.py:9-21): Dense +
  ReLU per hidden dim, Dense(1); dropout is inactive at evaluation.
* hidden dims default to the env-model argparser's (128, 256, 128)
  (argparser.py:184-189).

Flat vectors are in flax leaf order (path-sorted): Dense_0/bias,
Dense_0/kernel, ..., then LayerNorm_0/bias, LayerNorm_0/scale.
"""
from __future__ import annotations

from dataclasses import dataclass, field
import math

import numpy as np

from envmodel.flax_msgpack import load_flax_msgpack  # noqa: F401

DEFAULT_HIDDEN = (128, 256, 128)


@dataclass
class EnvModelSpec:
    obs_dim: int
    action_dim: int
    sp_hidden: tuple = field(default=DEFAULT_HIDDEN)
    tp_hidden: tuple = field(default=DEFAULT_HIDDEN)

    def sp_dims(self):
        return [self.obs_dim + self.action_dim, *self.sp_hidden, self.obs_dim]

    def tp_dims(self):
        return [self.obs_dim, *self.tp_hidden, 1]


def _dense_stack(dims, rng, scale: float):
    """flax nn.Dense defaults: kernel lecun_normal (truncated normal, variance
    1/fan_in), bias zeros.  ``scale`` multiplies the kernels (synthetic models)."""
    tree = {}
    for i in range(len(dims) - 1):
        std = math.sqrt(1.0 / dims[i]) / 0.87962566103423978  # truncated-normal correction (flax)
        k = rng.standard_normal((dims[i], dims[i + 1]))
        k = np.clip(k, -2.0, 2.0) * std * scale
        tree[f"Dense_{i}"] = {"kernel": k.astype(np.float32), "bias": np.zeros(dims[i + 1], np.float32)}
    return tree


def init_state_predictor(spec: EnvModelSpec, seed: int = 0, scale: float = 1.0) -> dict:
    rng = np.random.default_rng(seed)
    tree = _dense_stack(spec.sp_dims(), rng, scale)
    k0 = spec.obs_dim + spec.action_dim
    tree["LayerNorm_0"] = {"scale": np.ones(k0, np.float32), "bias": np.zeros(k0, np.float32)}
    return tree


def init_termination_predictor(spec: EnvModelSpec, seed: int = 1, scale: float = 1.0, bias: float = 0.0) -> dict:
    rng = np.random.default_rng(seed)
    tree = _dense_stack(spec.tp_dims(), rng, scale)
    last = f"Dense_{len(spec.tp_dims()) - 2}"
    tree[last]["bias"] = np.full(1, bias, np.float32)
    return tree


def _flatten(tree: dict, names) -> np.ndarray:
    parts = []
    for mod, leaf in names:
        parts.append(np.asarray(tree[mod][leaf], np.float32).reshape(-1))
    return np.concatenate(parts).astype(np.float32)


def sp_leaf_names(spec: EnvModelSpec):
    n = len(spec.sp_dims()) - 1
    names = [(f"Dense_{i}", leaf) for i in range(n) for leaf in ("bias", "kernel")]
    return sorted(names) + [("LayerNorm_0", "bias"), ("LayerNorm_0", "scale")]


def tp_leaf_names(spec: EnvModelSpec):
    n = len(spec.tp_dims()) - 1
    return sorted((f"Dense_{i}", leaf) for i in range(n) for leaf in ("bias", "kernel"))


def flatten_state_predictor(spec: EnvModelSpec, tree: dict) -> np.ndarray:
    return _flatten(_unwrap_sp(tree), sp_leaf_names(spec))


def flatten_termination_predictor(spec: EnvModelSpec, tree: dict) -> np.ndarray:
    return _flatten(_unwrap(tree), tp_leaf_names(spec))


def _unwrap(tree: dict) -> dict:
    return tree["params"] if "params" in tree else tree


def _unwrap_sp(tree: dict) -> dict:
    """Accept a baseline tree or a multistep one (params/ScanCell_0/cell/...)."""
    t = _unwrap(tree)
    if "ScanCell_0" in t:
        t = t["ScanCell_0"]["cell"]
    return t


def spec_from_trees(sp_tree: dict, tp_tree: dict) -> EnvModelSpec:
    """Infer hidden dims from parameter shapes (a loaded checkpoint)."""
    sp, tp = _unwrap_sp(sp_tree), _unwrap(tp_tree)
    ns = sum(1 for k in sp if k.startswith("Dense_"))
    nt = sum(1 for k in tp if k.startswith("Dense_"))
    sp_k = [np.asarray(sp[f"Dense_{i}"]["kernel"]).shape for i in range(ns)]
    tp_k = [np.asarray(tp[f"Dense_{i}"]["kernel"]).shape for i in range(nt)]
    obs_dim = sp_k[-1][1]
    action_dim = sp_k[0][0] - obs_dim
    return EnvModelSpec(obs_dim, action_dim, tuple(s[1] for s in sp_k[:-1]), tuple(s[1] for s in tp_k[:-1]))
