"""CPU oracle for the world-model rollout evaluator -- TEST INFRASTRUCTURE ONLY.

float64 NumPy restatement of the reference's simulated evaluation, used only
by ``tests/`` as the checker of ``fqlpop_rollout`` / ``fqlpop_envmodel_step``
(the product path never imports it):

* ``state_predictor``   -- envmodel/baseline.py:25-37 (BaselineStatePredictor):
  x = LayerNorm(concat(s, a)) (flax LayerNorm: eps 1e-6, fast variance
  E[x^2] - E[x]^2 clipped at 0, scale and bias), Dense + ReLU per hidden dim,
  next = Dense(obs_dim)(x) + s.  multistep = the same cell
  (envmodel/multistep.py:10-54, utils/envmodel.py:46-49).
* ``termination_predictor`` -- envmodel/termination_predictor.py:14-21:
  Dense + ReLU per hidden dim, Dense(1), squeeze (dropout off at eval).
* ``rollout`` -- evaluator/evaluation.py:75-114 driving
  task/offline_task_simulated.py:85-107: a = clip(sample_actions(s)),
  s' = state_predictor(s, a), terminated = termination_predictor(s') > 0,
  truncated at max_episode_steps; an env's result is its first
  terminated-or-truncated step (success = terminated there), later steps
  are ``invalid`` and ignored.

Parity status: restated from the in-tree reference files above; the
reference cannot run here (jax / flax absent) and ships no trained env model
or rollout output, so the GPU path is checked against this restatement only.
"""
from __future__ import annotations

import numpy as np

from oracle.fql_oracle import LN_EPS, OracleConfig, sample_actions


def _dense(tree: dict, i: int, x: np.ndarray) -> np.ndarray:
    d = tree[f"Dense_{i}"]
    return x @ np.asarray(d["kernel"], np.float64) + np.asarray(d["bias"], np.float64)


def state_predictor(tree: dict, obs: np.ndarray, act: np.ndarray) -> np.ndarray:
    x = np.concatenate([obs, act], axis=-1).astype(np.float64)
    mu = x.mean(-1, keepdims=True)
    var = np.maximum((x * x).mean(-1, keepdims=True) - mu * mu, 0.0)
    ln = tree["LayerNorm_0"]
    x = (x - mu) / np.sqrt(var + LN_EPS) * np.asarray(ln["scale"], np.float64) + np.asarray(ln["bias"], np.float64)
    n = sum(1 for k in tree if k.startswith("Dense_"))
    for i in range(n - 1):
        x = np.maximum(_dense(tree, i, x), 0.0)
    return _dense(tree, n - 1, x) + obs


def termination_predictor(tree: dict, obs: np.ndarray) -> np.ndarray:
    x = obs.astype(np.float64)
    n = sum(1 for k in tree if k.startswith("Dense_"))
    for i in range(n - 1):
        x = np.maximum(_dense(tree, i, x), 0.0)
    return _dense(tree, n - 1, x)[..., 0]


def rollout(cfg: OracleConfig, params: dict, sp_tree: dict, tp_tree: dict, init_obs: np.ndarray,
            noise: np.ndarray, max_steps: int):
    """One member: noise [max_steps][n_envs][A].  Returns (success [n_envs],
    length [n_envs], obs after the last step run, number of steps run)."""
    obs = init_obs.astype(np.float64)
    n = obs.shape[0]
    done = np.zeros(n, bool)
    success = np.zeros(n)
    length = np.zeros(n)
    t = 0
    for t in range(1, max_steps + 1):
        a = sample_actions(cfg, params, obs, noise[t - 1].astype(np.float64))
        obs = state_predictor(sp_tree, obs, a)
        term = termination_predictor(tp_tree, obs) > 0
        new = ~done & (term | (t >= max_steps))
        success[new & term] = 1.0
        length[new] = t
        done |= new
        if done.all():
            break
    return success, length, obs, t
