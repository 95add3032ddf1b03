"""CPU oracle for the FQL ``agent.update()`` hot path -- TEST INFRASTRUCTURE ONLY.

This module is the float64 NumPy restatement that the HIP path is checked
against.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker: the product path
(``flow-q-learning_amd/``) never imports, calls or links anything here.

Parity status: **parity unpinned** at per-step granularity.  The reference's
hot path lives in the un-vendored ``fql`` git submodule
(``/root/reference/.gitmodules:1-4`` -> ``MazenAmria/fql``, commit not recorded,
``/root/reference/fql/`` empty) and jax/flax/optax are not installed, so no
reference output of ``FQLAgent.update`` can be produced or found here, and the
reference ships no per-step fixtures.  This
restatement follows the upstream FQL semantics as written in SURVEY.md
Appendix A ([EXT] ``fql/agents/fql.py``, ``fql/utils/networks.py``,
``fql/utils/flax_utils.py``) and the in-tree call sites:

* ``trainer/experiment.py:44-49,108-116`` -- create / update / total_loss calls
* ``trainer/config.py:5-22`` -- hyper-parameters (lr, discount, tau, q_agg,
  alpha, flow_steps, layer norms, normalize_q_loss)

Its gradients are cross-checked against an independent implementation
(torch float64 autograd, ``oracle/fql_torch.py``) and finite differences in
``tests/test_oracle.py``; closed forms (Adam step 1, EMA, Euler with a zero
net, GELU/LN) are known-answer tests there too.

Noise is *injected* (x0, t, z_distill, z_next, z_metric) because JAX threefry
bit-parity is unreproducible without JAX (hard part ii).
"""
from __future__ import annotations

from dataclasses import dataclass, field
import math

import numpy as np

LN_EPS = 1e-6
SQRT_2_OVER_PI = math.sqrt(2.0 / math.pi)

TRAIN_INFO_KEYS = (
    "critic/critic_loss", "critic/q_mean", "critic/q_max", "critic/q_min",
    "actor/actor_loss", "actor/bc_flow_loss", "actor/distill_loss",
    "actor/q_loss", "actor/q", "actor/mse",
    "grad/max", "grad/min", "grad/norm",
)
VAL_INFO_KEYS = TRAIN_INFO_KEYS[:10]

NETS = ("critic", "target_critic", "actor_bc_flow", "actor_onestep_flow")
TRAINABLE = ("critic", "actor_bc_flow", "actor_onestep_flow")


@dataclass
class OracleConfig:
    """Mirror of ``trainer/config.py:5-22`` (AgentConfig) fields used by update."""
    obs_dim: int = 28
    action_dim: int = 5
    hidden_dims: tuple = (512, 512, 512, 512)
    layer_norm: bool = True          # critic LN (scripts/tune-alpha-cube.sh:16)
    actor_layer_norm: bool = False   # trainer/config.py:16
    discount: float = 0.99
    tau: float = 0.005
    q_agg: str = "mean"
    alpha: float = 10.0
    flow_steps: int = 10
    normalize_q_loss: bool = False
    lr: float = 3e-4
    batch_size: int = 256
    num_qs: int = 2


# ----------------------------------------------------------------------------
# elementwise pieces
# ----------------------------------------------------------------------------
def gelu(x):
    """jax.nn.gelu(approximate=True) [EXT flax MLP activation]."""
    return 0.5 * x * (1.0 + np.tanh(SQRT_2_OVER_PI * (x + 0.044715 * x ** 3)))


def gelu_grad(x):
    t = np.tanh(SQRT_2_OVER_PI * (x + 0.044715 * x ** 3))
    return 0.5 * (1.0 + t) + 0.5 * x * (1.0 - t * t) * SQRT_2_OVER_PI * (1.0 + 3 * 0.044715 * x * x)


def layer_norm_stats(g):
    """flax nn.LayerNorm(epsilon=1e-6), fast variance E[x^2]-E[x]^2 clipped at 0."""
    mu = g.mean(-1, keepdims=True)
    var = np.maximum((g * g).mean(-1, keepdims=True) - mu * mu, 0.0)
    rstd = 1.0 / np.sqrt(var + LN_EPS)
    return mu, rstd


# ----------------------------------------------------------------------------
# parameters
# ----------------------------------------------------------------------------
def net_dims(cfg: OracleConfig, net: str):
    D, A = cfg.obs_dim, cfg.action_dim
    if net in ("critic", "target_critic"):
        return [D + A, *cfg.hidden_dims, 1]
    if net == "actor_bc_flow":
        return [D + A + 1, *cfg.hidden_dims, A]
    return [D + A, *cfg.hidden_dims, A]


def net_has_ln(cfg: OracleConfig, net: str) -> bool:
    return cfg.layer_norm if net in ("critic", "target_critic") else cfg.actor_layer_norm


def init_params(cfg: OracleConfig, seed: int) -> dict:
    """Build-defined init: W ~ U(+-sqrt(6/(in+out))) (variance_scaling(1,'fan_avg',
    'uniform')), b = 0, LN scale 1 / bias 0, target := critic."""
    rng = np.random.default_rng(seed)
    params = {}
    for net in ("critic", "actor_bc_flow", "actor_onestep_flow"):
        dims = net_dims(cfg, net)
        ens = cfg.num_qs if net == "critic" else None
        p = {}
        for i in range(len(dims) - 1):
            lim = math.sqrt(6.0 / (dims[i] + dims[i + 1]))
            shp = (dims[i], dims[i + 1]) if ens is None else (ens, dims[i], dims[i + 1])
            p[f"Dense_{i}/kernel"] = rng.uniform(-lim, lim, size=shp)
            p[f"Dense_{i}/bias"] = np.zeros(shp[:-2] + (dims[i + 1],))
            if i < len(dims) - 2 and net_has_ln(cfg, net):
                p[f"LayerNorm_{i}/scale"] = np.ones(shp[:-2] + (dims[i + 1],))
                p[f"LayerNorm_{i}/bias"] = np.zeros(shp[:-2] + (dims[i + 1],))
        params[net] = p
    params["target_critic"] = {k: v.copy() for k, v in params["critic"].items()}
    return params


def leaf_order(cfg: OracleConfig, net: str):
    """Leaf names of one network in flax tree (sorted-key) order."""
    dims = net_dims(cfg, net)
    names = []
    for i in range(len(dims) - 1):
        names += [f"Dense_{i}/bias", f"Dense_{i}/kernel"]
    if net_has_ln(cfg, net):
        for i in range(len(dims) - 2):
            names += [f"LayerNorm_{i}/bias", f"LayerNorm_{i}/scale"]
    return sorted(names)


def ens_slice(p: dict, e):
    if e is None:
        return p
    return {k: v[e] for k, v in p.items()}


# ----------------------------------------------------------------------------
# MLP forward / backward  ([EXT] fql/utils/networks.py MLP)
# ----------------------------------------------------------------------------
def mlp_forward(p: dict, x: np.ndarray, ln: bool):
    n = sum(1 for k in p if k.endswith("/kernel"))
    cache = []
    h = x
    for i in range(n):
        W, b = p[f"Dense_{i}/kernel"], p[f"Dense_{i}/bias"]
        u = h @ W + b
        if i < n - 1:
            g = gelu(u)
            if ln:
                mu, rstd = layer_norm_stats(g)
                xhat = (g - mu) * rstd
                out = xhat * p[f"LayerNorm_{i}/scale"] + p[f"LayerNorm_{i}/bias"]
            else:
                mu = rstd = xhat = None
                out = g
            cache.append((h, u, xhat, rstd))
            h = out
        else:
            cache.append((h,))
            h = u
    return h, cache


def mlp_backward(p: dict, cache, dout: np.ndarray, ln: bool, need_dx: bool):
    """Reverse-mode pass of ``mlp_forward``; returns (grads, dx)."""
    n = len(cache)
    grads = {}
    dh = dout
    for i in reversed(range(n)):
        W = p[f"Dense_{i}/kernel"]
        if i == n - 1:
            X = cache[i][0]
            du = dh
        else:
            X, u, xhat, rstd = cache[i]
            if ln:
                scale = p[f"LayerNorm_{i}/scale"]
                grads[f"LayerNorm_{i}/scale"] = (dh * xhat).sum(0)
                grads[f"LayerNorm_{i}/bias"] = dh.sum(0)
                dxh = dh * scale
                dg = rstd * (dxh - dxh.mean(-1, keepdims=True)
                             - xhat * (dxh * xhat).mean(-1, keepdims=True))
            else:
                dg = dh
            du = dg * gelu_grad(u)
        grads[f"Dense_{i}/kernel"] = X.T @ du
        grads[f"Dense_{i}/bias"] = du.sum(0)
        if i > 0 or need_dx:
            dh = du @ W.T
    return grads, (dh if need_dx else None)


def value_forward(cfg, pnet, obs, act):
    """[EXT] Value: ensemble of num_qs MLPs on concat(s, a) -> [E, B]."""
    x = np.concatenate([obs, act], axis=-1)
    outs, caches = [], []
    for e in range(cfg.num_qs):
        out, cache = mlp_forward(ens_slice(pnet, e), x, cfg.layer_norm)
        outs.append(out[:, 0])
        caches.append(cache)
    return np.stack(outs), caches


def actor_forward(cfg, pnet, obs, act, t=None):
    """[EXT] ActorVectorField: MLP(concat(s, a[, t]))."""
    parts = [obs, act] + ([t] if t is not None else [])
    return mlp_forward(pnet, np.concatenate(parts, axis=-1), cfg.actor_layer_norm)


def compute_flow_actions(cfg, params, obs, noises):
    """[EXT] FQLAgent.compute_flow_actions: 10 Euler steps of v_theta, then clip."""
    x = noises
    B = obs.shape[0]
    for i in range(cfg.flow_steps):
        t = np.full((B, 1), np.float64(np.float32(i / cfg.flow_steps)))
        v, _ = actor_forward(cfg, params["actor_bc_flow"], obs, x, t)
        x = x + v / cfg.flow_steps
    return np.clip(x, -1.0, 1.0)


def sample_actions(cfg, params, obs, noises):
    """[EXT] FQLAgent.sample_actions with injected noise: clip(mu_omega(s, z))."""
    a, _ = actor_forward(cfg, params["actor_onestep_flow"], obs, noises)
    return np.clip(a, -1.0, 1.0)


# ----------------------------------------------------------------------------
# losses + gradients
# ----------------------------------------------------------------------------
def loss_and_grads(cfg: OracleConfig, params: dict, batch: dict, noise: dict,
                   want_grads: bool = True):
    """[EXT] FQLAgent.total_loss = critic_loss + actor_loss, with hand-written
    reverse mode.  ``noise`` keys: z_next, x0, t, z_d, z_metric."""
    B, A = batch["actions"].shape
    s, a = batch["observations"], batch["actions"]
    s2 = batch["next_observations"]
    info = {}
    grads = {}

    # ---- critic loss ------------------------------------------------------
    a_next = sample_actions(cfg, params, s2, noise["z_next"])
    qt, _ = value_forward(cfg, params["target_critic"], s2, a_next)
    q_next = qt.min(0) if cfg.q_agg == "min" else qt.mean(0)
    y = batch["rewards"] + cfg.discount * batch["masks"] * q_next
    q, q_cache = value_forward(cfg, params["critic"], s, a)
    critic_loss = ((q - y[None]) ** 2).mean()
    info.update({"critic/critic_loss": critic_loss, "critic/q_mean": q.mean(),
                 "critic/q_max": q.max(), "critic/q_min": q.min()})

    # ---- actor: BC flow ---------------------------------------------------
    x0, t = noise["x0"], noise["t"]
    x_t = (1 - t) * x0 + t * a
    vel = a - x0
    pred, bc_cache = actor_forward(cfg, params["actor_bc_flow"], s, x_t, t)
    bc_loss = ((pred - vel) ** 2).mean()

    # ---- actor: distillation + Q -----------------------------------------
    a_flow = compute_flow_actions(cfg, params, s, noise["z_d"])
    a_pi, os_cache = actor_forward(cfg, params["actor_onestep_flow"], s, noise["z_d"])
    distill = ((a_pi - a_flow) ** 2).mean()
    a_pi_c = np.clip(a_pi, -1.0, 1.0)
    qpi, qpi_cache = value_forward(cfg, params["critic"], s, a_pi_c)
    qb = qpi.mean(0)
    lam = 1.0 / np.abs(qb).mean() if cfg.normalize_q_loss else 1.0
    q_loss = -lam * qb.mean()
    actor_loss = bc_loss + cfg.alpha * distill + q_loss
    a_met = sample_actions(cfg, params, s, noise["z_metric"])
    mse = ((a_met - a) ** 2).mean()
    info.update({"actor/actor_loss": actor_loss, "actor/bc_flow_loss": bc_loss,
                 "actor/distill_loss": distill, "actor/q_loss": q_loss,
                 "actor/q": qb.mean(), "actor/mse": mse})
    if not want_grads:
        return critic_loss + actor_loss, info, None

    E = cfg.num_qs
    # critic grads (critic loss only)
    gc = {}
    dq = 2.0 * (q - y[None]) / (E * B)
    for e in range(E):
        ge, _ = mlp_backward(ens_slice(params["critic"], e), q_cache[e],
                             dq[e][:, None], cfg.layer_norm, need_dx=False)
        for k, v in ge.items():
            gc.setdefault(k, [None] * E)[e] = v
    grads["critic"] = {k: np.stack(v) for k, v in gc.items()}

    # bc flow grads
    dpred = 2.0 * (pred - vel) / (B * A)
    grads["actor_bc_flow"], _ = mlp_backward(params["actor_bc_flow"], bc_cache, dpred,
                                             cfg.actor_layer_norm, need_dx=False)

    # onestep grads: alpha*distill + q_loss (critic frozen)
    D = cfg.obs_dim
    da = np.zeros_like(a_pi)
    dqpi = -lam / (E * B) * np.ones(B)
    for e in range(E):
        _, dx = mlp_backward(ens_slice(params["critic"], e), qpi_cache[e],
                             dqpi[:, None], cfg.layer_norm, need_dx=True)
        da += dx[:, D:]
    inside = (a_pi > -1.0) & (a_pi < 1.0)
    dapi = cfg.alpha * 2.0 * (a_pi - a_flow) / (B * A) + np.where(inside, da, 0.0)
    grads["actor_onestep_flow"], _ = mlp_backward(params["actor_onestep_flow"], os_cache,
                                                  dapi, cfg.actor_layer_norm, need_dx=False)
    grads["target_critic"] = {k: np.zeros_like(v) for k, v in params["target_critic"].items()}
    return critic_loss + actor_loss, info, grads


def grad_stats(cfg: OracleConfig, grads: dict):
    """[EXT] flax_utils.TrainState.apply_loss_fn: max/min over every leaf,
    norm = L1 over leaves of the per-leaf L2 norm (target leaves are zero)."""
    leaves = [grads[net][k] for net in NETS for k in leaf_order(cfg, net)]
    gmax = max(float(l.max()) for l in leaves)
    gmin = min(float(l.min()) for l in leaves)
    gnorm = sum(float(np.sqrt((l * l).sum())) for l in leaves)
    return gmax, gmin, gnorm


def init_opt_state(params: dict) -> dict:
    return {"m": {n: {k: np.zeros_like(v) for k, v in p.items()} for n, p in params.items()},
            "v": {n: {k: np.zeros_like(v) for k, v in p.items()} for n, p in params.items()},
            "count": 0}


def update(cfg: OracleConfig, params: dict, opt: dict, batch: dict, noise: dict):
    """[EXT] FQLAgent.update: grads -> optax.adam(lr) over the whole param dict
    -> target EMA from the pre-update critic.  Returns (params', opt', info)."""
    _, info, grads = loss_and_grads(cfg, params, batch, noise)
    gmax, gmin, gnorm = grad_stats(cfg, grads)
    info.update({"grad/max": gmax, "grad/min": gmin, "grad/norm": gnorm})

    t = opt["count"] + 1
    b1, b2, eps = 0.9, 0.999, 1e-8
    bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
    new_p, new_m, new_v = {}, {}, {}
    for net in NETS:
        new_p[net], new_m[net], new_v[net] = {}, {}, {}
        for k, p in params[net].items():
            g = grads[net][k]
            m = b1 * opt["m"][net][k] + (1 - b1) * g
            v = b2 * opt["v"][net][k] + (1 - b2) * g * g
            upd = (m / bc1) / (np.sqrt(v / bc2) + eps)
            new_p[net][k] = p - cfg.lr * upd
            new_m[net][k], new_v[net][k] = m, v
    # target EMA from the OLD critic params (target_update reads self.network)
    new_p["target_critic"] = {
        k: cfg.tau * params["critic"][k] + (1 - cfg.tau) * params["target_critic"][k]
        for k in params["target_critic"]}
    return new_p, {"m": new_m, "v": new_v, "count": t}, info


def total_loss(cfg: OracleConfig, params: dict, batch: dict, noise: dict):
    """Validation path (``trainer/experiment.py:115``): losses only, 10 info keys."""
    loss, info, _ = loss_and_grads(cfg, params, batch, noise, want_grads=False)
    return loss, info


# ----------------------------------------------------------------------------
# helpers for tests / fixtures
# ----------------------------------------------------------------------------
def make_noise(cfg: OracleConfig, B: int, rng: np.random.Generator) -> dict:
    A = cfg.action_dim
    return {"z_next": rng.standard_normal((B, A)), "x0": rng.standard_normal((B, A)),
            "t": rng.uniform(0.0, 1.0, (B, 1)), "z_d": rng.standard_normal((B, A)),
            "z_metric": rng.standard_normal((B, A))}


def make_batch(cfg: OracleConfig, B: int, rng: np.random.Generator) -> dict:
    """Synthetic transitions of the SURVEY 8d shape."""
    D, A = cfg.obs_dim, cfg.action_dim
    obs = rng.standard_normal((B, D))
    rew = np.where(rng.uniform(size=B) < 0.05, 0.0, -1.0)
    return {"observations": obs,
            "actions": rng.uniform(-1 + 1e-5, 1 - 1e-5, (B, A)),
            "rewards": rew, "masks": 1.0 - (rew == 0.0),
            "next_observations": obs + 0.05 * rng.standard_normal((B, D))}


def cast_tree(tree, dtype):
    if isinstance(tree, dict):
        return {k: cast_tree(v, dtype) for k, v in tree.items()}
    if isinstance(tree, np.ndarray):
        return tree.astype(dtype)
    return tree
