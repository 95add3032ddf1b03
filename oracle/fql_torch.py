"""PyTorch-CPU restatement of the FQL update -- TEST / BASELINE INFRASTRUCTURE ONLY.

Two uses, both as a checker or a timed baseline, never as the product path:

* float64 + autograd: an implementation of the loss that shares no backward
  code with ``oracle/fql_oracle.py``, so ``tests/test_oracle.py`` can check the
  oracle's hand-written gradients against it;
* float32 on the host cores: ``bench.py``'s ``cpu_baseline`` (kind "port";
  BASELINE.md section 3: the JAX reference cannot run here or on the GPU box).

Semantics follow SURVEY.md Appendix A ([EXT] upstream ``fql/agents/fql.py``)
exactly as ``oracle/fql_oracle.py`` does; parity against the reference itself is
unpinned (see that module's header).
"""
from __future__ import annotations

import math

import torch

from oracle.fql_oracle import NETS, OracleConfig, leaf_order, net_has_ln

SQRT_2_OVER_PI = math.sqrt(2.0 / math.pi)


def gelu(x):
    return 0.5 * x * (1.0 + torch.tanh(SQRT_2_OVER_PI * (x + 0.044715 * x ** 3)))


def mlp(p: dict, x, ln: bool, e=None):
    n = sum(1 for k in p if k.endswith("/kernel"))
    h = x
    for i in range(n):
        W, b = p[f"Dense_{i}/kernel"], p[f"Dense_{i}/bias"]
        if e is not None:
            W, b = W[e], b[e]
        h = h @ W + b
        if i < n - 1:
            h = gelu(h)
            if ln:
                sc, bi = p[f"LayerNorm_{i}/scale"], p[f"LayerNorm_{i}/bias"]
                if e is not None:
                    sc, bi = sc[e], bi[e]
                mu = h.mean(-1, keepdim=True)
                var = torch.clamp((h * h).mean(-1, keepdim=True) - mu * mu, min=0.0)
                h = (h - mu) * torch.rsqrt(var + 1e-6) * sc + bi
    return h


def value(cfg, p, obs, act):
    x = torch.cat([obs, act], -1)
    return torch.stack([mlp(p, x, cfg.layer_norm, e)[:, 0] for e in range(cfg.num_qs)])


def actor(cfg, p, obs, act, t=None):
    parts = [obs, act] + ([t] if t is not None else [])
    return mlp(p, torch.cat(parts, -1), cfg.actor_layer_norm)


def to_torch(tree, dtype, requires_grad=False):
    out = {}
    for k, v in tree.items():
        if isinstance(v, dict):
            out[k] = to_torch(v, dtype, requires_grad)
        else:
            out[k] = torch.as_tensor(v, dtype=dtype).clone().requires_grad_(requires_grad)
    return out


def total_loss(cfg: OracleConfig, P: dict, batch: dict, noise: dict):
    """Autograd form of [EXT] FQLAgent.total_loss.  ``P`` holds leaf tensors with
    requires_grad on the trainable nets; stop-gradients as upstream."""
    s, a, s2 = batch["observations"], batch["actions"], batch["next_observations"]
    B, A = a.shape
    info = {}
    with torch.no_grad():
        a_next = torch.clamp(actor(cfg, P["actor_onestep_flow"], s2, noise["z_next"]), -1, 1)
        qt = value(cfg, P["target_critic"], s2, a_next)
        q_next = qt.min(0).values if cfg.q_agg == "min" else qt.mean(0)
        y = batch["rewards"] + cfg.discount * batch["masks"] * q_next
    q = value(cfg, P["critic"], s, a)
    critic_loss = ((q - y[None]) ** 2).mean()
    info.update({"critic/critic_loss": critic_loss, "critic/q_mean": q.mean(),
                 "critic/q_max": q.max(), "critic/q_min": q.min()})

    x0, t = noise["x0"], noise["t"]
    x_t = (1 - t) * x0 + t * a
    pred = actor(cfg, P["actor_bc_flow"], s, x_t, t)
    bc_loss = ((pred - (a - x0)) ** 2).mean()

    with torch.no_grad():
        x = noise["z_d"]
        for i in range(cfg.flow_steps):
            tt = torch.full((B, 1), float(torch.tensor(i / cfg.flow_steps, dtype=torch.float32)),
                            dtype=x.dtype)
            x = x + actor(cfg, P["actor_bc_flow"], s, x, tt) / cfg.flow_steps
        a_flow = torch.clamp(x, -1, 1)
    a_pi = actor(cfg, P["actor_onestep_flow"], s, noise["z_d"])
    distill = ((a_pi - a_flow) ** 2).mean()
    frozen = {k: v.detach() for k, v in P["critic"].items()}
    qb = value(cfg, frozen, s, torch.clamp(a_pi, -1, 1)).mean(0)
    q_loss = -qb.mean()
    if cfg.normalize_q_loss:
        q_loss = q_loss / qb.abs().mean().detach()
    actor_loss = bc_loss + cfg.alpha * distill + q_loss
    with torch.no_grad():
        a_met = torch.clamp(actor(cfg, P["actor_onestep_flow"], s, noise["z_metric"]), -1, 1)
        mse = ((a_met - a) ** 2).mean()
    info.update({"actor/actor_loss": actor_loss, "actor/bc_flow_loss": bc_loss,
                 "actor/distill_loss": distill, "actor/q_loss": q_loss,
                 "actor/q": qb.mean(), "actor/mse": mse})
    return critic_loss + actor_loss, info


class TorchFQL:
    """Stateful CPU trainer (params + Adam) used as the timed CPU baseline."""

    def __init__(self, cfg: OracleConfig, params: dict, dtype=torch.float32):
        self.cfg = cfg
        self.P = to_torch(params, dtype)
        for net in ("critic", "actor_bc_flow", "actor_onestep_flow"):
            for v in self.P[net].values():
                v.requires_grad_(True)
        self.m = {n: {k: torch.zeros_like(v) for k, v in p.items()} for n, p in self.P.items()
                  if n != "target_critic"}
        self.v = {n: {k: torch.zeros_like(v) for k, v in p.items()} for n, p in self.P.items()
                  if n != "target_critic"}
        self.count = 0

    def update(self, batch: dict, noise: dict):
        cfg = self.cfg
        for p in self.P.values():
            for v in p.values():
                v.grad = None
        loss, info = total_loss(cfg, self.P, batch, noise)
        loss.backward()
        with torch.no_grad():
            leaves = []
            for net in NETS:
                for k in leaf_order(cfg, net):
                    g = self.P[net][k].grad
                    leaves.append(torch.zeros_like(self.P[net][k]) if g is None else g)
            info["grad/max"] = max(l.max() for l in leaves)
            info["grad/min"] = min(l.min() for l in leaves)
            info["grad/norm"] = sum(torch.linalg.vector_norm(l) for l in leaves)
            old_critic = {k: v.detach().clone() for k, v in self.P["critic"].items()}
            self.count += 1
            t = self.count
            bc1, bc2 = 1 - 0.9 ** t, 1 - 0.999 ** t
            for net in ("critic", "actor_bc_flow", "actor_onestep_flow"):
                for k, p in self.P[net].items():
                    g = p.grad
                    m = self.m[net][k].mul_(0.9).add_(g, alpha=0.1)
                    v = self.v[net][k].mul_(0.999).addcmul_(g, g, value=0.001)
                    p.sub_(cfg.lr * (m / bc1) / (torch.sqrt(v / bc2) + 1e-8))
            for k, tp in self.P["target_critic"].items():
                tp.mul_(1 - cfg.tau).add_(old_critic[k], alpha=cfg.tau)
        return {k: float(v.detach()) if hasattr(v, 'detach') else float(v) for k, v in info.items()}


def grads_autograd(cfg: OracleConfig, params: dict, batch: dict, noise: dict):
    """float64 autograd gradients of total_loss (for checking the oracle)."""
    P = to_torch(params, torch.float64)
    for net in ("critic", "actor_bc_flow", "actor_onestep_flow"):
        for v in P[net].values():
            v.requires_grad_(True)
    bt = {k: torch.as_tensor(v, dtype=torch.float64) for k, v in batch.items()}
    nt = {k: torch.as_tensor(v, dtype=torch.float64) for k, v in noise.items()}
    loss, info = total_loss(cfg, P, bt, nt)
    loss.backward()
    out = {}
    for net in NETS:
        out[net] = {k: (v.grad.numpy() if v.grad is not None else torch.zeros_like(v).numpy())
                    for k, v in P[net].items()}
    return float(loss.detach()), {k: float(v.detach()) for k, v in info.items()}, out


__all__ = ["TorchFQL", "grads_autograd", "total_loss", "net_has_ln"]
