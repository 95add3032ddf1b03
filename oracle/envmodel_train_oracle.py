"""CPU oracle for the env-model trainer -- TEST INFRASTRUCTURE ONLY.

float64 NumPy restatement, with hand-written backward passes, of one training
step of the reference's world-model trainers.  Used only
by ``tests/`` as the checker of ``fqlpop_emtrain_*`` (the product path never
imports it):

* multistep state predictor -- the same step on ``MultistepStatePredictor``
  (envmodel/multistep.py:31-54), backpropagation through time (``multistep_step``);
* state predictor -- ``StatePredictorTrainer.train_step``
  (envmodel/state_predictor_trainer.py:67-95) on ``BaselineStatePredictor``
  (envmodel/baseline.py:25-37) with ``state_prediction_loss``
  (envmodel/loss.py:80-111) as bound by train_env_model.py:37-44
  (reconstruction_weight = 0; the frozen termination predictor scores the
  predicted next observation when termination_weight > 0, utils/envmodel.py);
* termination predictor -- ``TerminationPredictorTrainer.train_step``
  (envmodel/termination_predictor_trainer.py:55-76) on ``TerminationPredictor``
  (envmodel/termination_predictor.py:14-21, dropout 0.1 on the input while
  training) with ``focal_loss`` (envmodel/loss.py:33-66; train_env_model.py:79);
* the optimiser -- ``optax.adam(optax.cosine_decay_schedule(init_lr, steps))``
  (state_predictor_trainer.py:57-61, termination_predictor_trainer.py:45-49):
  b1 .9, b2 .999, eps 1e-8 outside the sqrt, bias correction with count+1,
  learning rate schedule(count) with count starting at 0;
* ``eval_step`` logs (state_predictor_trainer.py:97-117,
  termination_predictor_trainer.py:78-112).

Reference quirk kept: the termination trainer passes the same ``self.rng`` to
dropout every step, so its dropout mask is one fixed [B, obs] mask; the GPU
path draws its own fixed mask (Philox) and the tests inject one mask into both.

Parity status: restated from the in-tree reference files above; jax / flax /
optax are absent here, so per-step values are unpinned by the reference itself.
The hand-written gradients are cross-checked against torch autograd in
tests/test_emtrain_cpu.py.
"""
from __future__ import annotations

import math

import numpy as np

LN_EPS = 1e-6


def _n_dense(tree: dict) -> int:
    return sum(1 for k in tree if k.startswith("Dense_"))


def _W(tree, i):
    return np.asarray(tree[f"Dense_{i}"]["kernel"], np.float64)


def _b(tree, i):
    return np.asarray(tree[f"Dense_{i}"]["bias"], np.float64)


def _relu_mlp_fwd(tree: dict, x: np.ndarray):
    """Dense + ReLU per hidden layer, last Dense linear.  Returns (out, inputs of every Dense)."""
    n = _n_dense(tree)
    ins = []
    for i in range(n):
        ins.append(x)
        x = x @ _W(tree, i) + _b(tree, i)
        if i < n - 1:
            x = np.maximum(x, 0.0)
    return x, ins


def _relu_mlp_bwd(tree: dict, ins, g_out: np.ndarray, want_params: bool = True):
    """Backward of _relu_mlp_fwd: returns (grads tree or None, grad w.r.t. the input)."""
    n = _n_dense(tree)
    grads = {}
    g = g_out
    for i in reversed(range(n)):
        if want_params:
            grads[f"Dense_{i}"] = {"kernel": ins[i].T @ g, "bias": g.sum(0)}
        g = g @ _W(tree, i).T
        if i > 0:
            g = g * (ins[i] > 0)  # ReLU': ins[i] = relu(u_{i-1}); 0 at 0 as jax.nn.relu
    return (grads if want_params else None), g


def _softplus(x):
    return np.maximum(x, 0.0) + np.log1p(np.exp(-np.abs(x)))


def sigmoid_bce(logits, labels):
    """optax.sigmoid_binary_cross_entropy: relu(x) - x z + log1p(exp(-|x|))."""
    return _softplus(logits) - logits * labels


def state_predictor_step(tree: dict, batch: dict, termination_weight: float = 0.0,
                         true_termination_weight: float = 30.0, tp_tree: dict | None = None):
    """Loss, logs and parameter grads of one state-predictor train_step
    (train_env_model.py:37-44 binding: reconstruction_weight = 0)."""
    obs = np.asarray(batch["observations"], np.float64)
    act = np.asarray(batch["actions"], np.float64)
    nxt = np.asarray(batch["next_observations"], np.float64)
    term = (np.asarray(batch["rewards"]) == 0).astype(np.float64)
    B, D = obs.shape
    x0 = np.concatenate([obs, act], -1)
    mu = x0.mean(-1, keepdims=True)
    var = np.maximum((x0 * x0).mean(-1, keepdims=True) - mu * mu, 0.0)
    rs = 1.0 / np.sqrt(var + LN_EPS)
    xhat = (x0 - mu) * rs
    ln = tree["LayerNorm_0"]
    h0 = xhat * np.asarray(ln["scale"], np.float64) + np.asarray(ln["bias"], np.float64)
    out, ins = _relu_mlp_fwd(tree, h0)
    pred = out + obs
    diff = pred - nxt
    mse = float(np.mean(diff * diff))
    tw = float(termination_weight)
    norm = 1.0 + tw  # (1 + termination_weight + reconstruction_weight), reconstruction_weight = 0
    g_pred = 2.0 * diff / (B * D)
    logs = {"next_observation_loss": mse}
    t_loss = 0.0
    if tw > 0:
        logit, tins = _relu_mlp_fwd(tp_tree, pred)
        logit = logit[:, 0]
        w = float(true_termination_weight)
        ce = sigmoid_bce(logit, term)
        tl = np.where(term == 1, ce, 0.0)
        fl = np.where(term == 0, ce, 0.0)
        t_loss = float(np.mean((w * tl + fl) / (w + 1)))
        p = 1.0 / (1.0 + np.exp(-logit))
        g_logit = np.where(term == 1, w, 1.0) / (w + 1) * (p - term) / B
        _, g_tp_in = _relu_mlp_bwd(tp_tree, tins, g_logit[:, None], want_params=False)
        g_pred = g_pred + tw * g_tp_in
        logs["termination_loss"] = t_loss
        logs["true_termination_loss"] = float(tl.sum() / term.sum()) if term.sum() > 0 else float("nan")
        logs["false_termination_loss"] = float(fl.sum() / (1 - term).sum()) if (1 - term).sum() > 0 else float("nan")
    loss = (mse + tw * t_loss) / norm
    logs["loss"] = loss
    g_pred = g_pred / norm
    grads, g_h0 = _relu_mlp_bwd(tree, ins, g_pred)
    grads["LayerNorm_0"] = {"scale": (g_h0 * xhat).sum(0), "bias": g_h0.sum(0)}
    return loss, logs, grads, pred


def _ln_fwd(x0: np.ndarray):
    mu = x0.mean(-1, keepdims=True)
    var = np.maximum((x0 * x0).mean(-1, keepdims=True) - mu * mu, 0.0)
    rs = 1.0 / np.sqrt(var + LN_EPS)
    return (x0 - mu) * rs, rs


def multistep_step(tree: dict, batch: dict, termination_weight: float = 0.0,
                   true_termination_weight: float = 30.0, tp_tree: dict | None = None):
    """Loss, logs and parameter grads of one train_step on MultistepStatePredictor
    (envmodel/multistep.py:31-54; train_env_model.py:46-66 binding, reconstruction
    weight 0): the baseline cell scanned over the T steps of [B, T, ..] sequences from
    observations[:, 0] (the carry is each step's prediction), state_prediction_loss
    (envmodel/loss.py:80-111) over all B x T predictions, gradients by
    backpropagation through time.  Returns (loss, logs, grads, predictions [B, T, D])."""
    obs = np.asarray(batch["observations"], np.float64)
    act = np.asarray(batch["actions"], np.float64)
    nxt = np.asarray(batch["next_observations"], np.float64)
    term = (np.asarray(batch["rewards"]) == 0).astype(np.float64)
    B, T, D = obs.shape
    ln = tree["LayerNorm_0"]
    scale = np.asarray(ln["scale"], np.float64)
    bias = np.asarray(ln["bias"], np.float64)
    tw = float(termination_weight)
    norm = 1.0 + tw
    w = float(true_termination_weight)
    o = obs[:, 0]
    caches, g_direct, preds = [], [], []
    sq, tl_sum, fl_sum, t_loss_sum = 0.0, 0.0, 0.0, 0.0
    for t in range(T):
        xhat, rs = _ln_fwd(np.concatenate([o, act[:, t]], -1))
        out, ins = _relu_mlp_fwd(tree, xhat * scale + bias)
        pred = out + o
        diff = pred - nxt[:, t]
        sq += float((diff * diff).sum())
        g = 2.0 * diff / (B * T * D)
        if tw > 0:
            logit, tins = _relu_mlp_fwd(tp_tree, pred)
            logit = logit[:, 0]
            z = term[:, t]
            ce = sigmoid_bce(logit, z)
            tl_sum += float(np.where(z == 1, ce, 0.0).sum())
            fl_sum += float(np.where(z == 0, ce, 0.0).sum())
            t_loss_sum += float(((w * np.where(z == 1, ce, 0.0) + np.where(z == 0, ce, 0.0)) / (w + 1)).sum())
            p = 1.0 / (1.0 + np.exp(-logit))
            g_logit = np.where(z == 1, w, 1.0) / (w + 1) * (p - z) / (B * T)
            _, g_tp_in = _relu_mlp_bwd(tp_tree, tins, g_logit[:, None], want_params=False)
            g = g + tw * g_tp_in
        caches.append((xhat, rs, ins))
        g_direct.append(g / norm)
        preds.append(pred)
        o = pred
    mse = sq / (B * T * D)
    logs = {"next_observation_loss": mse}
    t_loss = 0.0
    if tw > 0:
        t_loss = t_loss_sum / (B * T)
        n_pos, n_neg = term.sum(), (1 - term).sum()
        logs["termination_loss"] = t_loss
        logs["true_termination_loss"] = tl_sum / n_pos if n_pos > 0 else float("nan")
        logs["false_termination_loss"] = fl_sum / n_neg if n_neg > 0 else float("nan")
    loss = (mse + tw * t_loss) / norm
    logs["loss"] = loss
    grads = zeros_like_tree(tree)
    carry = np.zeros((B, D))
    for t in reversed(range(T)):
        xhat, rs, ins = caches[t]
        G = g_direct[t] + carry
        gt, g_h0 = _relu_mlp_bwd(tree, ins, G)
        for mod, d in gt.items():
            for leaf, v in d.items():
                grads[mod][leaf] += v
        grads["LayerNorm_0"]["scale"] += (g_h0 * xhat).sum(0)
        grads["LayerNorm_0"]["bias"] += g_h0.sum(0)
        gy = g_h0 * scale
        g_x0 = rs * (gy - gy.mean(-1, keepdims=True) - xhat * (gy * xhat).mean(-1, keepdims=True))
        carry = G + g_x0[:, :D]  # residual + the LayerNorm input path of the carried observation
    return loss, logs, grads, np.stack(preds, 1)


def focal_terms(logits, labels, alpha=0.25, gamma=2.0):
    """envmodel/loss.py:33-66 per-row loss and d loss_i / d logit_i."""
    p = 1.0 / (1.0 + np.exp(-logits))
    ce = sigmoid_bce(logits, labels)
    pt = np.where(labels == 1, p, 1 - p)
    af = np.where(labels == 1, alpha, 1 - alpha)
    li = af * (1.0 - pt) ** gamma * ce
    logp = -_softplus(-logits)   # log p
    log1mp = -_softplus(logits)  # log (1 - p)
    d_pos = (1 - p) ** gamma * (gamma * p * logp - (1 - p))
    d_neg = p ** gamma * (-gamma * (1 - p) * log1mp + p)
    dli = af * np.where(labels == 1, d_pos, d_neg)
    return li, dli


def termination_predictor_step(tree: dict, batch: dict, keep_mask: np.ndarray, rate: float = 0.1,
                               alpha: float = 0.25, gamma: float = 2.0):
    """Loss, logs and grads of one termination-predictor train_step: dropout
    (keep_mask [B, obs], scaled by 1 / (1 - rate)) on next_observations."""
    x = np.asarray(batch["next_observations"], np.float64) * keep_mask / (1.0 - rate)
    z = (np.asarray(batch["rewards"]) == 0).astype(np.float64)
    B = x.shape[0]
    logit, ins = _relu_mlp_fwd(tree, x)
    logit = logit[:, 0]
    li, dli = focal_terms(logit, z, alpha, gamma)
    loss = float(li.mean())
    logs = {"loss": loss,
            "true_loss": float((li * z).sum() / (z.sum() + 1e-8)),
            "false_loss": float((li * (1 - z)).sum() / ((1 - z).sum() + 1e-8))}
    grads, _ = _relu_mlp_bwd(tree, ins, (dli / B)[:, None])
    return loss, logs, grads


def termination_eval_logs(tree: dict, batch: dict, alpha: float = 0.25, gamma: float = 2.0) -> dict:
    """termination_predictor_trainer.py:78-112 (dropout off)."""
    logit, _ = _relu_mlp_fwd(tree, np.asarray(batch["next_observations"], np.float64))
    logit = logit[:, 0]
    z = (np.asarray(batch["rewards"]) == 0)
    li, _ = focal_terms(logit, z.astype(np.float64), alpha, gamma)
    pred = logit > 0
    tp = float(np.sum(pred & z))
    pp = float(np.sum(pred))
    ap = float(np.sum(z))
    zf = z.astype(np.float64)
    return {"loss": float(li.mean()),
            "true_loss": float((li * zf).sum() / (zf.sum() + 1e-8)),
            "false_loss": float((li * (1 - zf)).sum() / ((1 - zf).sum() + 1e-8)),
            "accuracy": float(np.mean(pred == z)),
            "precision": tp / pp if pp > 0 else 1.0,
            "recall": tp / ap if ap > 0 else 1.0}


def cosine_lr(init_lr: float, decay_steps: int, count: int) -> float:
    """optax.cosine_decay_schedule(init_value, decay_steps) with alpha = 0."""
    c = min(count, decay_steps)
    return init_lr * 0.5 * (1.0 + math.cos(math.pi * c / decay_steps))


def adam_update(tree: dict, grads: dict, m: dict, v: dict, count: int, lr: float):
    """optax.adam: returns (new tree, new m, new v); count = updates done so far."""
    t = count + 1
    nt, nm, nv = {}, {}, {}
    for mod in tree:
        nt[mod], nm[mod], nv[mod] = {}, {}, {}
        for leaf in tree[mod]:
            g = np.asarray(grads[mod][leaf], np.float64)
            mm = 0.9 * np.asarray(m[mod][leaf], np.float64) + 0.1 * g
            vv = 0.999 * np.asarray(v[mod][leaf], np.float64) + 0.001 * g * g
            mh = mm / (1 - 0.9 ** t)
            vh = vv / (1 - 0.999 ** t)
            nt[mod][leaf] = np.asarray(tree[mod][leaf], np.float64) - lr * mh / (np.sqrt(vh) + 1e-8)
            nm[mod][leaf], nv[mod][leaf] = mm, vv
    return nt, nm, nv


def zeros_like_tree(tree: dict) -> dict:
    return {mod: {leaf: np.zeros_like(np.asarray(x, np.float64)) for leaf, x in d.items()} for mod, d in tree.items()}
