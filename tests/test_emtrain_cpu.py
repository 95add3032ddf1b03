"""CPU checks of the env-model trainer oracle (oracle/envmodel_train_oracle.py):
hand-written gradients vs torch autograd in float64, known answers of the focal
loss, the cosine schedule and the Adam step."""
import math
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flow-q-learning_amd"))

from oracle import envmodel_train_oracle as T  # noqa: E402
T_ = T
import envmodel as em  # noqa: E402


def _batch(rng, B, D, A, p_term=0.2):
    obs = rng.standard_normal((B, D))
    return {"observations": obs, "actions": rng.uniform(-1, 1, (B, A)),
            "next_observations": obs + 0.1 * rng.standard_normal((B, D)),
            "rewards": np.where(rng.uniform(size=B) < p_term, 0.0, -1.0)}


def _torch_tree(tree):
    return {m: {k: torch.tensor(np.asarray(v, np.float64), requires_grad=True) for k, v in d.items()}
            for m, d in tree.items()}


def _torch_mlp(tt, x):
    n = sum(1 for k in tt if k.startswith("Dense_"))
    for i in range(n):
        x = x @ tt[f"Dense_{i}"]["kernel"] + tt[f"Dense_{i}"]["bias"]
        if i < n - 1:
            x = torch.relu(x)
    return x


def _ln_torch(x, scale, bias):
    mu = x.mean(-1, keepdim=True)
    var = torch.clamp((x * x).mean(-1, keepdim=True) - mu * mu, min=0.0)
    return (x - mu) / torch.sqrt(var + T.LN_EPS) * scale + bias


def _bce_torch(logits, z):
    return torch.nn.functional.softplus(logits) - logits * z


@pytest.mark.parametrize("tw", [0.0, 1.0])
def test_state_predictor_grads_vs_autograd(tw):
    rng = np.random.default_rng(0)
    spec = em.EnvModelSpec(7, 3, (16, 24, 16), (12, 12))
    sp = em.init_state_predictor(spec, 1)
    sp["LayerNorm_0"]["scale"] = (1 + 0.1 * rng.standard_normal(10)).astype(np.float32)
    sp["LayerNorm_0"]["bias"] = (0.1 * rng.standard_normal(10)).astype(np.float32)
    tp = em.init_termination_predictor(spec, 2)
    b = _batch(rng, 32, 7, 3)
    loss, logs, grads, _ = T.state_predictor_step(sp, b, tw, 30.0, tp)
    tt = _torch_tree(sp)
    obs = torch.tensor(b["observations"])
    x0 = torch.cat([obs, torch.tensor(b["actions"])], -1)
    h0 = _ln_torch(x0, tt["LayerNorm_0"]["scale"], tt["LayerNorm_0"]["bias"])
    pred = _torch_mlp({k: v for k, v in tt.items() if k.startswith("Dense_")}, h0) + obs
    mse = ((pred - torch.tensor(b["next_observations"])) ** 2).mean()
    total = mse
    if tw > 0:
        ttp = {m: {k: torch.tensor(np.asarray(v, np.float64)) for k, v in d.items()} for m, d in tp.items()}
        logit = _torch_mlp(ttp, pred)[:, 0]
        z = torch.tensor((b["rewards"] == 0).astype(np.float64))
        ce = _bce_torch(logit, z)
        w = 30.0
        tl = torch.where(z == 1, ce, torch.zeros_like(ce))
        fl = torch.where(z == 0, ce, torch.zeros_like(ce))
        total = mse + tw * ((w * tl + fl) / (w + 1)).mean()
    total = total / (1 + tw)
    total.backward()
    assert abs(loss - total.item()) < 1e-12
    assert abs(logs["next_observation_loss"] - mse.item()) < 1e-12
    for m, d in tt.items():
        for k, v in d.items():
            np.testing.assert_allclose(grads[m][k], v.grad.numpy(), rtol=1e-9, atol=1e-12)


def test_termination_predictor_grads_vs_autograd():
    rng = np.random.default_rng(1)
    spec = em.EnvModelSpec(9, 2, (8, 8), (16, 32, 16))
    tp = em.init_termination_predictor(spec, 3)
    b = _batch(rng, 64, 9, 2, p_term=0.3)
    keep = rng.uniform(size=(64, 9)) >= 0.1
    loss, logs, grads = T.termination_predictor_step(tp, b, keep.astype(np.float64))
    tt = _torch_tree(tp)
    x = torch.tensor(b["next_observations"]) * torch.tensor(keep.astype(np.float64)) / 0.9
    logit = _torch_mlp(tt, x)[:, 0]
    z = torch.tensor((b["rewards"] == 0).astype(np.float64))
    p = torch.sigmoid(logit)
    ce = _bce_torch(logit, z)
    pt = torch.where(z == 1, p, 1 - p)
    af = torch.where(z == 1, torch.full_like(p, 0.25), torch.full_like(p, 0.75))
    li = af * (1 - pt) ** 2 * ce
    li.mean().backward()
    assert abs(loss - li.mean().item()) < 1e-12
    for m, d in tt.items():
        for k, v in d.items():
            np.testing.assert_allclose(grads[m][k], v.grad.numpy(), rtol=1e-8, atol=1e-12)


def test_focal_known_answers():
    # logit 0: p = 0.5, ce = log 2, (1 - pt)^2 = 0.25
    li, _ = T.focal_terms(np.array([0.0, 0.0]), np.array([1.0, 0.0]))
    np.testing.assert_allclose(li, [0.25 * 0.25 * math.log(2), 0.75 * 0.25 * math.log(2)], rtol=1e-12)
    # finite differences of the per-row derivative
    x = np.linspace(-6, 6, 25)
    for z in (0.0, 1.0):
        _, d = T.focal_terms(x, np.full_like(x, z))
        h = 1e-6
        fd = (T.focal_terms(x + h, np.full_like(x, z))[0] - T.focal_terms(x - h, np.full_like(x, z))[0]) / (2 * h)
        np.testing.assert_allclose(d, fd, rtol=1e-6, atol=1e-10)


def test_cosine_schedule_and_adam_first_step():
    assert T.cosine_lr(1e-3, 100, 0) == pytest.approx(1e-3)
    assert T.cosine_lr(1e-3, 100, 50) == pytest.approx(5e-4)
    assert T.cosine_lr(1e-3, 100, 100) == pytest.approx(0.0, abs=1e-18)
    assert T.cosine_lr(1e-3, 100, 250) == pytest.approx(0.0, abs=1e-18)
    tree = {"Dense_0": {"kernel": np.ones((2, 2)), "bias": np.zeros(2)}}
    g = {"Dense_0": {"kernel": np.array([[1.0, -2.0], [0.5, 0.0]]), "bias": np.array([3.0, -1e-3])}}
    nt, _, _ = T.adam_update(tree, g, T.zeros_like_tree(tree), T.zeros_like_tree(tree), 0, 1e-3)
    # first Adam step: -lr * g / (|g| + eps)
    want = 1.0 - 1e-3 * g["Dense_0"]["kernel"] / (np.abs(g["Dense_0"]["kernel"]) + 1e-8)
    np.testing.assert_allclose(nt["Dense_0"]["kernel"], want, rtol=1e-12)


def test_env_model_argparser_matches_reference_fixture():
    """Our get_env_model_argparser / build_env_model_config_from_args against the
    REFERENCE argparser's output (tests/golden/reference_env_model_argparser.json)."""
    import json

    import argparser
    with open(os.path.join(ROOT, "tests", "golden", "reference_env_model_argparser.json")) as f:
        cases = json.load(f)
    assert len(cases) >= 4
    for case in cases:
        cfg = argparser.build_env_model_config_from_args(argparser.get_env_model_argparser().parse_args(case["argv"]))
        d = dict(vars(cfg))
        d["save_directory"] = str(d["save_directory"])
        d["data_directory"] = str(d["data_directory"])
        d["model_config"] = {k: list(v) if isinstance(v, tuple) else v for k, v in d["model_config"].items()}
        assert d == case["config"], case["argv"]


def test_trainer_flat_layout_roundtrip():
    from envmodel.trainer import _leaf_shapes, unflatten
    spec = em.EnvModelSpec(28, 5)
    sp = em.init_state_predictor(spec, 0)
    flat = em.flatten_state_predictor(spec, sp)
    names = em.sp_leaf_names(spec)
    tree = unflatten(names, _leaf_shapes(names, spec.sp_dims(), 33), flat)
    for m in sp:
        for k in sp[m]:
            np.testing.assert_array_equal(tree[m][k], sp[m][k])
    tp = em.init_termination_predictor(spec, 1)
    names = em.tp_leaf_names(spec)
    tree = unflatten(names, _leaf_shapes(names, spec.tp_dims()), em.flatten_termination_predictor(spec, tp))
    for m in tp:
        for k in tp[m]:
            np.testing.assert_array_equal(tree[m][k], tp[m][k])


def _seq_batch(rng, B, T, D, A, p_term=0.2):
    obs = rng.standard_normal((B, T, D))
    return {"observations": obs, "actions": rng.uniform(-1, 1, (B, T, A)),
            "next_observations": obs + 0.1 * rng.standard_normal((B, T, D)),
            "rewards": np.where(rng.uniform(size=(B, T)) < p_term, 0.0, -1.0)}


@pytest.mark.parametrize("tw", [0.0, 1.0])
def test_multistep_bptt_grads_vs_autograd(tw):
    """oracle.multistep_step (hand-written BPTT) against torch autograd through the
    scanned cell (envmodel/multistep.py:31-54) in float64."""
    rng = np.random.default_rng(4)
    B, T, D, A = 3, 6, 7, 3
    spec = em.EnvModelSpec(D, A, (16, 24, 16), (12, 12))
    sp = em.init_state_predictor(spec, 1)
    sp["LayerNorm_0"]["scale"] = (1 + 0.1 * rng.standard_normal(D + A)).astype(np.float32)
    sp["LayerNorm_0"]["bias"] = (0.1 * rng.standard_normal(D + A)).astype(np.float32)
    tp = em.init_termination_predictor(spec, 2)
    b = _seq_batch(rng, B, T, D, A, p_term=0.3)
    loss, logs, grads, preds = T_.multistep_step(sp, b, tw, 30.0, tp)
    tt = _torch_tree(sp)
    ttp = {m: {k: torch.tensor(np.asarray(v, np.float64)) for k, v in d.items()} for m, d in tp.items()}
    dense = {k: v for k, v in tt.items() if k.startswith("Dense_")}
    o = torch.tensor(b["observations"][:, 0])
    act = torch.tensor(b["actions"])
    out = []
    for t in range(T):
        h0 = _ln_torch(torch.cat([o, act[:, t]], -1), tt["LayerNorm_0"]["scale"], tt["LayerNorm_0"]["bias"])
        o = _torch_mlp(dense, h0) + o
        out.append(o)
    pred = torch.stack(out, 1)
    mse = ((pred - torch.tensor(b["next_observations"])) ** 2).mean()
    total = mse
    if tw > 0:
        logit = _torch_mlp(ttp, pred)[..., 0]
        z = torch.tensor((b["rewards"] == 0).astype(np.float64))
        ce = _bce_torch(logit, z)
        tl = torch.where(z == 1, ce, torch.zeros_like(ce))
        fl = torch.where(z == 0, ce, torch.zeros_like(ce))
        total = mse + tw * ((30.0 * tl + fl) / 31.0).mean()
        assert logs["true_termination_loss"] == pytest.approx(float(tl.detach().sum() / (z == 1).sum()), rel=1e-12)
    total = total / (1 + tw)
    total.backward()
    np.testing.assert_allclose(preds, pred.detach().numpy(), rtol=1e-12, atol=1e-12)
    assert abs(loss - total.item()) < 1e-12
    assert abs(logs["next_observation_loss"] - mse.item()) < 1e-12
    for m, d in tt.items():
        for k, v in d.items():
            np.testing.assert_allclose(grads[m][k], v.grad.numpy(), rtol=1e-9, atol=1e-12, err_msg=f"{m}/{k}")


def test_multistep_one_step_is_the_baseline_step():
    rng = np.random.default_rng(5)
    spec = em.EnvModelSpec(9, 2, (8, 8))
    sp = em.init_state_predictor(spec, 3)
    b = _seq_batch(rng, 4, 1, 9, 2)
    l1, _, g1, _ = T_.multistep_step(sp, b)
    l0, _, g0, _ = T_.state_predictor_step(sp, {k: v[:, 0] for k, v in b.items()})
    assert l1 == pytest.approx(l0, rel=1e-13)
    for m in g0:
        for k in g0[m]:
            np.testing.assert_allclose(g1[m][k], g0[m][k], rtol=1e-12, atol=1e-15)


def test_multistep_loader_windows_like_reference():
    """train_env_model.MultistepLoader = utils/data_loader.py:25-39: [n/1000][1000] episodes,
    windows of T consecutive steps inside one episode, start in [0, 1000 - T)."""
    import train_env_model as tem
    n, D, A, T = 3000, 3, 2, 16
    rows = np.arange(n, dtype=np.float32)
    ds = {"observations": np.repeat(rows[:, None], D, 1), "actions": np.zeros((n, A), np.float32),
          "rewards": rows.copy(), "next_observations": np.repeat(rows[:, None] + 1, D, 1)}
    ld = tem.MultistepLoader(ds, T)
    assert ld.dataset["observations"].shape == (3, 1000, D) and ld.dataset["rewards"].shape == (3, 1000)
    np.random.seed(1)
    b = ld.sample(64)
    assert b["observations"].shape == (64, T, D) and b["rewards"].shape == (64, T)
    first = b["rewards"][:, 0]
    np.testing.assert_array_equal(b["rewards"], first[:, None] + np.arange(T))  # consecutive steps
    start = first % 1000
    assert (start >= 0).all() and (start < 1000 - T).all()  # never crosses an episode boundary
    np.testing.assert_array_equal(b["next_observations"][..., 0], b["rewards"] + 1)
    with pytest.raises(ValueError):
        tem.MultistepLoader({k: v[:2500] for k, v in ds.items()}, T)
