"""CPU tests of the oracle (oracle/fql_oracle.py): known answers, finite
differences, an independent autograd implementation, and the golden fixture."""
import math
import os

import numpy as np
import pytest

from oracle import fql_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def small_cfg(**kw):
    kw.setdefault("hidden_dims", (16, 16, 16, 16))
    kw.setdefault("batch_size", 8)
    return O.OracleConfig(**kw)


def test_gelu_tanh_formula_and_grad():
    x = np.linspace(-6, 6, 101)
    want = 0.5 * x * (1 + np.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * x ** 3)))
    assert np.allclose(O.gelu(x), want, rtol=0, atol=0)
    eps = 1e-6
    fd = (O.gelu(x + eps) - O.gelu(x - eps)) / (2 * eps)
    assert np.allclose(O.gelu_grad(x), fd, atol=1e-8)


def test_layer_norm_fast_variance():
    rng = np.random.default_rng(0)
    g = rng.standard_normal((4, 32)) * 3 + 1
    mu, rstd = O.layer_norm_stats(g)
    assert np.allclose(mu[:, 0], g.mean(1))
    assert np.allclose(1 / rstd[:, 0] ** 2, g.var(1) + 1e-6)
    # constant row: fast variance may round below zero -> clipped, rstd = 1/sqrt(eps)
    mu, rstd = O.layer_norm_stats(np.full((1, 8), 0.3))
    assert np.isclose(rstd[0, 0], 1 / math.sqrt(1e-6))


def test_init_shapes_and_counts():
    cfg = O.OracleConfig()
    p = O.init_params(cfg, 0)
    count = {net: sum(v.size for v in p[net].values()) for net in O.NETS}
    # 809 985 per critic member, 808 453 bc, 807 941 onestep
    assert count["critic"] == 2 * 809_985
    assert count["target_critic"] == count["critic"]
    assert count["actor_bc_flow"] == 808_453
    assert count["actor_onestep_flow"] == 807_941
    lim = math.sqrt(6 / (33 + 512))
    assert np.abs(p["critic"]["Dense_0/kernel"]).max() <= lim
    assert np.all(p["critic"]["Dense_0/bias"] == 0) and np.all(p["critic"]["LayerNorm_0/scale"] == 1)


def test_euler_with_zero_velocity_net_is_clipped_noise():
    cfg = small_cfg()
    p = O.init_params(cfg, 0)
    for k in p["actor_bc_flow"]:
        p["actor_bc_flow"][k] = np.zeros_like(p["actor_bc_flow"][k])
    z = np.random.default_rng(1).standard_normal((8, 5)) * 2
    out = O.compute_flow_actions(cfg, p, np.zeros((8, 28)), z)
    assert np.array_equal(out, np.clip(z, -1, 1))


def test_euler_constant_velocity_integrates_exactly():
    cfg = small_cfg()
    p = O.init_params(cfg, 0)
    net = p["actor_bc_flow"]
    for k in net:
        net[k] = np.zeros_like(net[k])
    net["Dense_4/bias"] = np.full(5, 0.3)  # v = 0.3 everywhere
    z = np.zeros((4, 5))
    out = O.compute_flow_actions(cfg, p, np.zeros((4, 28)), z)
    assert np.allclose(out, 0.3)


def _loss_only(cfg, params, batch, noise):
    loss, _, _ = O.loss_and_grads(cfg, params, batch, noise, want_grads=False)
    return loss


@pytest.mark.parametrize("net,key", [
    ("critic", "Dense_0/kernel"), ("critic", "LayerNorm_1/scale"), ("critic", "Dense_4/bias"),
    ("actor_bc_flow", "Dense_2/kernel"), ("actor_onestep_flow", "Dense_0/kernel"),
    ("actor_onestep_flow", "Dense_4/kernel"),
])
def test_gradients_match_finite_differences(net, key):
    # each net's own objective: critic <- critic loss (the actor's Q term reads
    # frozen critic params); bc <- BC loss (the Euler target is stop-gradient);
    # onestep <- actor loss
    cfg = small_cfg(alpha=3.0)
    rng = np.random.default_rng(7)
    params = O.init_params(cfg, 3)
    batch, noise = O.make_batch(cfg, 8, rng), O.make_noise(cfg, 8, rng)
    _, _, grads = O.loss_and_grads(cfg, params, batch, noise)
    arr = params[net][key]
    flat_idx = rng.choice(arr.size, size=min(6, arr.size), replace=False)
    eps = 1e-6

    def objective(pp):
        if net == "critic":
            _, info, _ = O.loss_and_grads(cfg, pp, batch, noise, want_grads=False)
            return info["critic/critic_loss"]
        _, info, _ = O.loss_and_grads(cfg, pp, batch, noise, want_grads=False)
        if net == "actor_bc_flow":  # the flow target (distill) is a stop-gradient path
            return info["actor/bc_flow_loss"]
        return info["actor/actor_loss"]

    for fi in flat_idx:
        idx = np.unravel_index(fi, arr.shape)
        orig = arr[idx]
        arr[idx] = orig + eps
        lp = objective(params)
        arr[idx] = orig - eps
        lm = objective(params)
        arr[idx] = orig
        fd = (lp - lm) / (2 * eps)
        g = grads[net][key][idx]
        assert abs(fd - g) <= 1e-6 + 1e-5 * abs(g), (net, key, idx, fd, g)


def test_gradients_match_torch_autograd():
    torch = pytest.importorskip("torch")  # noqa: F841
    from oracle.fql_torch import grads_autograd
    for kw in ({}, {"q_agg": "min", "normalize_q_loss": True}, {"layer_norm": False, "actor_layer_norm": True}):
        cfg = small_cfg(**kw)
        rng = np.random.default_rng(11)
        p = O.init_params(cfg, 2)
        b, n = O.make_batch(cfg, 8, rng), O.make_noise(cfg, 8, rng)
        loss, info, g = O.loss_and_grads(cfg, p, b, n)
        l2, i2, g2 = grads_autograd(cfg, p, b, n)
        assert abs(loss - l2) < 1e-10
        for k in info:
            assert abs(info[k] - i2[k]) < 1e-10, k
        for net in O.NETS:
            for k in g[net]:
                assert np.allclose(g[net][k], g2[net][k], atol=1e-11, rtol=1e-9), (kw, net, k)


def test_adam_first_step_closed_form_and_ema():
    cfg = small_cfg()
    rng = np.random.default_rng(3)
    p = O.init_params(cfg, 1)
    b, n = O.make_batch(cfg, 8, rng), O.make_noise(cfg, 8, rng)
    _, _, g = O.loss_and_grads(cfg, p, b, n)
    p1, opt, info = O.update(cfg, p, O.init_opt_state(p), b, n)
    for net in ("critic", "actor_bc_flow", "actor_onestep_flow"):
        for k in p[net]:
            gg = g[net][k]
            # step 1: m_hat = g, v_hat = g^2 -> p - lr * g / (|g| + eps)
            want = p[net][k] - cfg.lr * gg / (np.abs(gg) + 1e-8)
            assert np.allclose(p1[net][k], want, rtol=1e-9, atol=1e-14), (net, k)
    for k in p["critic"]:
        want = cfg.tau * p["critic"][k] + (1 - cfg.tau) * p["target_critic"][k]
        assert np.allclose(p1["target_critic"][k], want)
    assert opt["count"] == 1
    # grad stats include the zero target leaves
    assert info["grad/max"] >= 0.0 >= info["grad/min"]


def test_total_loss_matches_update_info():
    cfg = small_cfg()
    rng = np.random.default_rng(4)
    p = O.init_params(cfg, 1)
    b, n = O.make_batch(cfg, 8, rng), O.make_noise(cfg, 8, rng)
    loss, vinfo = O.total_loss(cfg, p, b, n)
    _, _, tinfo = O.update(cfg, p, O.init_opt_state(p), b, n)
    for k in O.VAL_INFO_KEYS:
        assert vinfo[k] == tinfo[k]
    assert np.isclose(loss, vinfo["critic/critic_loss"] + vinfo["actor/actor_loss"])


def test_oracle_reproduces_golden_fixture():
    g = np.load(os.path.join(GOLDEN, "oracle_update_h64.npz"))
    H, B, alpha = g["config"]
    cfg = O.OracleConfig(hidden_dims=(int(H),) * 4, batch_size=int(B), alpha=float(alpha))
    p = {net: {} for net in O.NETS}
    for key in g.files:
        if key.startswith("params_in/"):
            _, net, leaf = key.split("/", 2)
            p[net][leaf] = g[key].astype(np.float64)
    opt = O.init_opt_state(p)
    for step in range(2):
        b = {k.split("/", 1)[1]: g[k].astype(np.float64) for k in g.files if k.startswith(f"batch{step}/")}
        n = {k.split("/", 1)[1]: g[k].astype(np.float64) for k in g.files if k.startswith(f"noise{step}/")}
        p, opt, info = O.update(cfg, p, opt, b, n)
        got = np.array([info[k] for k in O.TRAIN_INFO_KEYS])
        assert np.allclose(got, g[f"info{step}"], rtol=1e-12, atol=1e-14)
    for key in g.files:
        if key.startswith("params_out/"):
            _, net, leaf = key.split("/", 2)
            assert np.array_equal(p[net][leaf].astype(np.float32), g[key])
