"""HIP path vs the CPU oracle (oracle/fql_oracle.py, float64) on identical
batches, noise and initial parameters, called through the C ABI.

Tolerance (north_star): per-step losses / Q statistics within 1e-4 relative
(with an absolute floor of 1e-6 * scale for values near zero).  Parameters
after Adam: Adam's update m/(sqrt(v)+eps) ~ sign(g) at step 1, so a gradient
element whose fp32 value is a rounding-level cancellation can flip the step of
that element by up to 2*lr; we require the vast majority of elements to agree
to 1e-6 absolute and every element to stay within 2*lr + 1e-6.
"""
import numpy as np
import pytest

from oracle import fql_oracle as O

pytestmark = pytest.mark.gpu

REL = 1e-4


def _cfgs(H, B, alpha, **kw):
    ocfg = O.OracleConfig(hidden_dims=(H,) * 4, batch_size=B, alpha=alpha, **kw)
    return ocfg


def _pop(H, B, alphas, seeds, use_graph=True, **kw):
    from fqlpop import Population, PopulationConfig
    kw = {"obs_dim": 28, "action_dim": 5, **kw}
    pc = PopulationConfig(hidden_dims=(H,) * 4, batch_size=B, use_graph=use_graph, **kw)
    return Population(pc, alphas, seeds)


def _f32(tree):
    return O.cast_tree(O.cast_tree(tree, np.float32), np.float64)


def _close(a, b, rel=REL, floor=1e-6):
    return abs(a - b) <= rel * max(abs(a), abs(b)) + floor


def _check_info(got, want, keys, tag):
    bad = []
    for k in keys:
        g, w = got[k], float(want[k])
        scale = 1.0 if not k.startswith("grad/") else 1.0
        if not _close(g, w, floor=1e-6 * scale):
            bad.append(f"{k}: gpu={g:.8g} oracle={w:.8g} rel={abs(g - w) / max(abs(w), 1e-30):.3g}")
    assert not bad, f"{tag}:\n" + "\n".join(bad)


def _check_params(got_tree, want_tree, lr, tag):
    n_bad, n_tot, worst = 0, 0, 0.0
    for net in O.NETS:
        for k, w in want_tree[net].items():
            g = got_tree[net][k]
            d = np.abs(g.astype(np.float64) - w)
            worst = max(worst, float(d.max()))
            n_bad += int((d > 1e-6 + 1e-5 * np.abs(w)).sum())
            n_tot += d.size
    assert worst <= 2 * lr + 1e-5, f"{tag}: max |param diff| {worst}"
    assert n_bad <= max(5, 1e-3 * n_tot), f"{tag}: {n_bad}/{n_tot} params differ"


def _run_parity(H, B, alphas, n_steps, use_graph=True, **kw):
    seeds = [11 + i for i in range(len(alphas))]
    pop = _pop(H, B, alphas, seeds, use_graph=use_graph, **{k: v for k, v in kw.items()})
    ocfgs = [_cfgs(H, B, a, **kw) for a in alphas]
    params = [_f32(O.init_params(ocfgs[i], 100 + i)) for i in range(len(alphas))]
    opts = [O.init_opt_state(p) for p in params]
    for i, p in enumerate(params):
        pop.set_params(i, O.cast_tree(p, np.float32))
    rng = np.random.default_rng(1234)
    for step in range(n_steps):
        batches = [O.cast_tree(O.make_batch(ocfgs[0], B, rng), np.float32) for _ in alphas]
        noises = [O.cast_tree(O.make_noise(ocfgs[0], B, rng), np.float32) for _ in alphas]
        pop.step_injected(batches, noises)
        info = pop.read_info("train")
        for i in range(len(alphas)):
            b64 = O.cast_tree(batches[i], np.float64)
            n64 = O.cast_tree(noises[i], np.float64)
            params[i], opts[i], oinfo = O.update(ocfgs[i], params[i], opts[i], b64, n64)
            _check_info(info[i], oinfo, O.TRAIN_INFO_KEYS, f"step {step} member {i}")
    for i in range(len(alphas)):
        _check_params(pop.get_params(i), params[i], ocfgs[i].lr, f"member {i}")
        assert pop.get_count(i) == n_steps
    return pop


def test_update_parity_small_eager():
    _run_parity(64, 64, [3.0, 100.0], n_steps=3, use_graph=False)


def test_update_parity_small_graph():
    _run_parity(64, 64, [10.0], n_steps=2, use_graph=True)


def test_update_parity_full_size():
    """BASELINE config C2 shapes: H=512, B=256, obs 28, act 5."""
    _run_parity(512, 256, [10.0, 216.8], n_steps=1)


def test_update_parity_q_min_normalized():
    _run_parity(64, 64, [30.0], n_steps=2, q_agg="min", normalize_q_loss=True)


@pytest.mark.parametrize("H,B,kw", [
    (128, 64, dict(layer_norm=False)),            # critic without LayerNorm
    (256, 128, dict(flow_steps=3, discount=0.995)),  # antsoccer reproduce discount
    (1024, 64, dict()),                           # widest supported hidden dim
    (64, 192, dict(q_agg="min", tau=0.05)),       # odd multiple of 64 rows
    (512, 64, dict(flow_steps=3)),                # persistent Euler kernel, short flow
    (512, 192, dict(layer_norm=False, q_agg="min")),  # persistent Euler kernel, 12 column tiles
])
def test_update_parity_configs(H, B, kw):
    _run_parity(H, B, [4.0, 40.0], n_steps=2, **kw)


@pytest.mark.parametrize("D,A", [(26, 5), (27, 5), (30, 5), (31, 5)])
def test_update_parity_layer0_widths(D, A):
    """Layer-0 widths around the streamed kernels' k-step split (one ring pass of 8 k-steps =
    32 input rows, plus one tail k-step up to 36 rows; wider inputs run two ring passes):
    the Euler / BC input is K0 = D + A + 1 rows (32, 33, 36, 37 here), the critic's and the
    one-step actor's K0 = D + A (31, 32, 35, 36)."""
    _run_parity(512, 64, [7.0], n_steps=1, obs_dim=D, action_dim=A)


def test_update_parity_ant_full_size():
    """BASELINE config C3 shapes: obs 42, act 8, H=512, B=1024 (one step)."""
    from fqlpop import Population, PopulationConfig
    H, B = 512, 1024
    ocfg = O.OracleConfig(obs_dim=42, action_dim=8, hidden_dims=(H,) * 4, batch_size=B, alpha=10.0,
                          discount=0.995)
    pop = Population(PopulationConfig(obs_dim=42, action_dim=8, hidden_dims=(H,) * 4, batch_size=B,
                                      discount=0.995), [10.0], [3])
    p = _f32(O.init_params(ocfg, 21))
    o = O.init_opt_state(p)
    pop.set_params(0, O.cast_tree(p, np.float32))
    rng = np.random.default_rng(77)
    b = O.cast_tree(O.make_batch(ocfg, B, rng), np.float32)
    n = O.cast_tree(O.make_noise(ocfg, B, rng), np.float32)
    pop.step_injected([b], [n])
    p, o, oinfo = O.update(ocfg, p, o, O.cast_tree(b, np.float64), O.cast_tree(n, np.float64))
    _check_info(pop.read_info()[0], oinfo, O.TRAIN_INFO_KEYS, "ant full")
    _check_params(pop.get_params(0), p, ocfg.lr, "ant full")


def test_unsupported_configs_fail_loudly():
    from fqlpop import Population, PopulationConfig
    from fqlpop._lib import FqlpopError
    for kw in (dict(actor_layer_norm=True), dict(hidden_dims=(96,) * 4), dict(batch_size=100)):
        base = dict(hidden_dims=(64,) * 4, batch_size=64)
        base.update(kw)
        with pytest.raises(FqlpopError):
            Population(PopulationConfig(**base), [1.0], [0])


def test_update_parity_ant_shape():
    """antsoccer shapes (obs 42, act 8) at reduced width, B=128."""
    from fqlpop import Population, PopulationConfig
    H, B = 64, 128
    ocfg = O.OracleConfig(obs_dim=42, action_dim=8, hidden_dims=(H,) * 4, batch_size=B, alpha=5.53)
    pop = Population(PopulationConfig(obs_dim=42, action_dim=8, hidden_dims=(H,) * 4, batch_size=B),
                     [5.53], [7])
    p = _f32(O.init_params(ocfg, 5))
    o = O.init_opt_state(p)
    pop.set_params(0, O.cast_tree(p, np.float32))
    rng = np.random.default_rng(9)
    for step in range(2):
        b = O.cast_tree(O.make_batch(ocfg, B, rng), np.float32)
        n = O.cast_tree(O.make_noise(ocfg, B, rng), np.float32)
        pop.step_injected([b], [n])
        p, o, oinfo = O.update(ocfg, p, o, O.cast_tree(b, np.float64), O.cast_tree(n, np.float64))
        _check_info(pop.read_info()[0], oinfo, O.TRAIN_INFO_KEYS, f"ant step {step}")
    _check_params(pop.get_params(0), p, ocfg.lr, "ant")


def test_total_loss_parity():
    H, B = 64, 64
    pop = _pop(H, B, [10.0, 50.0], [1, 2])
    ocfg = _cfgs(H, B, 10.0)
    rng = np.random.default_rng(5)
    ps = [_f32(O.init_params(ocfg, 7 + i)) for i in range(2)]
    for i in range(2):
        pop.set_params(i, O.cast_tree(ps[i], np.float32))
    batches = [O.cast_tree(O.make_batch(ocfg, B, rng), np.float32) for _ in range(2)]
    noises = [O.cast_tree(O.make_noise(ocfg, B, rng), np.float32) for _ in range(2)]
    info = pop.total_loss(batches, noises)
    for i, a in enumerate([10.0, 50.0]):
        c = _cfgs(H, B, a)
        _, oinfo = O.total_loss(c, ps[i], O.cast_tree(batches[i], np.float64), O.cast_tree(noises[i], np.float64))
        _check_info(info[i], oinfo, O.VAL_INFO_KEYS, f"val member {i}")
    # total_loss must not update anything
    assert pop.get_count(0) == 0
    got = pop.get_params(0)
    assert np.array_equal(got["critic"]["Dense_1/kernel"], O.cast_tree(ps[0], np.float32)["critic"]["Dense_1/kernel"])


def test_sample_actions_parity():
    H, B = 64, 64
    pop = _pop(H, B, [10.0], [3])
    ocfg = _cfgs(H, B, 10.0)
    p = _f32(O.init_params(ocfg, 3))
    pop.set_params(0, O.cast_tree(p, np.float32))
    rng = np.random.default_rng(0)
    obs = rng.standard_normal((50, 28)).astype(np.float32)
    z = rng.standard_normal((50, 5)).astype(np.float32)
    got = pop.sample_actions(0, obs, noise=z)
    want = O.sample_actions(ocfg, p, obs.astype(np.float64), z.astype(np.float64))
    assert np.allclose(got, want, rtol=1e-4, atol=1e-5)
    # device RNG path: deterministic per seed, in [-1, 1]
    a1 = pop.sample_actions(0, obs, seed=42)
    a2 = pop.sample_actions(0, obs, seed=42)
    assert np.array_equal(a1, a2) and np.all(np.abs(a1) <= 1.0)


def test_state_roundtrip_and_target_ema():
    H, B = 64, 64
    pop = _pop(H, B, [10.0], [3])
    ocfg = _cfgs(H, B, 10.0)
    p = O.cast_tree(O.init_params(ocfg, 1), np.float32)
    p["target_critic"] = {k: v * 0.5 for k, v in p["target_critic"].items()}
    pop.set_params(0, p)
    got = pop.get_params(0)
    for net in O.NETS:
        for k in p[net]:
            assert np.array_equal(got[net][k], p[net][k]), (net, k)
    rng = np.random.default_rng(3)
    b = O.cast_tree(O.make_batch(ocfg, B, rng), np.float32)
    n = O.cast_tree(O.make_noise(ocfg, B, rng), np.float32)
    pop.step_injected([b], [n])
    after = pop.get_params(0)
    for k in p["critic"]:
        want = 0.005 * p["critic"][k].astype(np.float64) + 0.995 * p["target_critic"][k].astype(np.float64)
        assert np.allclose(after["target_critic"][k], want, rtol=1e-6, atol=1e-7), k


def test_device_sampling_deterministic_and_graph_matches_eager():
    H, B = 64, 64
    rng = np.random.default_rng(0)
    N = 5000
    obs = rng.standard_normal((N, 28)).astype(np.float32)
    rew = np.where(rng.uniform(size=N) < 0.05, 0.0, -1.0).astype(np.float32)
    data = {"observations": obs, "actions": rng.uniform(-1, 1, (N, 5)).astype(np.float32),
            "rewards": rew, "masks": (1.0 - (rew == 0)).astype(np.float32),
            "next_observations": (obs + 0.05 * rng.standard_normal((N, 28))).astype(np.float32)}
    outs = []
    for use_graph in (True, False, True):
        pop = _pop(H, B, [3.0, 30.0, 300.0], [5, 6, 7], use_graph=use_graph)
        pop.set_dataset(data)
        pop.step(4)
        info = pop.read_info_array()
        assert np.all(np.isfinite(info[:, :13]))
        outs.append((info.copy(), pop.get_flat(1)))
        assert pop.get_count(2) == 4
        pop.close()
    for info, flat in outs[1:]:
        assert np.array_equal(info, outs[0][0])
        assert np.array_equal(flat, outs[0][1])


def test_set_active_subset_matches_full_population():
    """Pruned members stay frozen; survivors compute exactly what they would
    in the full population (members are independent)."""
    H, B = 64, 64
    ocfg = _cfgs(H, B, 10.0)
    rng = np.random.default_rng(2)
    batches = [O.cast_tree(O.make_batch(ocfg, B, rng), np.float32) for _ in range(3)]
    noises = [O.cast_tree(O.make_noise(ocfg, B, rng), np.float32) for _ in range(3)]
    full = _pop(H, B, [3.0, 30.0, 300.0], [5, 6, 7])
    full.step_injected(batches, noises)
    sub = _pop(H, B, [3.0, 30.0, 300.0], [5, 6, 7])
    before0 = sub.get_flat(0)
    sub.set_active([0, 1, 1])
    sub.step_injected(batches[1:], noises[1:])
    assert np.array_equal(sub.get_flat(0), before0)
    assert np.array_equal(sub.get_flat(2), full.get_flat(2))
    assert sub.get_count(0) == 0 and sub.get_count(1) == 1


def test_euler_fused_matches_per_layer_path(monkeypatch):
    """The persistent Euler-flow kernel (H = 512) and the per-layer launches
    give the same update to within fp32 reassociation."""
    infos = []
    for flag in ("1", "0"):
        monkeypatch.setenv("FQLPOP_EULER", flag)
        pop = _run_parity(512, 64, [25.0], n_steps=1)
        infos.append(pop.read_info("train")[0])
    for k in O.TRAIN_INFO_KEYS:
        assert _close(infos[0][k], infos[1][k], rel=2e-5), (k, infos[0][k], infos[1][k])


def test_same_seed_members_with_different_alphas_draw_different_batches():
    """The device sampler is keyed by (seed, alpha): two members sharing a seed
    (tune_alpha.py's default --number_of_seeds=1 gives every alpha the same seed)
    draw different minibatches, as the reference's members do from the global
    np.random stream.  Step 1's critic statistics depend only on the batch and the
    (identical, same-seed) initial parameters, so they must differ; a member keyed
    like another (same seed and alpha) draws bit-identical batches."""
    H, B = 64, 64
    rng = np.random.default_rng(4)
    N = 5000
    obs = rng.standard_normal((N, 28)).astype(np.float32)
    rew = np.where(rng.uniform(size=N) < 0.05, 0.0, -1.0).astype(np.float32)
    data = {"observations": obs, "actions": rng.uniform(-1, 1, (N, 5)).astype(np.float32),
            "rewards": rew, "masks": (1.0 - (rew == 0)).astype(np.float32),
            "next_observations": (obs + 0.05 * rng.standard_normal((N, 28))).astype(np.float32)}
    pop = _pop(H, B, [3.0, 30.0, 3.0], [9, 9, 9])
    pop.set_dataset(data)
    assert np.array_equal(pop.get_flat(0), pop.get_flat(1))  # same seed -> same init
    pop.step(1)
    info = pop.read_info("train")
    crit = ("critic/critic_loss", "critic/q_mean", "critic/q_max", "critic/q_min")
    assert all(info[0][k] != info[1][k] for k in crit), (info[0], info[1])
    assert all(info[0][k] == info[2][k] for k in crit)
    assert np.array_equal(pop.get_flat(0), pop.get_flat(2))


def _sampled_run(H, B, steps, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(7)
    N = 4000
    obs = rng.standard_normal((N, 28)).astype(np.float32)
    rew = np.where(rng.uniform(size=N) < 0.05, 0.0, -1.0).astype(np.float32)
    data = {"observations": obs, "actions": rng.uniform(-1, 1, (N, 5)).astype(np.float32),
            "rewards": rew, "masks": (1.0 - (rew == 0)).astype(np.float32),
            "next_observations": (obs + 0.05 * rng.standard_normal((N, 28))).astype(np.float32)}
    pop = _pop(H, B, [3.0, 30.0, 300.0], [5, 6, 7])
    pop.set_dataset(data)
    pop.step(steps)
    out = (pop.read_info_array().copy(), [pop.get_flat(i, w) for i in range(3) for w in (0, 1, 2)])
    pop.close()
    for k in env:
        monkeypatch.delenv(k)
    return out


@pytest.mark.parametrize("H,B", [(512, 256), (256, 64)])
def test_fused_dw_optimiser_occupancy_variants_bit_identical(monkeypatch, H, B):
    """The fused dW + optimiser launch at 4 blocks per CU (tile 10, the default) and
    at 3 (tile 6) run the same body: parameters, Adam state, target and grad stats
    are bit-identical after several device-sampled steps."""
    ref = _sampled_run(H, B, 3, {"FQLPOP_DW_TILE_C": "6", "FQLPOP_DW_TILE_A": "6"}, monkeypatch)
    got = _sampled_run(H, B, 3, {}, monkeypatch)
    assert np.array_equal(got[0], ref[0])
    for a, b in zip(got[1], ref[1]):
        assert np.array_equal(a, b)
