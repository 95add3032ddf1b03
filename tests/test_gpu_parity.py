"""HIP path vs the CPU oracle (oracle/fql_oracle.py, float64) on identical
batches, noise and initial parameters, called through the C ABI.

Tolerance (north_star): per-step losses / Q statistics within 1e-4 relative
(with an absolute floor of 1e-6 for values near zero).  After every step:
Adam moments m and v of every leaf within 2.5e-4 of the leaf's scale (every gradient
element), and the optimiser step of every leaf exact against optax.adam / the EMA
applied to the GPU's own previous state (tests/_helpers.OptimiserChecker).
"""
import numpy as np
import pytest

from oracle import fql_oracle as O
from _helpers import OptimiserChecker, engine_options

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


def _run_parity(H, B, alphas, n_steps, use_graph=True, **kw):
    seeds = [11 + i for i in range(len(alphas))]
    pop = _pop(H, B, alphas, seeds, use_graph=use_graph, **{k: v for k, v in kw.items()})
    ocfgs = [_cfgs(H, B, a, **kw) for a in alphas]
    params = [_f32(O.init_params(ocfgs[i], 100 + i)) for i in range(len(alphas))]
    opts = [O.init_opt_state(p) for p in params]
    for i, p in enumerate(params):
        pop.set_params(i, O.cast_tree(p, np.float32))
    rng = np.random.default_rng(1234)
    checks = [OptimiserChecker(pop, i, ocfgs[i].lr, ocfgs[i].tau) for i in range(len(alphas))]
    for step in range(n_steps):
        batches = [O.cast_tree(O.make_batch(ocfgs[0], B, rng), np.float32) for _ in alphas]
        noises = [O.cast_tree(O.make_noise(ocfgs[0], B, rng), np.float32) for _ in alphas]
        for c in checks:
            c.before()
        pop.step_injected(batches, noises)
        info = pop.read_info("train")
        for i in range(len(alphas)):
            b64 = O.cast_tree(batches[i], np.float64)
            n64 = O.cast_tree(noises[i], np.float64)
            params[i], opts[i], oinfo = O.update(ocfgs[i], params[i], opts[i], b64, n64)
            _check_info(info[i], oinfo, O.TRAIN_INFO_KEYS, f"step {step} member {i}")
            checks[i].after(params[i], opts[i], step + 1, f"step {step} member {i}")
    for i in range(len(alphas)):
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
    chk = OptimiserChecker(pop, 0, ocfg.lr, ocfg.tau)
    chk.before()
    pop.step_injected([b], [n])
    p, o, oinfo = O.update(ocfg, p, o, O.cast_tree(b, np.float64), O.cast_tree(n, np.float64))
    _check_info(pop.read_info()[0], oinfo, O.TRAIN_INFO_KEYS, "ant full")
    chk.after(p, o, 1, "ant full")


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
    chk = OptimiserChecker(pop, 0, ocfg.lr, ocfg.tau)
    for step in range(2):
        b = O.cast_tree(O.make_batch(ocfg, B, rng), np.float32)
        n = O.cast_tree(O.make_noise(ocfg, B, rng), np.float32)
        chk.before()
        pop.step_injected([b], [n])
        p, o, oinfo = O.update(ocfg, p, o, O.cast_tree(b, np.float64), O.cast_tree(n, np.float64))
        _check_info(pop.read_info()[0], oinfo, O.TRAIN_INFO_KEYS, f"ant step {step}")
        chk.after(p, o, step + 1, f"ant step {step}")


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


def test_euler_fused_matches_per_layer_path():
    """The persistent Euler-flow kernel (H = 512) and the per-layer launches
    (engine option euler_fused = 0) give the same update to within fp32 reassociation."""
    infos = []
    for flag in (1, 0):
        with engine_options(euler_fused=flag):
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


def _sampled_run(H, B, steps, opts):
    with engine_options(**opts):
        return _sampled_run_now(H, B, steps)


def _sampled_run_now(H, B, steps, calls=None, probe=False):
    rng = np.random.default_rng(7)
    N = 4000
    obs = rng.standard_normal((N, 28)).astype(np.float32)
    rew = np.where(rng.uniform(size=N) < 0.05, 0.0, -1.0).astype(np.float32)
    data = {"observations": obs, "actions": rng.uniform(-1, 1, (N, 5)).astype(np.float32),
            "rewards": rew, "masks": (1.0 - (rew == 0)).astype(np.float32),
            "next_observations": (obs + 0.05 * rng.standard_normal((N, 28))).astype(np.float32)}
    pop = _pop(H, B, [3.0, 30.0, 300.0], [5, 6, 7])
    pop.set_dataset(data)
    if probe:
        pop.set_probe(True)
    for n in calls or [steps]:
        pop.step(n)
    out = (pop.read_info_array().copy(), [pop.get_flat(i, w) for i in range(3) for w in (0, 1, 2)])
    if probe:
        out = out + (pop.read_probe(), [pop.get_count(i) for i in range(3)])
    pop.close()
    return out


# (the fused dW + optimiser runs at H = 512 only: the streamed backward needs it)
@pytest.mark.parametrize("H,B,tile", [(512, 256, 6), (512, 64, 6)])
def test_fused_dw_optimiser_variants_bit_identical(H, B, tile):
    """The fused dW + optimiser launch at 4 blocks per CU (tile 10, the default) and at 3
    (tile 6) run the same arithmetic: parameters, Adam state, target and grad stats are
    bit-identical after several device-sampled steps."""
    ref = _sampled_run(H, B, 3, {"dw_tile_critic": tile, "dw_tile_actor": tile})
    got = _sampled_run(H, B, 3, {})
    assert np.array_equal(got[0], ref[0])
    for a, b in zip(got[1], ref[1]):
        assert np.array_equal(a, b)


def _synthetic_rows(N, D, A, seed):
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((N, D)).astype(np.float32)
    rew = np.where(rng.uniform(size=N) < 0.05, 0.0, -1.0).astype(np.float32)
    return {"observations": obs, "actions": rng.uniform(-1 + 1e-5, 1 - 1e-5, (N, A)).astype(np.float32),
            "rewards": rew, "masks": (1.0 - (rew == 0)).astype(np.float32),
            "next_observations": (obs + 0.05 * rng.standard_normal((N, D))).astype(np.float32)}


_C2_ALPHAS = np.logspace(np.log10(3), np.log10(1000), 16).tolist()   # bench.py / tune_alpha.py:43-45


@pytest.mark.parametrize("D,A,B,alphas,steps,kw,check", [
    (28, 5, 256, [10.0, 216.8], 3, {}, None),               # C2 shapes, 2 members: the split launches (auto)
    (28, 5, 256, _C2_ALPHAS, 2, {}, None),                  # BASELINE C2: the benchmarked 16-member population
    (42, 8, 1024, [31.6], 3, dict(discount=0.995), None),   # BASELINE C3 shapes (antsoccer)
    (42, 8, 1024, _C2_ALPHAS[::4], 2, dict(discount=0.995), None),  # C3, 4 members
    # BASELINE C3 itself: the full 16-member antsoccer population at B = 1024 steps on the
    # device; every other member (slots 0, 2, ..., 14) is oracle-checked (2.5-6 s of float64
    # oracle per member-step: all 16 would keep the test silent for up to 1.5 minutes)
    (42, 8, 1024, _C2_ALPHAS, 1, dict(discount=0.995), list(range(0, 16, 2))),
])
def test_production_step_matches_oracle_on_its_own_draws(D, A, B, alphas, steps, kw, check):
    """fqlpop_step -- the path Trainer and bench.py run -- against the oracle: the device
    sampler's rows, flow times and noises are reproduced on the host (tests/philox_np.py,
    Philox4x32-10 pinned to the Random123 known answers), the oracle updates on
    dataset[idx] with those noises, and all 13 info values of EVERY member (slot-dependent
    indexing: the 16-member case covers slots 0-15, two members per XCD) must agree to 1e-4
    at every step, and so must every leaf's Adam moments and optimiser step."""
    from fqlpop import Population, PopulationConfig
    from philox_np import draw, sample_key
    H, N = 512, 100_003
    data = _synthetic_rows(N, D, A, 5)
    pop = Population(PopulationConfig(obs_dim=D, action_dim=A, hidden_dims=(H,) * 4, batch_size=B, **kw),
                     alphas, [17 + i for i in range(len(alphas))])
    pop.set_dataset(data)
    ocfgs = [O.OracleConfig(obs_dim=D, action_dim=A, hidden_dims=(H,) * 4, batch_size=B, alpha=a, **kw)
             for a in alphas]
    params = [_f32(O.init_params(ocfgs[i], 300 + i)) for i in range(len(alphas))]
    opts = [O.init_opt_state(p) for p in params]
    for i, p in enumerate(params):
        pop.set_params(i, O.cast_tree(p, np.float32))
    keys = [sample_key(int(pop.seeds[i]), float(pop.alphas[i])) for i in range(len(alphas))]
    d64 = O.cast_tree(data, np.float64)
    members = list(range(len(alphas))) if check is None else check
    checks = {i: OptimiserChecker(pop, i, ocfgs[i].lr, ocfgs[i].tau) for i in members}
    for step in range(steps):
        for c in checks.values():
            c.before()
        pop.step(1)
        info = pop.read_info("train")
        for i in members:
            idx, noise = draw(keys[i], step, B, N, A)
            batch = {k: v[idx] for k, v in d64.items()}
            params[i], opts[i], oinfo = O.update(ocfgs[i], params[i], opts[i], batch, noise)
            _check_info(info[i], oinfo, O.TRAIN_INFO_KEYS, f"sampled step {step} member {i}")
            checks[i].after(params[i], opts[i], step + 1, f"sampled step {step} member {i}")
    pop.close()


def test_device_init_properties():
    """FQLAgent.create's init on device (a15; SURVEY Appendix A, build-defined): every
    Dense kernel ~ U(+-sqrt(6 / (fan_in + fan_out))) (inside the bound, mean ~ 0, variance
    ~ bound^2 / 3), zero biases, LayerNorm scale 1 and bias 0, target_critic == critic,
    Adam moments and count zero; members with different seeds differ."""
    from fqlpop import Population, PopulationConfig
    from fqlpop._lib import STATE_ADAM_M, STATE_ADAM_V
    H = 512
    pop = Population(PopulationConfig(hidden_dims=(H,) * 4, batch_size=256), [3.0, 10.0], [1, 2])
    dims = {"critic": [33, H, H, H, H, 1], "target_critic": [33, H, H, H, H, 1],
            "actor_bc_flow": [34, H, H, H, H, 5], "actor_onestep_flow": [33, H, H, H, H, 5]}
    trees = [pop.get_params(i) for i in range(2)]
    for tree in trees:
        for net, dd in dims.items():
            for l in range(len(dd) - 1):
                w = tree[net][f"Dense_{l}/kernel"].astype(np.float64)
                lim = np.sqrt(6.0 / (dd[l] + dd[l + 1]))
                assert w.shape[-2:] == (dd[l], dd[l + 1]), (net, l, w.shape)
                assert np.abs(w).max() <= lim * (1 + 1e-6), (net, l)
                if w.size >= 1000:
                    assert abs(w.mean()) < 0.05 * lim and abs(w.var() / (lim * lim / 3) - 1) < 0.05, (net, l)
                assert np.all(tree[net][f"Dense_{l}/bias"] == 0)
                if net in ("critic", "target_critic") and l < len(dd) - 2:
                    assert np.all(tree[net][f"LayerNorm_{l}/scale"] == 1)
                    assert np.all(tree[net][f"LayerNorm_{l}/bias"] == 0)
            for k in tree["critic"]:
                assert np.array_equal(tree["critic"][k], tree["target_critic"][k]), k
        # the two critic ensemble members are initialised independently
        assert not np.array_equal(tree["critic"]["Dense_1/kernel"][0], tree["critic"]["Dense_1/kernel"][1])
    assert not np.array_equal(trees[0]["actor_bc_flow"]["Dense_1/kernel"], trees[1]["actor_bc_flow"]["Dense_1/kernel"])
    for i in range(2):
        assert pop.get_count(i) == 0
        assert not np.any(pop.get_flat(i, STATE_ADAM_M)) and not np.any(pop.get_flat(i, STATE_ADAM_V))
    pop.close()
