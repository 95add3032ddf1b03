"""GPU parity of the env-model trainer (fqlpop_emtrain_*)
against the float64 restatement in oracle/envmodel_train_oracle.py: injected
batches, logs and parameters after every step; device sampling: determinism
and a loss that falls on a learnable synthetic dynamics."""
import numpy as np
import pytest

import envmodel as em
from envmodel.trainer import EnvModelTrainerConfig, StatePredictorTrainer, TerminationPredictorTrainer
from oracle import envmodel_train_oracle as T

T_ = T

pytestmark = pytest.mark.gpu


def _batch(rng, B, D, A, p_term=0.25):
    obs = rng.standard_normal((B, D)).astype(np.float32)
    return {"observations": obs, "actions": rng.uniform(-1, 1, (B, A)).astype(np.float32),
            "next_observations": (obs + 0.1 * rng.standard_normal((B, D))).astype(np.float32),
            "rewards": np.where(rng.uniform(size=B) < p_term, 0.0, -1.0).astype(np.float32)}


def _f64(tree):
    return {m: {k: np.asarray(v, np.float64) for k, v in d.items()} for m, d in tree.items()}


def _assert_tree_close(got, want, rtol, atol):
    for m in want:
        for k in want[m]:
            np.testing.assert_allclose(got[m][k], want[m][k], rtol=rtol, atol=atol, err_msg=f"{m}/{k}")


def _assert_moments_close(tr, want_m):
    """Adam's first moment is linear in the gradients: the gradient check.
    Tolerance 1e-3 of each leaf's scale (fp32 sums over the minibatch)."""
    from envmodel.trainer import unflatten
    got = unflatten(tr._names, tr._shapes, tr.flat(1))
    for m in want_m:
        for k in want_m[m]:
            w = want_m[m][k]
            np.testing.assert_allclose(got[m][k], w, rtol=1e-3, atol=1e-3 * float(np.abs(w).max()) + 1e-12,
                                       err_msg=f"m {m}/{k}")


def _assert_params_close(got, want, steps, lr=1e-3):
    """Parameters: Adam normalises each update, so an element whose gradient is
    ~0 can move by up to lr either way on fp32 vs f64 rounding.  All but 1e-3
    of the elements within (1e-4 rel, 3e-6 * steps abs); every one within 2 lr
    per step."""
    for m in want:
        for k in want[m]:
            g, w = np.asarray(got[m][k], np.float64), want[m][k]
            bad = ~np.isclose(g, w, rtol=1e-4, atol=3e-6 * steps)
            assert bad.mean() <= 1e-3, (m, k, int(bad.sum()))
            assert np.abs(g - w).max() <= 2 * lr * steps, (m, k)


@pytest.mark.parametrize("tw,shape", [(0.0, (28, 5, (128, 256, 128))), (1.0, (28, 5, (128, 256, 128))),
                                      (0.0, (42, 8, (64, 96)))])
def test_state_predictor_steps_match_oracle(tw, shape):
    D, A, hid = shape
    spec = em.EnvModelSpec(D, A, hid, (128, 256, 128) if tw > 0 else (64,))
    rng = np.random.default_rng(0)
    sp = em.init_state_predictor(spec, 1)
    sp["LayerNorm_0"]["scale"] = (1 + 0.1 * rng.standard_normal(D + A)).astype(np.float32)
    sp["LayerNorm_0"]["bias"] = (0.1 * rng.standard_normal(D + A)).astype(np.float32)
    tp = em.init_termination_predictor(spec, 2)
    cfg = EnvModelTrainerConfig(steps=50, termination_weight=tw, batch_size=64, init_learning_rate=1e-3)
    tr = StatePredictorTrainer(spec, sp, None, None, cfg, tp_params=tp if tw > 0 else None)
    ref, m, v = _f64(sp), T.zeros_like_tree(sp), T.zeros_like_tree(sp)
    for step in range(3):
        b = _batch(rng, 64, D, A)
        _, logs = tr.train_step(None, b)
        loss, want_logs, grads, _ = T.state_predictor_step(ref, b, tw, 30.0, _f64(tp))
        for k in logs:
            assert logs[k] == pytest.approx(want_logs[k], rel=1e-4, abs=1e-7), (step, k)
        ref, m, v = T.adam_update(ref, grads, m, v, step, T.cosine_lr(1e-3, 50, step))
        _assert_moments_close(tr, m)
        _assert_params_close(tr.params, ref, step + 1)
    assert tr.count == 3
    # eval_step: logs of the current parameters, no update
    b = _batch(rng, 64, D, A)
    logs = tr.eval_step(None, b)
    _, want_logs, _, _ = T.state_predictor_step(ref, b, tw, 30.0, _f64(tp))
    assert logs["next_observation_loss"] == pytest.approx(want_logs["next_observation_loss"], rel=1e-4)
    assert tr.count == 3
    tr.close()


def test_termination_predictor_steps_match_oracle():
    D = 28
    spec = em.EnvModelSpec(D, 5, (8,), (128, 256, 128))
    rng = np.random.default_rng(1)
    tp = em.init_termination_predictor(spec, 3)
    cfg = EnvModelTrainerConfig(steps=40, batch_size=128, init_learning_rate=1e-3)
    tr = TerminationPredictorTrainer(spec, tp, None, None, cfg)
    ref, m, v = _f64(tp), T.zeros_like_tree(tp), T.zeros_like_tree(tp)
    keep = rng.uniform(size=(128, D)) >= 0.1
    for step in range(3):
        b = _batch(rng, 128, D, 5, p_term=0.3)
        _, logs = tr.train_step(None, b, keep_mask=keep)
        loss, want_logs, grads = T.termination_predictor_step(ref, b, keep.astype(np.float64))
        for k in logs:
            assert logs[k] == pytest.approx(want_logs[k], rel=1e-4, abs=1e-7), (step, k)
        ref, m, v = T.adam_update(ref, grads, m, v, step, T.cosine_lr(1e-3, 40, step))
        _assert_moments_close(tr, m)
        _assert_params_close(tr.params, ref, step + 1)
    b = _batch(rng, 128, D, 5, p_term=0.3)
    logs = tr.eval_step(None, b)
    want = T.termination_eval_logs(ref, b)
    for k in ("loss", "true_loss", "false_loss"):
        assert logs[k] == pytest.approx(want[k], rel=1e-4, abs=1e-7), k
    for k in ("accuracy", "precision", "recall"):
        assert logs[k] == pytest.approx(want[k], abs=1.5 / 128), k
    tr.close()


def _seq_batch(rng, B, T, D, A, p_term=0.25):
    obs = rng.standard_normal((B, T, D)).astype(np.float32)
    return {"observations": obs, "actions": rng.uniform(-1, 1, (B, T, A)).astype(np.float32),
            "next_observations": (obs + 0.1 * rng.standard_normal((B, T, D))).astype(np.float32),
            "rewards": np.where(rng.uniform(size=(B, T)) < p_term, 0.0, -1.0).astype(np.float32)}


def _relu_margin(ref, b, tw, tp):
    """Smallest |pre-activation| of any hidden ReLU (both nets, every step) in the oracle's
    float64 forward of multistep_step."""
    lo = [np.inf]
    orig = T_._relu_mlp_fwd

    def fwd(tree, x):
        ins = []
        n = T_._n_dense(tree)
        for i in range(n):
            ins.append(x)
            x = x @ T_._W(tree, i) + T_._b(tree, i)
            if i < n - 1:
                lo[0] = min(lo[0], float(np.abs(x).min()))
                x = np.maximum(x, 0.0)
        return x, ins

    T_._relu_mlp_fwd = fwd
    try:
        T_.multistep_step(ref, b, tw, 30.0, tp)
    finally:
        T_._relu_mlp_fwd = orig
    return lo[0]


# A hidden unit whose float64 pre-activation is within fp32 rounding of zero (|u| ~ 1e-7: about
# one per T = 48 window of this config) can take the other side of the ReLU in an fp32 kernel,
# and a flipped mask moves every upstream BPTT gradient by ~1e-4..1e-3 of its scale: the
# elementwise comparison is then ill-posed, whatever the kernel's summation order.  Batches are
# drawn until every pre-activation is at least RELU_MARGIN from zero.
RELU_MARGIN = 2e-6


def _seq_batch_with_margin(rng, ref, tw, tp, B, T, D, A):
    for _ in range(64):
        b = _seq_batch(rng, B, T, D, A)
        if _relu_margin(ref, b, tw, tp) >= RELU_MARGIN:
            return b
    raise AssertionError("no batch with a ReLU margin in 64 draws")


@pytest.mark.parametrize("tw,T", [(0.0, 8), (1.0, 8), (0.0, 48)])
def test_multistep_steps_match_oracle(tw, T):
    """FQLPOP_EM_MULTISTEP (BPTT through the scanned cell) against oracle.multistep_step:
    logs, Adam moments and parameters after every injected step (batches with a ReLU margin:
    see RELU_MARGIN)."""
    D, A = 28, 5
    spec = em.EnvModelSpec(D, A, (128, 256, 128), (128, 256, 128) if tw > 0 else (64,))
    rng = np.random.default_rng(7)
    sp = em.init_state_predictor(spec, 1)
    sp["LayerNorm_0"]["scale"] = (1 + 0.1 * rng.standard_normal(D + A)).astype(np.float32)
    sp["LayerNorm_0"]["bias"] = (0.1 * rng.standard_normal(D + A)).astype(np.float32)
    tp = em.init_termination_predictor(spec, 2)
    cfg = EnvModelTrainerConfig(steps=50, model="multistep", sequence_length=T, termination_weight=tw,
                                batch_size=32, init_learning_rate=1e-3)
    tr = StatePredictorTrainer(spec, sp, None, None, cfg, tp_params=tp if tw > 0 else None)
    ref, m, v = _f64(sp), T_.zeros_like_tree(sp), T_.zeros_like_tree(sp)
    for step in range(3):
        b = _seq_batch_with_margin(rng, ref, tw, _f64(tp), 32, T, D, A)
        _, logs = tr.train_step(None, b)
        _, want_logs, grads, _ = T_.multistep_step(ref, b, tw, 30.0, _f64(tp))
        for k in logs:
            assert logs[k] == pytest.approx(want_logs[k], rel=2e-4, abs=1e-7), (step, k)
        ref, m, v = T_.adam_update(ref, grads, m, v, step, T_.cosine_lr(1e-3, 50, step))
        _assert_moments_close(tr, m)
        _assert_params_close(tr.params, ref, step + 1)
    logs = tr.eval_step(None, _seq_batch(rng, 32, T, D, A))
    assert np.isfinite(logs["loss"])
    with pytest.raises(ValueError):
        tr.train_step(None, _batch(rng, 32, D, A))  # single-step batches are refused
    tr.close()


class _Loader:
    def __init__(self, ds):
        self.dataset = ds

    def sample(self, n):
        idx = np.random.randint(len(self.dataset["observations"]), size=n)
        return {k: v[idx] for k, v in self.dataset.items()}


def _dynamics_dataset(n, D, A, seed=0):
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((n, D)).astype(np.float32)
    act = rng.uniform(-1, 1, (n, A)).astype(np.float32)
    M = (0.3 * rng.standard_normal((D + A, D))).astype(np.float32)
    nxt = obs + np.tanh(np.concatenate([obs, act], 1) @ M)
    return {"observations": obs, "actions": act, "next_observations": nxt.astype(np.float32),
            "rewards": np.where(nxt[:, 0] > 1.5, 0.0, -1.0).astype(np.float32)}


def test_device_sampled_training_learns_and_is_deterministic():
    D, A = 28, 5
    spec = em.EnvModelSpec(D, A)
    ds = _dynamics_dataset(20000, D, A)
    sp = em.init_state_predictor(spec, 0)
    cfg = EnvModelTrainerConfig(steps=400, termination_weight=0.0, batch_size=256, seed=5)
    runs = []
    for _ in range(2):
        tr = StatePredictorTrainer(spec, sp, _Loader(dict(ds)), None, cfg)
        b = {k: v[:256] for k, v in ds.items()}
        before = tr.eval_step(None, b)["next_observation_loss"]
        tr.steps(400)
        after = tr.eval_step(None, b)["next_observation_loss"]
        runs.append((before, after, tr.flat()))
        assert tr.count == 400
        tr.close()
    assert runs[1][1] < 0.5 * runs[0][0], runs[0][:2]
    np.testing.assert_array_equal(runs[0][2], runs[1][2])  # same seed -> bit-identical
    # termination predictor on the same data: loss falls, accuracy above the base rate
    tp = em.init_termination_predictor(spec, 1)
    tr = TerminationPredictorTrainer(spec, tp, _Loader(dict(ds)), None,
                                     EnvModelTrainerConfig(steps=300, batch_size=256, seed=2))
    b = {k: v[-256:] for k, v in ds.items()}
    before = tr.eval_step(None, b)["loss"]
    tr.steps(300)
    ev = tr.eval_step(None, b)
    assert ev["loss"] < before
    base = max(np.mean(b["rewards"] == 0), 1 - np.mean(b["rewards"] == 0))
    assert ev["accuracy"] >= base - 1e-6
    tr.close()


def test_train_loop_logs_like_reference():
    D, A = 28, 5
    spec = em.EnvModelSpec(D, A)
    ds = _dynamics_dataset(4000, D, A, seed=3)

    class Log:
        def __init__(self):
            self.rows = []

        def log(self, d, step):
            self.rows.append((step, d))

    lg = Log()
    tr = StatePredictorTrainer(spec, em.init_state_predictor(spec, 0), _Loader(dict(ds)), _Loader(dict(ds)),
                               EnvModelTrainerConfig(steps=120, termination_weight=0.0, val_batches=2), logger=lg)
    tr.train()
    keys = {k for _, d in lg.rows for k in d}
    assert {"train/loss", "train/next_observation_loss", "val/loss", "val/next_observation_loss"} <= keys
    assert sorted({s for s, d in lg.rows if "val/loss" in d}) == [0, 100, 119]  # final pass at steps - 1, as the reference
    tr.close()


def test_train_env_model_driver(tmp_path):
    """train_env_model.py end to end on a synthetic .npz: termination predictor, then the
    baseline with termination_weight > 0 loading it, saved flax-msgpack params readable back."""
    import train_env_model as tem
    D, A = 28, 5
    ds = _dynamics_dataset(3000, D, A, seed=9)
    data = tmp_path / "data"
    data.mkdir()
    np.savez(data / "cube-single-play.npz", observations=ds["observations"], actions=ds["actions"],
             next_observations=ds["next_observations"], rewards=ds["rewards"],
             masks=(ds["rewards"] != 0).astype(np.float32))  # OGBench singletask: masks = 1 - success
    common = [f"--data_directory={data}", f"--save_directory={tmp_path / 'exp'}", "--val_batches=2"]
    out = tem.main(["--model=termination_predictor", "--steps=150"] + common)
    tp = em.load_flax_msgpack(out / "termination_predictor.pt")["params"]
    assert tp["Dense_0"]["kernel"].shape == (D, 128)
    out = tem.main(["--model=baseline", "--steps=150", "--termination_weight=1"] + common)
    sp = em.load_flax_msgpack(out / "baseline.pt")["params"]
    assert sp["LayerNorm_0"]["scale"].shape == (D + A,)
    assert (out / "baseline_config.yaml").exists() and (out / "baseline_log.csv").exists()


def _trajectory_dataset(n_ep, D, A, seed=0):
    """Episode-major rows of 1000-step trajectories: o' = 0.9 o + 0.3 tanh([o, a] M)."""
    rng = np.random.default_rng(seed)
    M = (0.3 * rng.standard_normal((D + A, D))).astype(np.float32)
    o = rng.standard_normal((n_ep, D)).astype(np.float32)
    cols = {k: [] for k in ("observations", "actions", "next_observations")}
    for _ in range(1000):
        a = rng.uniform(-1, 1, (n_ep, A)).astype(np.float32)
        o2 = (0.9 * o + 0.3 * np.tanh(np.concatenate([o, a], 1) @ M)).astype(np.float32)
        cols["observations"].append(o)
        cols["actions"].append(a)
        cols["next_observations"].append(o2)
        o = o2
    ds = {k: np.stack(v, 1).reshape(n_ep * 1000, -1) for k, v in cols.items()}
    ds["rewards"] = np.where(ds["next_observations"][:, 0] > 1.0, 0.0, -1.0).astype(np.float32)
    return ds


def test_multistep_device_sampling_learns_and_driver(tmp_path):
    """Device-sampled MultistepLoader windows: deterministic for a seed, the rollout loss
    falls; then train_env_model.py --model=multistep end to end (flax nn.scan tree)."""
    import train_env_model as tem
    D, A = 28, 5
    ds = _trajectory_dataset(8, D, A, seed=11)
    spec = em.EnvModelSpec(D, A)
    sp = em.init_state_predictor(spec, 0)
    cfg = EnvModelTrainerConfig(steps=150, model="multistep", sequence_length=16, termination_weight=0.0,
                                batch_size=64, seed=3)
    runs = []
    for _ in range(2):
        ld = tem.MultistepLoader(dict(ds), 16)
        np.random.seed(0)
        b = ld.sample(64)
        tr = StatePredictorTrainer(spec, sp, ld, None, cfg)
        before = tr.eval_step(None, b)["next_observation_loss"]
        tr.steps(150)
        after = tr.eval_step(None, b)["next_observation_loss"]
        runs.append((before, after, tr.flat()))
        tr.close()
    assert runs[0][1] < 0.5 * runs[0][0], runs[0][:2]
    np.testing.assert_array_equal(runs[0][2], runs[1][2])
    data = tmp_path / "data"
    data.mkdir()
    np.savez(data / "cube-single-play.npz", masks=(ds["rewards"][:3000] != 0).astype(np.float32),
             **{k: ds[k][:3000] for k in ds})
    out = tem.main(["--model=multistep", "--steps=40", "--sequence_length=16", "--termination_weight=0",
                    f"--data_directory={data}", f"--save_directory={tmp_path / 'exp'}", "--val_batches=2"])
    tree = em.load_flax_msgpack(out / "multistep.pt")["params"]
    cell = tree["ScanCell_0"]["cell"]
    assert cell["Dense_0"]["kernel"].shape == (D + A, 128) and cell["LayerNorm_0"]["scale"].shape == (D + A,)


@pytest.mark.parametrize("tw,T", [(0.0, 48), (1.0, 16)])
def test_multistep_sweep_matches_round5_kernel(tw, T):
    """Round 6's multistep path (engine option em_seq_sweep: the 1024-thread BPTT sweep with
    the next op's weight fragments in flight, dW as a GEMM over the stored records) against
    round 5's em_seq_grad_kernel on the same device-sampled windows, one train step: logs
    within 1e-4, Adam moments within 1e-3 of each leaf's scale and parameters as against the
    oracle (only the order of the fp32 sums differs).  One step: an untrained cell rolled over
    T steps diverges, so later steps amplify rounding differences (4 steps at T = 48 differed by
    6.5e-4 in the loss).  Both paths are oracle-checked on injected batches above."""
    from _helpers import engine_options
    from envmodel.trainer import unflatten
    D, A = 28, 5
    ds = _trajectory_dataset(8, D, A, seed=5)
    spec = em.EnvModelSpec(D, A, (128, 256, 128), (128, 256, 128))
    sp = em.init_state_predictor(spec, 0)
    tp = em.init_termination_predictor(spec, 2)
    cfg = EnvModelTrainerConfig(steps=50, model="multistep", sequence_length=T, termination_weight=tw,
                                batch_size=64, seed=9, init_learning_rate=1e-3)
    out = {}
    for path in (0, 1):
        with engine_options(em_seq_sweep=path):
            tr = StatePredictorTrainer(spec, sp, _Loader(ds), None, cfg, tp_params=tp if tw > 0 else None)
            tr.steps(1)
            out[path] = (tr.read_logs(), unflatten(tr._names, tr._shapes, tr.flat(0)),
                         unflatten(tr._names, tr._shapes, tr.flat(1)))
            tr.close()
    for k, v in out[0][0].items():
        assert out[1][0][k] == pytest.approx(v, rel=1e-4, abs=1e-7), k
    for m in out[0][2]:
        for k in out[0][2][m]:
            w = out[0][2][m][k]
            np.testing.assert_allclose(out[1][2][m][k], w, rtol=1e-3, atol=1e-3 * float(np.abs(w).max()) + 1e-12,
                                       err_msg=f"m {m}/{k}")
    _assert_params_close(out[1][1], _f64(out[0][1]), 1)
