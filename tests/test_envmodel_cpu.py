"""CPU tests of the world-model evaluator's host side: flax-ordered flat
parameters vs the C ABI's layout, the flax msgpack format, and known answers
of the rollout oracle (oracle/envmodel_oracle.py)."""
import ctypes

import numpy as np

import envmodel as em
from envmodel.flax_msgpack import load_flax_msgpack, msgpack_restore, msgpack_serialize
from oracle import envmodel_oracle as EO
from oracle import fql_oracle as O


def test_flat_sizes_match_c_abi():
    from fqlpop import _lib
    lib = _lib.load_library()
    for obs, act, sp, tp in [(28, 5, (128, 256, 128), (128, 256, 128)), (42, 8, (64,), (32, 32)), (7, 3, (), ())]:
        spec = em.EnvModelSpec(obs, act, sp, tp)
        c = _lib.EnvModelConfig()
        c.obs_dim, c.action_dim, c.sp_num_hidden, c.tp_num_hidden = obs, act, len(sp), len(tp)
        for i, d in enumerate(sp):
            c.sp_hidden[i] = d
        for i, d in enumerate(tp):
            c.tp_hidden[i] = d
        n_sp, n_tp = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(lib.fqlpop_envmodel_param_count(ctypes.byref(c), ctypes.byref(n_sp), ctypes.byref(n_tp)))
        sp_flat = em.flatten_state_predictor(spec, em.init_state_predictor(spec, 0))
        tp_flat = em.flatten_termination_predictor(spec, em.init_termination_predictor(spec, 1))
        assert sp_flat.shape[0] == n_sp.value and tp_flat.shape[0] == n_tp.value


def test_flat_order_is_flax_path_order():
    spec = em.EnvModelSpec(3, 2, (4,), (5,))
    tree = em.init_state_predictor(spec, 0)
    tree["LayerNorm_0"]["bias"] = np.arange(5, dtype=np.float32) + 100
    flat = em.flatten_state_predictor(spec, tree)
    # Dense_0/bias(4) Dense_0/kernel(5x4) Dense_1/bias(3) Dense_1/kernel(4x3) LayerNorm_0/bias(5) LayerNorm_0/scale(5)
    assert flat.shape[0] == 4 + 20 + 3 + 12 + 5 + 5
    np.testing.assert_array_equal(flat[4:24], tree["Dense_0"]["kernel"].reshape(-1))
    np.testing.assert_array_equal(flat[39:44], tree["LayerNorm_0"]["bias"])
    # a multistep checkpoint nests the cell (utils/envmodel.py:46-49)
    nested = {"params": {"ScanCell_0": {"cell": tree}}}
    np.testing.assert_array_equal(em.flatten_state_predictor(spec, nested), flat)
    assert em.spec_from_trees(nested, em.init_termination_predictor(spec)) == spec


def test_flax_msgpack_roundtrip(tmp_path):
    spec = em.EnvModelSpec(6, 2, (8, 4), (3,))
    tree = {"params": em.init_state_predictor(spec, 3)}
    blob = msgpack_serialize(tree)
    back = msgpack_restore(blob)
    for mod, leaves in tree["params"].items():
        for k, v in leaves.items():
            np.testing.assert_array_equal(back["params"][mod][k], v)
            assert back["params"][mod][k].dtype == np.float32
    p = tmp_path / "baseline.pt"
    p.write_bytes(blob)
    assert set(load_flax_msgpack(p)["params"]) == set(tree["params"])


def test_flax_msgpack_chunked_array():
    import msgpack
    a = np.arange(12, dtype=np.float32).reshape(3, 4)
    chunks = {"0": a.reshape(-1)[:5], "1": a.reshape(-1)[5:]}
    tree = {"x": {"__msgpack_chunked_array__": True, "shape": [3, 4], "chunks": chunks}}
    blob = msgpack.packb(tree, default=lambda x: msgpack.ExtType(
        1, msgpack.packb((x.shape, x.dtype.name, x.tobytes()), use_bin_type=True)))
    np.testing.assert_array_equal(msgpack_restore(blob)["x"], a)


def _models(spec, tp_bias):
    sp = em.init_state_predictor(spec, 0)
    tp = em.init_termination_predictor(spec, 1, scale=0.0, bias=tp_bias)
    return sp, tp


def test_oracle_rollout_known_answers():
    cfg = O.OracleConfig(hidden_dims=(16,) * 4)
    params = O.cast_tree(O.init_params(cfg, 0), np.float64)
    spec = em.EnvModelSpec(cfg.obs_dim, cfg.action_dim, (8,), (8,))
    rng = np.random.default_rng(0)
    obs0 = rng.standard_normal((5, cfg.obs_dim))
    noise = rng.standard_normal((7, 5, cfg.action_dim))
    # logit = +1 everywhere: every env terminates (success) at step 1
    sp, tp = _models(spec, 1.0)
    s, l, obs, t = EO.rollout(cfg, params, sp, tp, obs0, noise, 7)
    assert s.tolist() == [1.0] * 5 and l.tolist() == [1.0] * 5 and t == 1
    # logit = -1: nothing terminates, all truncated at max_steps with success 0
    sp, tp = _models(spec, -1.0)
    s, l, obs, t = EO.rollout(cfg, params, sp, tp, obs0, noise, 7)
    assert s.tolist() == [0.0] * 5 and l.tolist() == [7.0] * 5 and t == 7
    # zero state predictor: s' = s (residual only), LayerNorm irrelevant
    zero = {k: {kk: np.zeros_like(vv) for kk, vv in v.items()} for k, v in sp.items()}
    assert np.allclose(EO.state_predictor(zero, obs0, noise[0]), obs0)
