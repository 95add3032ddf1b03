"""The agent state-dict layouts (fql/utils/serialization.py): the engine's flat member
state <-> the upstream flax.serialization.to_state_dict(FQLAgent) tree [EXT, unpinned]."""
import numpy as np
import pytest

from oracle import fql_oracle as O


def _flat_state(seed=0):
    cfg = O.OracleConfig(hidden_dims=(8,) * 4, batch_size=4)
    p = O.cast_tree(O.init_params(cfg, seed), np.float32)
    rng = np.random.default_rng(seed)
    mu = {n: {k: rng.standard_normal(v.shape).astype(np.float32) for k, v in t.items()} for n, t in p.items()}
    nu = {n: {k: rng.uniform(size=v.shape).astype(np.float32) for k, v in t.items()} for n, t in p.items()}
    return {"params": p, "opt_state": {"count": 7, "mu": mu, "nu": nu}}


def test_flat_flax_round_trip():
    from fql.utils.serialization import flat_to_flax, flax_to_flat, is_flax_layout, params_of
    flat = _flat_state()
    fx = flat_to_flax(flat, rng=[1, 2])
    assert is_flax_layout(fx) and not is_flax_layout(flat)
    net = fx["network"]
    assert net["step"] == 7 and int(net["opt_state"]["0"]["count"]) == 7 and net["opt_state"]["1"] == {}
    assert fx["rng"].dtype == np.uint32 and list(fx["rng"]) == [1, 2]
    crit = net["params"]["modules_critic"]["value_net"]
    assert crit["Dense_0"]["kernel"].shape == (2, 33, 8)            # ensemble axis first
    assert set(crit["LayerNorm_3"]) == {"scale", "bias"}
    assert set(net["params"]["modules_actor_bc_flow"]) == {"mlp"}
    assert net["params"]["modules_actor_bc_flow"]["mlp"]["Dense_4"]["kernel"].shape == (8, 5)
    back = flax_to_flat(fx)
    assert back["opt_state"]["count"] == 7
    for part in ("params",):
        for n, t in flat[part].items():
            for k, v in t.items():
                np.testing.assert_array_equal(back[part][n][k], v)
    for m in ("mu", "nu"):
        for n, t in flat["opt_state"][m].items():
            for k, v in t.items():
                np.testing.assert_array_equal(back["opt_state"][m][n][k], v)
    assert params_of(fx)["critic"]["Dense_1/kernel"] is not None
    np.testing.assert_array_equal(params_of(fx)["critic"]["Dense_1/kernel"], flat["params"]["critic"]["Dense_1/kernel"])


def test_flax_layout_rejects_inconsistent_state():
    from fql.utils.serialization import flat_to_flax, flax_to_flat
    fx = flat_to_flax(_flat_state())
    fx["network"]["step"] = 3
    with pytest.raises(ValueError):
        flax_to_flat(fx)
    fx = flat_to_flax(_flat_state())
    fx["network"]["params"]["modules_bogus"] = {}
    with pytest.raises(KeyError):
        flax_to_flat(fx)
