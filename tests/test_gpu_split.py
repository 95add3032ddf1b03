"""Split launches (engine option ``split``; kernels.hip, "split streamed forward"): small
populations run the streamed forwards and the Euler flow as clusters of 2, 4 or 8 blocks
per 16-column tile that hand every hidden layer's output to each other through L2 / MALL.

Each output element keeps the unsplit fp32 chain (full K in the unsplit k order, the
LayerNorm and head partials summed in the unsplit order), so a split run must be
BIT-IDENTICAL to the unsplit one: parameters, Adam moments, target critic, info and val
info after several device-sampled steps, for every split factor and member count.  That
is also what keeps a member's results independent of how many members share its GPU (the
world size of a sharded population).  Oracle parity of the split path itself: the 2-member
production-step test of test_gpu_parity.py runs on it (auto split)."""
import numpy as np
import pytest

from _helpers import engine_options

pytestmark = pytest.mark.gpu


def _data(N, D, A, seed):
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((N, D)).astype(np.float32)
    rew = np.where(rng.uniform(size=N) < 0.05, 0.0, -1.0).astype(np.float32)
    return {"observations": obs, "actions": rng.uniform(-1 + 1e-5, 1 - 1e-5, (N, A)).astype(np.float32),
            "rewards": rew, "masks": (1.0 - (rew == 0)).astype(np.float32),
            "next_observations": (obs + 0.05 * rng.standard_normal((N, D))).astype(np.float32)}


def _run(opts, n_members, D=28, A=5, B=256, steps=3, probe=False, **kw):
    from fqlpop import Population, PopulationConfig
    alphas = [3.0 * 3.3 ** i for i in range(n_members)]
    with engine_options(**opts):
        pop = Population(PopulationConfig(obs_dim=D, action_dim=A, hidden_dims=(512,) * 4, batch_size=B, **kw),
                         alphas, [11 + i for i in range(n_members)])
        pop.set_dataset(_data(20_000, D, A, 3))
        if probe:
            pop.set_probe(True)
        pop.step(steps)
        info = pop.read_info_array().copy()
        cover = None
        if probe:
            cover = (pop.read_probe()[1],) + pop.probe_coverage()
            pop.set_probe(False)
        rng = np.random.default_rng(9)
        val = {"observations": rng.standard_normal((B, D)).astype(np.float32),
               "actions": rng.uniform(-1, 1, (B, A)).astype(np.float32),
               "rewards": -np.ones(B, np.float32), "masks": np.ones(B, np.float32),
               "next_observations": rng.standard_normal((B, D)).astype(np.float32)}
        pop.total_loss([val] * n_members)
        vinfo = pop.read_info_array("val").copy()
        flats = [pop.get_flat(i, w) for i in range(n_members) for w in (0, 1, 2)]
        name = pop.dominant_kernel_info()[0]
        pop.close()
    if probe:
        return info, vinfo, flats, name, cover
    return info, vinfo, flats, name


def _same(a, b):
    assert np.array_equal(a[0], b[0]), "train info differs"
    assert np.array_equal(a[1], b[1]), "val info differs"
    for i, (x, y) in enumerate(zip(a[2], b[2])):
        assert np.array_equal(x, y), f"state {i} differs (max |d| {np.abs(x - y).max()})"


@pytest.mark.parametrize("n,F", [(1, 8), (2, 8), (2, 4), (2, 2), (3, 4)])
def test_split_bit_identical_to_unsplit_cube(n, F):
    ref = _run({"split": 0}, n)
    got = _run({"split": F}, n)
    assert got[3].startswith("split_fwd_kernel"), got[3]
    assert ref[3] == "euler_flow_kernel"
    _same(got, ref)


@pytest.mark.parametrize("n,split", [(1, 8), (2, 8), (4, 1), (8, 1)])
def test_small_population_schedule_bit_identical(n, split):
    """The 4th-stream schedule (engine option small_sched, on at every population size since
    round 5: the target critic and the critic's TD-column backward on a fourth stream, the
    Q-loss columns' backward as a launch of its own) changes where launches run, not what
    they compute: bit-identical to three streams, split (1-2 members) and unsplit (8)."""
    ref = _run({"split": split, "small_sched": 0}, n)
    got = _run({"split": split, "small_sched": 1}, n)
    _same(got, ref)


def test_split_auto_bit_identical_antsoccer_shape():
    """BASELINE C3 shapes (obs 42, act 8, B = 1024), one member: auto splits the Euler
    flow (64 tiles x 4 blocks), the BC forward and the target critic (128 tiles x 2); the
    one-step and critic forwards (192, 256 tiles) stay unsplit."""
    ref = _run({"split": 0}, 1, D=42, A=8, B=1024, steps=2, discount=0.995)
    got = _run({}, 1, D=42, A=8, B=1024, steps=2, discount=0.995)
    _same(got, ref)


def test_split_no_error_word_and_probe_times_split_launch():
    """The in-step probe times the split Euler launch (every block's stamps), and no
    hand-off wait gave up (the runtime raises on the error word at sync)."""
    from fqlpop import Population, PopulationConfig
    pop = Population(PopulationConfig(hidden_dims=(512,) * 4, batch_size=256), [3.0, 30.0], [1, 2])
    pop.set_dataset(_data(20_000, 28, 5, 4))
    pop.set_probe(True)
    pop.step(6)
    pop.sync()
    us, n, _ = pop.read_probe()
    assert n == 6 and us > 0
    name = pop.dominant_kernel_info()[0]
    assert name.startswith("split_fwd_kernel"), name
    pop.close()


def test_split_euler_512_blocks_with_probe():
    """4 members at split_blocks=512 run the Euler flow as 64 tiles x 8
    blocks = 512 blocks (the launch whose stamps overran round 4's 256-block probe buffer).
    With the probe on: bit-identical to unsplit, no error word (read_info / sync raise on
    it), and every block of every timed launch wrote both of its stamps."""
    steps = 3
    ref = _run({"split": 0}, 4, steps=steps)
    got = _run({"split_blocks": 512}, 4, steps=steps, probe=True)
    assert got[3].startswith("split_fwd_kernel"), got[3]
    _same(got, ref)
    launches, seen, expected = got[4]
    assert launches == steps
    assert expected == steps * 512, expected
    assert seen == expected



def _prune_revive(opts):
    from fqlpop import Population, PopulationConfig
    with engine_options(**opts):
        pop = Population(PopulationConfig(hidden_dims=(512,) * 4, batch_size=256), [3.0, 30.0, 300.0], [4, 5, 6])
        pop.set_dataset(_data(20_000, 28, 5, 6))
        pop.step(3)
        pop.set_active([1, 0, 1])  # fewer clusters per split launch
        pop.step(2)
        pop.set_active([1, 1, 1])  # more again: exchange words of the dropped clusters were cleared
        pop.step(2)
        pop.sync()
        out = ([pop.get_flat(i, w) for i in range(3) for w in (0, 1, 2)], [pop.get_count(i) for i in range(3)],
               pop.read_info_array().copy())
        pop.close()
    return out


def test_prune_and_revive_split_bit_identical():
    """A member dropped and revived (SuccessiveHalving's pruning, the distributed trainer's
    member moves) changes the number of clusters of every split launch twice; the split run
    stays bit-identical to the unsplit one, no hand-off wait gives up, and get_state /
    get_count (which now refuse state a failed split launch wrote) return normally."""
    ref = _prune_revive({"split": 0})
    got = _prune_revive({})
    assert got[1] == ref[1] == [7, 5, 7]
    assert np.array_equal(got[2], ref[2])
    for i, (x, y) in enumerate(zip(got[0], ref[0])):
        assert np.array_equal(x, y), f"state {i} differs"


def test_split_euler_pre0_non_tail_shape_bit_identical():
    """the split Euler flow's layer-0 precompute (PRE0) for a shape WITHOUT the
    layer-0 tail k-step: obs 24, act 4 (K0 = 29: 8 k-steps, 6 of them observation rows, 2 of
    the step's own) against the unsplit kernel, 1 and 2 members."""
    for n in (1, 2):
        ref = _run({"split": 0}, n, D=24, A=4)
        got = _run({}, n, D=24, A=4)
        assert got[3].startswith("split_fwd_kernel"), got[3]
        _same(got, ref)


def test_split_failure_is_sticky_until_restored():
    """a split launch that gave up poisons the members it stepped.  The
    error is reported by the next call, and then step, get_state, get_count and read_info keep
    refusing a poisoned member (no checkpoint of state such a launch wrote) until its params,
    Adam m and Adam v are restored with set_state; the restored member exports again and the
    population trains again once every member is restored."""
    from fqlpop import FqlpopError, Population, PopulationConfig
    from fqlpop._lib import check
    pop = Population(PopulationConfig(hidden_dims=(512,) * 4, batch_size=256), [3.0, 30.0], [1, 2])
    pop.set_dataset(_data(20_000, 28, 5, 4))
    pop.step(2)
    pop.sync()
    saved = [[pop.get_flat(i, w) for w in (0, 1, 2)] for i in range(2)]
    count = [pop.get_count(i) for i in range(2)]
    check(pop.lib.fqlpop_debug_fail_split(pop._h))
    with pytest.raises(FqlpopError, match="hand-off wait timed out"):
        pop.step(1)
    for call in (lambda: pop.step(1), lambda: pop.get_flat(0, 0), lambda: pop.get_flat(1, 1),
                 lambda: pop.get_count(0), lambda: pop.read_info_array()):
        with pytest.raises(FqlpopError, match="restore"):
            call()
    pop.sync()  # reported once; the poison stays
    for w in (0, 1):  # params and m only: still poisoned
        pop.set_flat(0, saved[0][w], w)
    with pytest.raises(FqlpopError, match="member 0"):
        pop.get_flat(0, 0)
    pop.set_flat(0, saved[0][2], 2)
    assert np.array_equal(pop.get_flat(0, 0), saved[0][0])
    assert pop.get_count(0) == count[0]
    with pytest.raises(FqlpopError, match="member 1"):
        pop.step(1)
    pop.set_member(1, 30.0, 2, reinit=True)
    pop.step(2)
    pop.sync()
    assert np.all(np.isfinite(pop.read_info_array()[:, :13]))
    pop.close()
