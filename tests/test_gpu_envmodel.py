"""GPU parity of the world-model rollout evaluator (fqlpop_envmodel_step,
fqlpop_rollout) against the float64 restatement in oracle/envmodel_oracle.py,
and the Trainer driving SuccessiveHalving on its GPU scores."""
import numpy as np
import pytest

import envmodel as em
from oracle import envmodel_oracle as EO
from oracle import fql_oracle as O

pytestmark = pytest.mark.gpu
H = 512  # the rollout kernel streams the 512-wide actor


def _population(n, obs_dim=28, act_dim=5, seed=0):
    from fqlpop import Population, PopulationConfig
    pop = Population(PopulationConfig(obs_dim=obs_dim, action_dim=act_dim, hidden_dims=(H,) * 4, batch_size=64),
                     [10.0] * n, list(range(1, n + 1)))
    cfg = O.OracleConfig(obs_dim=obs_dim, action_dim=act_dim, hidden_dims=(H,) * 4, batch_size=64)
    params = []
    for i in range(n):
        p = O.cast_tree(O.init_params(cfg, seed + i), np.float32)
        pop.set_params(i, p)
        params.append(O.cast_tree(p, np.float64))
    return pop, cfg, params


def _env_model(spec, tp_bias=0.0, tp_scale=1.0, seed=0):
    sp = em.init_state_predictor(spec, seed)
    for k in sp:  # non-trivial LayerNorm parameters
        if k.startswith("LayerNorm"):
            rng = np.random.default_rng(seed + 7)
            sp[k]["scale"] = (1.0 + 0.2 * rng.standard_normal(sp[k]["scale"].shape)).astype(np.float32)
            sp[k]["bias"] = (0.1 * rng.standard_normal(sp[k]["bias"].shape)).astype(np.float32)
    tp = em.init_termination_predictor(spec, seed + 1, scale=tp_scale, bias=tp_bias)
    return sp, tp


def _upload(pop, spec, sp, tp):
    pop.set_env_model(em.flatten_state_predictor(spec, sp), em.flatten_termination_predictor(spec, tp),
                      spec.sp_hidden, spec.tp_hidden)


@pytest.mark.parametrize("obs_dim,act_dim,sp_h,tp_h", [(28, 5, (128, 256, 128), (128, 256, 128)),
                                                       (42, 8, (64, 96), (40,))])
def test_envmodel_step_matches_oracle(obs_dim, act_dim, sp_h, tp_h):
    pop, cfg, _ = _population(1, obs_dim, act_dim)
    spec = em.EnvModelSpec(obs_dim, act_dim, sp_h, tp_h)
    sp, tp = _env_model(spec)
    _upload(pop, spec, sp, tp)
    rng = np.random.default_rng(3)
    obs = rng.standard_normal((37, obs_dim)).astype(np.float32)
    act = rng.uniform(-1, 1, (37, act_dim)).astype(np.float32)
    nxt, logit = pop.envmodel_step(obs, act)
    want = EO.state_predictor(sp, obs.astype(np.float64), act.astype(np.float64))
    np.testing.assert_allclose(nxt, want, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(logit, EO.termination_predictor(tp, want), rtol=1e-4, atol=1e-5)
    pop.close()


def _run_both(pop, cfg, params, spec, sp, tp, n_envs, steps, seed=5):
    rng = np.random.default_rng(seed)
    obs0 = rng.standard_normal((n_envs, cfg.obs_dim)).astype(np.float32)
    noise = rng.standard_normal((len(params), steps, n_envs, cfg.action_dim)).astype(np.float32)
    succ, length, oobs = pop.rollout(obs0, steps, noise=noise, return_obs=True)
    want = [EO.rollout(cfg, params[i], sp, tp, obs0.astype(np.float64), noise[i].astype(np.float64), steps)
            for i in range(len(params))]
    return succ, length, oobs, want


def test_rollout_single_block_matches_oracle():
    # tp logits far from 0 for a few steps: nothing terminates, compare trajectories
    pop, cfg, params = _population(2)
    spec = em.EnvModelSpec(28, 5)
    sp, tp = _env_model(spec, tp_bias=-50.0, tp_scale=0.1)
    _upload(pop, spec, sp, tp)
    succ, length, oobs, want = _run_both(pop, cfg, params, spec, sp, tp, n_envs=12, steps=4)
    for i, (s, l, obs, t) in enumerate(want):
        np.testing.assert_array_equal(succ[i], s)
        np.testing.assert_array_equal(length[i], l)
        np.testing.assert_allclose(oobs[i], obs, rtol=2e-3, atol=2e-4)
    pop.close()


def test_rollout_terminations_match_oracle():
    pop, cfg, params = _population(3)
    spec = em.EnvModelSpec(28, 5, (64, 128), (64,))
    sp, tp = _env_model(spec, tp_bias=-14.0, tp_scale=1.0, seed=11)
    _upload(pop, spec, sp, tp)
    succ, length, _, want = _run_both(pop, cfg, params, spec, sp, tp, n_envs=40, steps=12)
    agree = total = 0
    for i, (s, l, _, _) in enumerate(want):
        agree += int((succ[i] == s).sum() + (length[i] == l).sum())
        total += 2 * s.shape[0]
    # chaotic rollouts: an env whose logit sits within float error of 0 may flip;
    # with these models (|logit| >> 1e-4 almost everywhere) all must agree
    assert agree == total, (succ, length, [w[:2] for w in want])
    assert 0 < succ.mean() < 1  # the case exercises both outcomes
    pop.close()


def test_rollout_device_noise_deterministic():
    pop, cfg, params = _population(2)
    spec = em.EnvModelSpec(28, 5)
    sp, tp = _env_model(spec, tp_bias=-0.2, seed=4)
    _upload(pop, spec, sp, tp)
    obs0 = np.random.default_rng(0).standard_normal((50, 28)).astype(np.float32)
    a = pop.rollout(obs0, 30, seed=7, return_obs=True)
    b = pop.rollout(obs0, 30, seed=7, return_obs=True)
    c = pop.rollout(obs0, 30, seed=8, return_obs=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert not np.array_equal(a[2], c[2])
    pop.close()


def test_rollout_requires_env_model_and_512():
    from fqlpop import FqlpopError, Population, PopulationConfig
    pop, _, _ = _population(1)
    with pytest.raises(FqlpopError, match="no env model"):
        pop.rollout(np.zeros((4, 28), np.float32), 3)
    pop.close()
    small = Population(PopulationConfig(hidden_dims=(64,) * 4, batch_size=64), [1.0], [0])
    spec = em.EnvModelSpec(28, 5)
    sp, tp = _env_model(spec)
    _upload(small, spec, sp, tp)
    with pytest.raises(FqlpopError, match="512"):
        small.rollout(np.zeros((4, 28), np.float32), 3)
    small.close()


def test_simulated_task_trainer_halving(tmp_path):
    from hpo.successive_halving import SuccessiveHalving
    from task.offline_task_simulated import OfflineTaskWithSimulatedEvaluations
    from trainer.config import AgentConfig, ExperimentConfig, TrainerConfig
    from trainer.trainer import Trainer
    from evaluator.evaluation import evaluate_agent
    task = OfflineTaskWithSimulatedEvaluations(n_rows=20_000, n_val_rows=2_000, num_evaluation_envs=20,
                                               max_episode_steps=25)
    agent = AgentConfig(actor_hidden_dims=(H,) * 4, value_hidden_dims=(H,) * 4, batch_size=64)
    cfg = TrainerConfig(agent=agent, steps=40, eval_interval=10, log_interval=10, save_directory=tmp_path)
    configs = [ExperimentConfig(alpha=a, seed=s) for a, s in [(3.0, 1), (10.0, 2), (30.0, 3), (100.0, 4)]]
    strategy = SuccessiveHalving(set(configs), total_evaluations=8, fraction=0.5, history_length=1)
    tr = Trainer(task, strategy, cfg)
    tr.train(max_evaluations=100)
    assert len(tr.candidates) < len(configs)  # halving on the GPU rollout scores
    scores = [v for vs in strategy.candidate_scores.values() for v in vs]
    assert scores and all(0.0 <= v <= 1.0 for v in scores)
    for c in tr.candidates:
        assert tr.experiments[c].current_step == cfg.steps
    # the reference per-step loop over the same task (fqlpop_envmodel_step per step)
    exp = next(iter(tr.experiments.values()))
    task.attach(tr.population)
    info, transitions = evaluate_agent(exp.agent, task, seed=0)
    assert 0.0 <= info["success"] <= 1.0 and len(transitions) <= 25


def test_rollout_antsoccer_32_members_matches_oracle():
    """BASELINE config C5's evaluation at its shapes: 32 members of the antsoccer actor
    (obs 42, act 8, 512 x 4) x 50 envs (eval_episodes) in one launch, with the
    multistep default state predictor (128, 256, 128) and a termination predictor that
    ends some episodes.  Success flags and episode lengths must equal the oracle's for
    every env of every member; observations of the envs still running after the last
    step within 2e-3."""
    n = 32
    pop, cfg, params = _population(n, 42, 8, seed=40)
    spec = em.EnvModelSpec(42, 8, (128, 256, 128), (128, 128))
    sp, tp = _env_model(spec, tp_bias=4.0, tp_scale=3.0, seed=21)  # ~12 % terminate; |logit| > 0.7 throughout
    _upload(pop, spec, sp, tp)
    succ, length, oobs, want = _run_both(pop, cfg, params, spec, sp, tp, n_envs=50, steps=8, seed=9)
    assert succ.shape == (n, 50)
    for i, (s, l, obs, _) in enumerate(want):
        np.testing.assert_array_equal(succ[i], s, err_msg=f"member {i}")
        np.testing.assert_array_equal(length[i], l, err_msg=f"member {i}")
        np.testing.assert_allclose(oobs[i], obs, rtol=2e-3, atol=2e-4, err_msg=f"member {i}")
    assert 0 < succ.mean() < 1, succ.mean()  # both outcomes occur
    pop.close()
