"""GPU tests of the reference-shaped surface over the HIP engine: the golden
fixture through the C ABI, FQLAgent, Experiment/Trainer (Identity and
SuccessiveHalving), load_agent and the tune_alpha.py driver end to end."""
import os
import pickle

import numpy as np
import pytest

from oracle import fql_oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
SMALL = "(64, 64, 64, 64)"


def test_golden_fixture_through_c_abi():
    from fqlpop import Population, PopulationConfig
    g = np.load(os.path.join(GOLDEN, "oracle_update_h64.npz"))
    H, B, alpha = (int(g["config"][0]), int(g["config"][1]), float(g["config"][2]))
    pop = Population(PopulationConfig(hidden_dims=(H,) * 4, batch_size=B), [alpha], [0])
    tree = {net: {} for net in O.NETS}
    for k in g.files:
        if k.startswith("params_in/"):
            _, net, leaf = k.split("/", 2)
            tree[net][leaf] = g[k]
    pop.set_params(0, tree)
    for step in range(2):
        b = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith(f"batch{step}/")}
        n = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith(f"noise{step}/")}
        pop.step_injected([b], [n])
        info = pop.read_info()[0]
        want = g[f"info{step}"]
        for j, key in enumerate(O.TRAIN_INFO_KEYS):
            assert abs(info[key] - want[j]) <= 1e-4 * abs(want[j]) + 1e-6, (step, key, info[key], want[j])
    got = pop.get_params(0)
    worst = max(float(np.abs(got[net][leaf] - g[f"params_out/{net}/{leaf}"]).max())
                for net in O.NETS for leaf in got[net])
    assert worst <= 2 * 3e-4 + 1e-5


def test_fqlagent_surface():
    from fql.agents.fql import FQLAgent
    from trainer.config import AgentConfig
    from dataclasses import asdict
    cfg = asdict(AgentConfig(actor_hidden_dims=(64,) * 4, value_hidden_dims=(64,) * 4, batch_size=64))
    rng = np.random.default_rng(0)
    ocfg = O.OracleConfig(hidden_dims=(64,) * 4, batch_size=64)
    batch = O.cast_tree(O.make_batch(ocfg, 64, rng), np.float32)
    agent = FQLAgent.create(3, batch["observations"][:1], batch["actions"][:1], cfg)
    assert agent.config["ob_dims"] == (28,) and agent.config["action_dim"] == 5
    sd0 = agent.to_state_dict()
    assert set(sd0) == {"rng", "network"} and set(sd0["network"]) == {"step", "params", "opt_state"}
    assert set(sd0["network"]["params"]) == {"modules_actor_bc_flow", "modules_actor_onestep_flow",
                                             "modules_critic", "modules_target_critic"}
    before = sd0["network"]["params"]["modules_actor_onestep_flow"]["mlp"]["Dense_0"]["kernel"].copy()
    agent, info = agent.update(batch)
    assert set(info) == set(O.TRAIN_INFO_KEYS) and all(np.isfinite(v) for v in info.values())
    assert agent.step == 1
    sd1 = agent.to_state_dict()
    after = sd1["network"]["params"]["modules_actor_onestep_flow"]["mlp"]["Dense_0"]["kernel"]
    assert sd1["network"]["step"] == 1 and int(sd1["network"]["opt_state"]["0"]["count"]) == 1
    assert not np.array_equal(before, after)
    loss, vinfo = agent.total_loss(batch, grad_params=None)
    assert set(vinfo) == set(O.VAL_INFO_KEYS) and np.isfinite(loss)
    acts = agent.sample_actions(observations=batch["observations"][:7], seed=np.array([0, 42], np.uint32))
    assert acts.shape == (7, 5) and np.all(np.abs(acts) <= 1)
    # state dict round trip into a fresh agent reproduces the same actions
    other = FQLAgent.create(9, batch["observations"][:1], batch["actions"][:1], cfg)
    other.from_state_dict(agent.to_state_dict())
    z = rng.standard_normal((7, 5)).astype(np.float32)
    a1 = agent.population.sample_actions(0, batch["observations"][:7], noise=z)
    a2 = other.population.sample_actions(0, batch["observations"][:7], noise=z)
    assert np.array_equal(a1, a2) and other.step == 1


def _trainer_config(tmp_path, steps=40, eval_interval=10, log_interval=5):
    from trainer.config import AgentConfig, TrainerConfig
    return TrainerConfig(steps=steps, eval_interval=eval_interval, log_interval=log_interval,
                         save_directory=tmp_path, env_name="cube-single-play-singletask-task2-v0",
                         agent=AgentConfig(actor_hidden_dims=(64,) * 4, value_hidden_dims=(64,) * 4,
                                           batch_size=64))


def test_trainer_successive_halving_and_load_agent(tmp_path):
    from hpo.successive_halving import SuccessiveHalving
    from task.offline_task_synthetic import OfflineTaskSynthetic
    from trainer.config import ExperimentConfig
    from trainer.trainer import Trainer
    from utils.agent import load_agent
    task = OfflineTaskSynthetic(n_rows=20_000, n_val_rows=2_000, num_evaluation_envs=4, max_episode_steps=8)
    cfg = _trainer_config(tmp_path)
    configs = [ExperimentConfig(seed=s, alpha=a) for a, s in [(3.0, 1), (30.0, 2), (300.0, 3), (1000.0, 4)]]
    strategy = SuccessiveHalving(set(configs), total_evaluations=8, fraction=0.5, history_length=1)
    trainer = Trainer(task, strategy, cfg)
    trainer.train(max_evaluations=100)
    # halving at the milestones shrank the population; survivors reached the end
    assert len(trainer.candidates) < len(configs)
    for c in trainer.candidates:
        exp = trainer.experiments[c]
        assert exp.current_step == cfg.steps and c in trainer.finished_candidates
        d = tmp_path / cfg.env_name / exp.experiment_name
        rows = open(d / "train.csv").read().strip().splitlines()
        assert rows[0].startswith("critic/critic_loss") and len(rows) == 1 + cfg.steps // cfg.log_interval
        assert len(open(d / "val.csv").read().strip().splitlines()) == len(rows)
        assert (d / "params.pkl").exists()
        agent = load_agent(d, task.sample("train", 1))
        assert agent.step == cfg.steps
    # resumable state
    sd = trainer.state_dict()
    assert set(sd) >= {"experiments", "candidates", "untrained_candidates", "finished_candidates"}


def test_population_members_are_independent_in_trainer(tmp_path):
    """A member trained inside a population reaches the same state as the same
    member trained alone (lock-step batching changes nothing per member)."""
    from hpo.identity import Identity
    from task.offline_task_synthetic import OfflineTaskSynthetic
    from trainer.config import ExperimentConfig
    from trainer.trainer import Trainer
    task = OfflineTaskSynthetic(n_rows=5_000, n_val_rows=500, num_evaluation_envs=2, max_episode_steps=4)
    cfg = _trainer_config(tmp_path, steps=6, eval_interval=6, log_interval=3)
    c1, c2 = ExperimentConfig(seed=11, alpha=5.0), ExperimentConfig(seed=12, alpha=50.0)
    t_pair = Trainer(task, Identity([c1, c2], 0), cfg)
    t_pair.train(max_evaluations=2)
    t_solo = Trainer(task, Identity([c2], 0), cfg)
    t_solo.train(max_evaluations=1)
    from fql.utils.serialization import params_of
    a = params_of(t_pair.experiments[c2].agent.to_state_dict())
    b = params_of(t_solo.experiments[c2].agent.to_state_dict())
    for net in O.NETS:
        for leaf in a[net]:
            assert np.array_equal(a[net][leaf], b[net][leaf]), (net, leaf)


def test_tune_alpha_driver(tmp_path):
    import tune_alpha
    common = [f"--save_directory={tmp_path}", "--steps=20", "--eval_interval=10", "--log_interval=10",
              f"--agent.actor_hidden_dims={SMALL}", f"--agent.value_hidden_dims={SMALL}",
              "--agent.batch_size=64", "--agent.layer_norm", "--eval_episodes=4", "--synthetic_rows=5000"]
    tune_alpha.main(common + ["--number_of_alphas=3", "--number_of_seeds=2", "--max_evaluations=100"])
    ckpt = tmp_path / "cube-single-play-singletask-task2-v0" / "checkpoint.pkl"
    with open(ckpt, "rb") as f:
        state = pickle.load(f)
    assert len(state["trainer"]["experiments"]) == 6
    assert all(e["current_step"] == 20 for e in state["trainer"]["experiments"].values())
    # resume: loading the checkpoint and training further is a no-op at the end
    tune_alpha.main(common + ["--number_of_alphas=3", "--number_of_seeds=2", "--max_evaluations=6"])
    # single-experiment mode (scripts/tune-alpha-*.sh) writes a checkpoint per eval_interval
    tune_alpha.main(common + ["--number_of_alphas=3", "--number_of_seeds=2", "--single_experiment", "--job_id=4"])
    ckpts = list((tmp_path / "cube-single-play-singletask-task2-v0").glob("*/checkpoint_20.pkl"))
    assert len(ckpts) >= 1


def test_tune_alpha_two_ranks_and_resume(tmp_path):
    """tune_alpha.py under torch.distributed.run (2 ranks sharing this box's GPU, gloo):
    halving over the world-model scores (4 candidates, 8 evaluations: milestones [4, 2],
    so 4 -> 2 after the second round, when the budget is spent), rank 0 writes the
    reference-shaped checkpoint, and a one-rank run resumes from it to the end."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = os.path.join(root, "flow-q-learning_amd", "tune_alpha.py")
    args = [f"--save_directory={tmp_path}", "--steps=40", "--eval_interval=10", "--log_interval=10",
            "--agent.batch_size=64", "--agent.layer_norm", "--eval_episodes=8", "--synthetic_rows=5000",
            "--task=simulated", "--max_episode_steps=20", "--number_of_alphas=4", "--number_of_seeds=1",
            "--strategy=successive_halving", "--fraction=0.5", "--history_length=1", "--max_evaluations=8"]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), script] + args,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ckpt = tmp_path / "cube-single-play-singletask-task2-v0" / "checkpoint.pkl"

    def load():
        with open(ckpt, "rb") as f:
            return pickle.load(f)
    state = load()
    tr = state["trainer"]
    assert len(tr["experiments"]) == 4 and len(tr["candidates"]) == 2  # every member recorded, 2 pruned
    assert all(tr["experiments"][c]["current_step"] == 20 for c in tr["candidates"])
    assert tr["round_index"] == 2 and len(state["strategy"]["candidate_scores"]) == 4
    import tune_alpha
    tune_alpha.main(args)  # resume on one rank: the two survivors train to the end
    tr = load()["trainer"]
    assert len(tr["candidates"]) == 2 and set(tr["finished_candidates"]) == set(tr["candidates"])
    assert all(tr["experiments"][c]["current_step"] == 40 for c in tr["candidates"])


def test_integration_md_binding_stub():
    """The reference-side ctypes stub printed in INTEGRATION.md section 3 runs
    against the built library and agrees with the shipped surface."""
    import fqlpop._lib as L
    from trainer.config import AgentConfig
    from dataclasses import asdict
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "INTEGRATION.md")).read()
    code = text.split("```python", 1)[1].split("```", 1)[0]
    code = code.replace('ctypes.CDLL("libfqlpop.so")', f'ctypes.CDLL({L.LIB_PATH!r})')
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    cfg = asdict(AgentConfig(actor_hidden_dims=(64,) * 4, value_hidden_dims=(64,) * 4, batch_size=64))
    rng = np.random.default_rng(3)
    ocfg = O.OracleConfig(hidden_dims=(64,) * 4, batch_size=64)
    batch = O.cast_tree(O.make_batch(ocfg, 64, rng), np.float32)
    agent = ns["FQLAgent"].create(5, batch["observations"][:1], batch["actions"][:1], cfg)
    agent, info = agent.update(batch)
    assert set(info) == set(O.TRAIN_INFO_KEYS) and all(np.isfinite(v) for v in info.values())
    loss, vinfo = agent.total_loss(batch)
    assert np.isfinite(loss) and len(vinfo) == 10
    acts = agent.sample_actions(batch["observations"][:9], seed=np.array([0, 1], np.uint32))
    assert acts.shape == (9, 5) and np.all(np.abs(acts) <= 1)
