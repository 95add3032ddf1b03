"""BASELINE config C4 on the HIP path: tune_alpha.py with a 64-alpha cube population
(B = 256, H = 512 x 4, critic LayerNorm) under SuccessiveHalving f = 0.5, h = 4, sharded
over two ranks (both on this box's one GPU, gloo for the collectives) against the same
sweep in one process.  Reference: tune_alpha.py:40-87, hpo/successive_halving.py:53-115,
trainer/trainer.py:69-120."""
import os
import pickle
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import fql_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = "cube-single-play-singletask-task2-v0"

# 8 rounds of 10 updates; SuccessiveHalving over a horizon of 8 evaluations per candidate:
# milestones [6, 5, 4, 4, 4, 4], so 64 -> 32 -> 16 -> 8 after rounds 4, 5 and 6.
ARGS = ["--steps=80", "--eval_interval=10", "--log_interval=10", "--agent.batch_size=256", "--agent.layer_norm",
        "--eval_episodes=16", "--synthetic_rows=20000", "--task=simulated", "--max_episode_steps=20",
        "--number_of_alphas=64", "--number_of_seeds=1", "--strategy=successive_halving", "--fraction=0.5",
        "--history_length=4", "--halving_horizon=8", "--max_evaluations=100000", "--env_model=baseline"]


def _load(save_dir):
    with open(os.path.join(save_dir, ENV, "checkpoint.pkl"), "rb") as f:  # written by tune_alpha.py
        return pickle.load(f)


def test_c4_64_alpha_halving_two_ranks_match_one_process(tmp_path):
    from fql.utils.serialization import flax_to_flat
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = os.path.join(ROOT, "flow-q-learning_amd", "tune_alpha.py")
    d2, d1 = str(tmp_path / "w2"), str(tmp_path / "w1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), script,
                        f"--save_directory={d2}"] + ARGS, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run([sys.executable, script, f"--save_directory={d1}"] + ARGS, capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    two, one = _load(d2), _load(d1)
    t2, t1 = two["trainer"], one["trainer"]
    # the same decisions: 64 -> 32 -> 16 -> 8 survivors, every member ever created recorded
    assert len(t1["experiments"]) == len(t2["experiments"]) == 64
    assert set(t1["candidates"]) == set(t2["candidates"]) and len(t1["candidates"]) == 8
    assert t1["round_index"] == t2["round_index"] == 8
    s1, s2 = one["strategy"]["candidate_scores"], two["strategy"]["candidate_scores"]
    assert s1 == s2
    assert sorted(len(v) for v in s1.values()) == [4] * 32 + [5] * 16 + [6] * 8 + [8] * 8
    # survivors bit-identical (parameters, Adam state) and trained to the end
    for c in t1["candidates"]:
        e1, e2 = t1["experiments"][c], t2["experiments"][c]
        assert e1["current_step"] == e2["current_step"] == 80
        f1, f2 = flax_to_flat(e1["agent"]), flax_to_flat(e2["agent"])
        assert f1["opt_state"]["count"] == f2["opt_state"]["count"] == 80
        for part in ("params",):
            for net in f1[part]:
                for k, v in f1[part][net].items():
                    np.testing.assert_array_equal(v, f2[part][net][k], err_msg=f"{c} {net}/{k}")
        for m in ("mu", "nu"):
            for net in f1["opt_state"][m]:
                for k, v in f1["opt_state"][m][net].items():
                    np.testing.assert_array_equal(v, f2["opt_state"][m][net][k])

    # one survivor's next update (its trained state: step 81's Adam bias corrections) on an
    # injected batch against the float64 oracle
    from fqlpop import Population, PopulationConfig
    c = sorted(t1["candidates"], key=lambda x: x.alpha)[0]
    flat = flax_to_flat(t1["experiments"][c]["agent"])
    cfg = O.OracleConfig(hidden_dims=(512,) * 4, batch_size=256, alpha=c.alpha)
    pop = Population(PopulationConfig(hidden_dims=(512,) * 4, batch_size=256), [c.alpha], [c.seed])
    pop.load_state_dict(0, flat)
    p = O.cast_tree(flat["params"], np.float64)
    opt = {"m": O.cast_tree(flat["opt_state"]["mu"], np.float64), "v": O.cast_tree(flat["opt_state"]["nu"], np.float64),
           "count": 80}
    rng = np.random.default_rng(64)
    b = O.cast_tree(O.make_batch(cfg, 256, rng), np.float32)
    n = O.cast_tree(O.make_noise(cfg, 256, rng), np.float32)
    pop.step_injected([b], [n])
    _, _, want = O.update(cfg, p, opt, O.cast_tree(b, np.float64), O.cast_tree(n, np.float64))
    got = pop.read_info()[0]
    for k in O.TRAIN_INFO_KEYS:
        assert abs(got[k] - want[k]) <= 1e-4 * max(abs(got[k]), abs(want[k])) + 1e-6, (k, got[k], want[k])
    assert pop.get_count(0) == 81
    pop.close()


ANT = "antsoccer-arena-navigate-singletask-task4-v0"
# BASELINE config C5's shape: a 32-alpha antsoccer population (obs 42, act 8, B = 1024) scored
# by the on-GPU world-model rollout (the multistep env model, 50 envs per member) every round
ARGS_C5 = ["--steps=20", "--eval_interval=10", "--log_interval=10", "--agent.batch_size=1024",
           "--agent.layer_norm", "--eval_episodes=50", "--synthetic_rows=20000", "--task=simulated",
           "--max_episode_steps=30", "--number_of_alphas=32", "--number_of_seeds=1", "--strategy=identity",
           "--max_evaluations=100000", "--env_model=multistep", f"--env_name={ANT}"]


def test_c5_32_alpha_antsoccer_world_model_eval_two_ranks_match_one_process(tmp_path):
    """C5 end to end: tune_alpha.py --task simulated trains the 32-member ant population and
    scores every member by the world-model rollout each round (task/offline_task_simulated.py:
    85-107, evaluator/evaluation.py:93-114); two ranks sharing the GPU against one process:
    the same eval scores for every member and every round, and bit-identical parameters and
    Adam state."""
    from fql.utils.serialization import flax_to_flat
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = os.path.join(ROOT, "flow-q-learning_amd", "tune_alpha.py")
    d2, d1 = str(tmp_path / "w2"), str(tmp_path / "w1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), script,
                        f"--save_directory={d2}"] + ARGS_C5, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run([sys.executable, script, f"--save_directory={d1}"] + ARGS_C5, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    load = lambda d: pickle.load(open(os.path.join(d, ANT, "checkpoint.pkl"), "rb"))  # noqa: E731
    two, one = load(d2), load(d1)
    t2, t1 = two["trainer"], one["trainer"]
    assert len(t1["experiments"]) == len(t2["experiments"]) == 32
    assert t1["round_index"] == t2["round_index"] == 2
    for c, e1 in t1["experiments"].items():
        e2 = t2["experiments"][c]
        # every round's world-model evaluation of the member (its eval.csv: success rate, ...)
        rows = [open(os.path.join(d, ANT, e["experiment_name"], "eval.csv")).read() for d, e in ((d1, e1), (d2, e2))]
        assert rows[0] == rows[1] and len(rows[0].strip().splitlines()) == 1 + 2, (c, rows)
        assert e1["current_step"] == e2["current_step"] == 20
        f1, f2 = flax_to_flat(e1["agent"]), flax_to_flat(e2["agent"])
        for net in f1["params"]:
            for k, v in f1["params"][net].items():
                np.testing.assert_array_equal(v, f2["params"][net][k], err_msg=f"{c} {net}/{k}")
        for m in ("mu", "nu"):
            for net in f1["opt_state"][m]:
                for k, v in f1["opt_state"][m][net].items():
                    np.testing.assert_array_equal(v, f2["opt_state"][m][net][k])
    # the ant shapes: the critic's first Dense takes [obs 42; act 8]
    c0 = next(iter(t1["experiments"]))
    assert flax_to_flat(t1["experiments"][c0]["agent"])["params"]["critic"]["Dense_0/kernel"].shape[-2] == 50
