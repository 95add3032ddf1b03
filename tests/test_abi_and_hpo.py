"""CPU tests: the C ABI library loads and exports every symbol include/fqlpop.h
declares; the HPO strategies, argparser and alpha/seed grid match the
REFERENCE implementation's outputs (tests/golden/reference_*.json, produced by
importing the reference modules: tests/golden/make_golden.py)."""
import json
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def header_symbols():
    text = open(os.path.join(ROOT, "include", "fqlpop.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fqlpop_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    import fqlpop
    lib = fqlpop.load_library()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(fqlpop.EXPORTED_SYMBOLS)


def test_library_reports_errors_without_gpu():
    import ctypes
    import fqlpop
    from fqlpop._lib import Config
    lib = fqlpop.load_library()
    c = Config(obs_dim=28, action_dim=5, hidden_dim=100, num_hidden=4, batch_size=256, num_qs=2,
               layer_norm=1, actor_layer_norm=0, flow_steps=10, q_agg_min=0, normalize_q_loss=0,
               discount=0.99, tau=0.005, lr=3e-4, use_graph=1)
    a = np.ones(1, np.float32)
    s = np.ones(1, np.uint64)
    h = ctypes.c_void_p()
    rc = lib.fqlpop_create(ctypes.byref(c), 1, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                           s.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 0, ctypes.byref(h))
    assert rc == -1 and b"hidden_dim" in lib.fqlpop_last_error()
    # FLOP count of SURVEY.md 8(d): 12.334 GFLOP per cube member-step
    c.hidden_dim = 512
    assert abs(lib.fqlpop_flops_per_member_step(ctypes.byref(c)) / 1e9 - 12.334) < 5e-3


def test_successive_halving_matches_reference_traces():
    from hpo.successive_halving import SuccessiveHalving
    from trainer.config import ExperimentConfig
    for case in json.load(open(os.path.join(GOLDEN, "reference_hpo.json"))):
        pop = {ExperimentConfig(seed=i, alpha=float(i)) for i in range(case["n"])}
        s = SuccessiveHalving(pop, case["total"], case["fraction"], case["history"])
        assert s.halving_milestones == case["milestones"]
        for step, kept in enumerate(case["trace"], start=1):
            for c in sorted(s.population, key=lambda c: c.seed):
                s.update(c, ((c.seed * 37 + step * 11) % 101) / 100.0)
            assert sorted(c.seed for c in s.sample()) == kept, (case["n"], step)


def test_successive_halving_known_answer_and_state_roundtrip():
    from hpo.identity import Identity
    from hpo.successive_halving import SuccessiveHalving
    from trainer.config import ExperimentConfig
    pop = {ExperimentConfig(seed=i, alpha=1.0 * i) for i in range(16)}
    s = SuccessiveHalving(pop, total_evaluations=50, fraction=0.5, history_length=1)
    assert s.halving_milestones == [25, 13, 7, 4]
    for c in pop:
        s.update(c, c.alpha)
    s2 = SuccessiveHalving(pop, 50, 0.5, 1, state_dict=s.state_dict())
    assert s2.performed_evaluations == 1 and dict(s2.candidate_scores) == dict(s.candidate_scores)
    ident = Identity(population=list(pop), total_evaluations=0)
    ident.update(next(iter(pop)), 1.0)
    assert ident.sample() == list(pop)


def test_argparser_matches_reference():
    from argparser import build_config_from_args, get_argparser
    for case in json.load(open(os.path.join(GOLDEN, "reference_argparser.json"))):
        cfg = build_config_from_args(get_argparser().parse_args(case["argv"]))
        got = dict(vars(cfg))
        got["agent"] = dict(vars(cfg.agent))
        got["save_directory"] = str(got["save_directory"])
        got["data_directory"] = str(got["data_directory"])
        want = case["config"]
        for k in ("actor_hidden_dims", "value_hidden_dims"):
            want["agent"][k] = tuple(want["agent"][k])
            got["agent"][k] = tuple(got["agent"][k])
        assert got == want, case["argv"]


def test_population_grid_matches_reference_runs():
    """alpha = logspace(3, 1000, n), seeds = random.sample(...) after seed(0) --
    the seeds of the reference's logged runs (results/real_success_rates_*.csv)."""
    import sys
    sys.path.insert(0, ROOT)
    from bench import population_values
    ref = json.load(open(os.path.join(GOLDEN, "reference_seeds.json")))
    for n, seeds in ref["random_sample_seed0"].items():
        alphas, got = population_values(int(n))
        assert got == seeds
        if n in ref["alpha_logspace"]:
            assert np.allclose(alphas, ref["alpha_logspace"][n])
    assert ref["random_sample_seed0"]["2"] == ref["results_csv"]["cube"]["seeds"]
    assert np.allclose(sorted(ref["alpha_logspace"]["20"]), ref["results_csv"]["cube"]["alphas"])


def test_synthetic_task_contract():
    from task.offline_task_synthetic import OfflineTaskSynthetic
    t = OfflineTaskSynthetic(n_rows=5000, n_val_rows=500, num_evaluation_envs=4, max_episode_steps=5)
    b = t.sample("train", 7)
    assert b["observations"].shape == (7, 28) and b["actions"].shape == (7, 5)
    assert set(np.unique(b["rewards"])) <= {-1.0, 0.0}
    assert np.all(b["masks"] == 1.0 - (b["rewards"] == 0))
    assert np.all(np.abs(t.train_dataset["actions"]) < 1)
    obs, _ = t.reset(seed=0)
    done = np.zeros(4, bool)
    for _ in range(5):
        obs, r, term, trunc, infos = t.step(np.zeros((4, 5)))
        done |= term | trunc
    assert done.all()
    from evaluator.evaluation import evaluate_actor_fn
    stats, trans = evaluate_actor_fn(lambda observations, temperature, seed=None: np.zeros((4, 5)), t, seed=1)
    assert 0.0 <= stats["success"] <= 1.0 and len(trans) == 5
