"""Generate the golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).  Needs /root/reference for the
reference-pinned fixtures; the committed outputs are what the tests read.

Fixtures
--------
* ``reference_hpo.json``       -- milestones and sample() traces of the
  REFERENCE SuccessiveHalving (reference hpo/successive_halving.py:10-115),
  produced by importing the reference module in a subprocess.
* ``reference_argparser.json`` -- TrainerConfig built by the REFERENCE
  argparser (reference argparser.py:9-169) for several argv lists.
* ``reference_env_model_argparser.json`` -- EnvModelTrainerConfig built by the
  REFERENCE env-model argparser (reference argparser.py:172-290).
* ``reference_seeds.json``     -- alpha grid / seed draws of reference
  tune_alpha.py:40-46 and the seeds recorded in the reference's
  results/real_success_rates_{cube,antsoccer}.csv.
* ``oracle_update_h64.npz``    -- two consecutive update() steps of the
  float64 oracle (H=64, B=64, cube shapes): params in/out, batches, noises,
  info.  A REGRESSION fixture of our own restatement (the reference's
  per-step FQL update cannot run here: parity unpinned).
"""
from __future__ import annotations

import csv
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

REF_SCRIPT = r'''
import json, sys
sys.path.insert(0, "/root/reference")
from hpo.successive_halving import SuccessiveHalving
from trainer.config import ExperimentConfig
import argparser

out = {"hpo": [], "argparser": []}
cases = [(16, 50, 0.5, 1), (64, 200, 0.5, 4), (27, 40, 0.5, 1), (10, 30, 0.3, 2), (8, 12, 0.75, 1)]
for n, e, f, h in cases:
    pop = [ExperimentConfig(seed=i, alpha=float(i)) for i in range(n)]
    s = SuccessiveHalving(set(pop), e, f, h)
    trace = []
    # deterministic score script: candidate i scores ((i * 37 + step * 11) % 101) / 100
    for step in range(1, e + 1):
        for c in sorted(s.population, key=lambda c: c.seed):
            s.update(c, ((c.seed * 37 + step * 11) % 101) / 100.0)
        kept = sorted(c.seed for c in s.sample())
        trace.append(kept)
    out["hpo"].append({"n": n, "total": e, "fraction": f, "history": h,
                       "milestones": s.halving_milestones, "trace": trace})
argvs = [[], ["--agent.layer_norm"], ["--agent.layer_norm", "--agent.alpha=216.8", "--steps=2000",
          "--agent.batch_size=1024", "--agent.q_agg=min", "--eval_interval=20000", "--use_wandb"],
         ["--agent.actor_hidden_dims=(256, 256)", "--agent.value_hidden_dims=(256,256)",
          "--agent.flow_steps=5", "--seed=3", "--env_name=antsoccer-arena-navigate-singletask-task4-v0"]]
for argv in argvs:
    cfg = argparser.build_config_from_args(argparser.get_argparser().parse_args(argv))
    d = dict(vars(cfg))
    d["agent"] = dict(vars(cfg.agent))
    d["save_directory"] = str(d["save_directory"])
    d["data_directory"] = str(d["data_directory"])
    out["argparser"].append({"argv": argv, "config": d})
out["env_model_argparser"] = []
em_argvs = [[], ["--model=baseline", "--termination_weight=0"],
            ["--model=termination_predictor", "--steps=40000"],
            ["--model=multistep", "--model.hidden_dims=(64, 64)", "--sequence_length=128", "--seed=4",
             "--env_name=antsoccer-arena-navigate-singletask-task4-v0"]]
for argv in em_argvs:
    cfg = argparser.build_env_model_config_from_args(argparser.get_env_model_argparser().parse_args(argv))
    d = dict(vars(cfg))
    d["save_directory"] = str(d["save_directory"])
    d["data_directory"] = str(d["data_directory"])
    d["model_config"] = {k: list(v) if isinstance(v, tuple) else v for k, v in d["model_config"].items()}
    out["env_model_argparser"].append({"argv": argv, "config": d})
print(json.dumps(out))
'''


def reference_fixtures():
    res = subprocess.run([sys.executable, "-c", REF_SCRIPT], cwd="/tmp", check=True, capture_output=True, text=True)
    data = json.loads(res.stdout)
    with open(os.path.join(HERE, "reference_hpo.json"), "w") as f:
        json.dump(data["hpo"], f)
    with open(os.path.join(HERE, "reference_argparser.json"), "w") as f:
        json.dump(data["argparser"], f, indent=1)
    with open(os.path.join(HERE, "reference_env_model_argparser.json"), "w") as f:
        json.dump(data["env_model_argparser"], f, indent=1)

    import random
    seeds = {}
    for k in (1, 2, 16, 64, 128):
        random.seed(0)
        seeds[str(k)] = random.sample(range(10000), k)
    recorded = {}
    for task in ("cube", "antsoccer"):
        with open(os.path.join(REF, "results", f"real_success_rates_{task}.csv")) as f:
            rows = list(csv.DictReader(f))
        recorded[task] = {"seeds": sorted({int(r["seed"]) for r in rows}),
                          "alphas": sorted({float(r["alpha"]) for r in rows})}
    alphas = {str(n): np.logspace(np.log10(3), np.log10(1000), num=n).tolist() for n in (16, 20, 64)}
    with open(os.path.join(HERE, "reference_seeds.json"), "w") as f:
        json.dump({"random_sample_seed0": seeds, "results_csv": recorded, "alpha_logspace": alphas}, f, indent=1)


def oracle_fixture():
    sys.path.insert(0, ROOT)
    from oracle import fql_oracle as O
    cfg = O.OracleConfig(hidden_dims=(64,) * 4, batch_size=64, alpha=30.0)
    rng = np.random.default_rng(2024)
    p32 = O.cast_tree(O.init_params(cfg, 5), np.float32)
    p = O.cast_tree(p32, np.float64)
    opt = O.init_opt_state(p)
    out = {}
    for name, leaf_tree in (("in", p32),):
        for net in O.NETS:
            for k, v in leaf_tree[net].items():
                out[f"params_{name}/{net}/{k}"] = v
    for step in range(2):
        b = O.cast_tree(O.make_batch(cfg, 64, rng), np.float32)
        n = O.cast_tree(O.make_noise(cfg, 64, rng), np.float32)
        p, opt, info = O.update(cfg, p, opt, O.cast_tree(b, np.float64), O.cast_tree(n, np.float64))
        for k, v in b.items():
            out[f"batch{step}/{k}"] = v
        for k, v in n.items():
            out[f"noise{step}/{k}"] = v
        out[f"info{step}"] = np.array([info[k] for k in O.TRAIN_INFO_KEYS], np.float64)
    for net in O.NETS:
        for k, v in p[net].items():
            out[f"params_out/{net}/{k}"] = v.astype(np.float32)
    out["config"] = np.array([64, 64, 30.0])
    np.savez_compressed(os.path.join(HERE, "oracle_update_h64.npz"), **out)


if __name__ == "__main__":
    if os.path.isdir(REF):
        reference_fixtures()
    oracle_fixture()
    print("golden fixtures written to", HERE)
