"""Diagnostics: run N population steps of the bench workload and close, so that the
FQLPOP_PHASE_PROBE reports (printed on stderr at destroy) describe in-step launches.

  make -C flow-q-learning_amd/csrc PHASE=1 OUT=devlib/libfqlpop_phase.so   # stamps compiled in
  FQLPOP_LIB=$PWD/flow-q-learning_amd/csrc/devlib/libfqlpop_phase.so FQLPOP_PHASE_PROBE=1 \
      python flow-q-learning_amd/csrc/tools/phase_run.py [steps] [workload] [NAME=VALUE engine options ...]
(the production build compiles the stamps out: their disabled branch cost 0.3 % in the step)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
import bench  # noqa: E402  (the bench's workload table and synthetic dataset)
from fqlpop import Population, PopulationConfig, set_engine_option  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
wl = bench.WORKLOADS[sys.argv[2] if len(sys.argv) > 2 else "cube"]
members = 16
for kv in sys.argv[3:]:  # e.g. serial=1: one stream, each launch uncontended; members=2: population size
    k, v = kv.split("=")
    if k == "members":
        members = int(v)
    else:
        set_engine_option(k, int(v))
rows = 200_000
data = bench.synthetic_dataset(rows, wl["obs_dim"], wl["action_dim"])
alphas, seeds = bench.population_values(members)
pop = Population(PopulationConfig(obs_dim=wl["obs_dim"], action_dim=wl["action_dim"],
                                  batch_size=wl["batch_size"]), alphas, seeds)
pop.set_dataset({k: torch.as_tensor(v).cuda() for k, v in data.items()})
pop.step(steps)
pop.sync()
pop.close()
print("phase_run done", steps, "steps", flush=True)
