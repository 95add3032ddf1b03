"""Multistep env-model kernel time split (developer tool, under rocprofv3 --kernel-trace):
train steps (forward + BPTT) and eval steps (forward only) of the same kernel.

  rocprofv3 --kernel-trace --stats -d out -o run -- python em_time.py [T]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flow-q-learning_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import envmodel as em  # noqa: E402
from envmodel.trainer import EnvModelTrainerConfig, StatePredictorTrainer  # noqa: E402
import train_env_model as tem  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 256
wl = bench.WORKLOADS["cube"]
data = bench.synthetic_dataset(200_000, wl["obs_dim"], wl["action_dim"])
ds = {k: data[k] for k in ("observations", "actions", "rewards", "next_observations")}
spec = em.EnvModelSpec(wl["obs_dim"], wl["action_dim"])
ld = tem.MultistepLoader(ds, T)
cfg = EnvModelTrainerConfig(steps=100, model="multistep", sequence_length=T, termination_weight=0.0)
tr = StatePredictorTrainer(spec, em.init_state_predictor(spec, 0), ld, None, cfg)
tr.steps(10)
tr.sync()
np.random.seed(0)
b = ld.sample(256)
for _ in range(10):
    tr.eval_step(None, b)
tr.sync()
tr.close()
print("em_time done", flush=True)
