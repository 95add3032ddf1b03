"""Multistep env-model training, the two BPTT paths side by side on one GPU (developer A/B):
engine option em_seq_sweep 1 (em_sweep_kernel + em_seq_dw_kernel) against 0 (round 5's
em_seq_grad_kernel).  Reference defaults: B = 256, T = 256, hidden (128, 256, 128), cube
shapes; termination_weight 0 and 1 (the reference argparser's default, with a frozen
termination predictor).  Prints one JSON line per (path, tw): train steps/s and the logs
after the same device-sampled steps.

  python flow-q-learning_amd/csrc/tools/em_multistep_ab.py [steps] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "flow-q-learning_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import envmodel as em  # noqa: E402
from envmodel.trainer import EnvModelTrainerConfig, StatePredictorTrainer  # noqa: E402
from fqlpop import set_engine_option  # noqa: E402


class _Loader:
    def __init__(self, ds):
        self.dataset = ds


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    D, A, n = 28, 5, 200_000
    rng = np.random.default_rng(0)
    obs = rng.standard_normal((n, D)).astype(np.float32)
    ds = {"observations": obs, "actions": rng.uniform(-1, 1, (n, A)).astype(np.float32),
          "next_observations": (obs + 0.05 * rng.standard_normal((n, D))).astype(np.float32),
          "rewards": np.where(rng.uniform(size=n) < 0.05, 0.0, -1.0).astype(np.float32)}
    for rep in range(reps):
        for tw in (0.0, 1.0):
            for path in (1, 0):
                set_engine_option("em_seq_sweep", path)
                spec = em.EnvModelSpec(D, A, (128, 256, 128), (128, 256, 128))
                cfg = EnvModelTrainerConfig(steps=1000, model="multistep", sequence_length=256,
                                            termination_weight=tw, batch_size=256)
                tr = StatePredictorTrainer(spec, em.init_state_predictor(spec, 0), _Loader(ds), None, cfg,
                                           tp_params=em.init_termination_predictor(spec, 1) if tw > 0 else None)
                tr.steps(3)
                tr.sync()
                t0 = time.perf_counter()
                tr.steps(steps)
                tr.sync()
                el = time.perf_counter() - t0
                logs = tr.read_logs()
                print(json.dumps({"rep": rep, "em_seq_sweep": path, "termination_weight": tw,
                                  "train_steps_per_s": round(steps / el, 2), "ms_per_step": round(1e3 * el / steps, 3),
                                  "logs": {k: round(float(v), 6) for k, v in logs.items()}}), flush=True)
                tr.close()
    set_engine_option("em_seq_sweep", 1)


if __name__ == "__main__":
    main()
