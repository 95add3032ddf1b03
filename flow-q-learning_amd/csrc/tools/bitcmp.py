"""Bit-identity check between builds (developer tool, on the GPU box from the repo root).

Runs 20 device-sampled population steps of the cube headline shape (4 members, B = 256,
H = 512) and prints a SHA-256 over every member's parameters and the last info rows.
Run it once per build (FQLPOP_LIB selects a second library) and compare the digests:
    python flow-q-learning_amd/csrc/tools/bitcmp.py
    FQLPOP_LIB=$PWD/flow-q-learning_amd/csrc/devlib/libfqlpop_ref.so python flow-q-learning_amd/csrc/tools/bitcmp.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "flow-q-learning_amd"))

from fqlpop import Population, PopulationConfig  # noqa: E402
from fqlpop._lib import STATE_PARAMS  # noqa: E402


def main():
    n, D, A = 50_000, 28, 5
    rng = np.random.default_rng(0)
    obs = rng.standard_normal((n, D), dtype=np.float32)
    rew = (rng.random(n) < 0.05).astype(np.float32) - 1.0
    data = {
        "observations": obs,
        "actions": rng.uniform(-1 + 1e-5, 1 - 1e-5, (n, A)).astype(np.float32),
        "rewards": rew,
        "masks": (1.0 - (rew == 0)).astype(np.float32),
        "next_observations": (obs + 0.05 * rng.standard_normal((n, D))).astype(np.float32),
    }
    pop = Population(PopulationConfig(), [3.0, 10.0, 100.0, 1000.0], [11, 12, 13, 14], device=0)
    pop.set_dataset(data)
    pop.step(20)
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(pop.read_info_array()).tobytes())
    for m in range(4):
        h.update(np.ascontiguousarray(pop.get_flat(m, STATE_PARAMS)).tobytes())
    pop.close()
    print("bitcmp", os.environ.get("FQLPOP_LIB", "in-tree"), h.hexdigest())


if __name__ == "__main__":
    main()
