"""Which leaves differ between two engine-option sets after n device-sampled steps
(developer tool for bit-identity checks of alternate kernels).

  python ws_diff.py "dw_tile_critic=6,dw_tile_actor=6" [steps] [H] [B]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flow-q-learning_amd")]
import numpy as np  # noqa: E402

from fqlpop import Population, PopulationConfig, reset_engine_options, set_engine_option  # noqa: E402


def run(opts, steps, H, B):
    reset_engine_options()
    for kv in filter(None, opts.split(",")):
        k, v = kv.split("=")
        set_engine_option(k, int(v))
    rng = np.random.default_rng(7)
    N = 4000
    obs = rng.standard_normal((N, 28)).astype(np.float32)
    rew = np.where(rng.uniform(size=N) < 0.05, 0.0, -1.0).astype(np.float32)
    data = {"observations": obs, "actions": rng.uniform(-1, 1, (N, 5)).astype(np.float32),
            "rewards": rew, "masks": (1.0 - (rew == 0)).astype(np.float32),
            "next_observations": (obs + 0.05 * rng.standard_normal((N, 28))).astype(np.float32)}
    pop = Population(PopulationConfig(hidden_dims=(H,) * 4, batch_size=B), [3.0, 30.0, 300.0], [5, 6, 7])
    pop.set_dataset(data)
    pop.step(steps)
    out = {w: [pop.get_flat(i, w) for i in range(3)] for w in (0, 1, 2)}
    leaves = pop.leaves
    pop.close()
    reset_engine_options()
    return out, leaves


opts = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
H = int(sys.argv[3]) if len(sys.argv) > 3 else 512
B = int(sys.argv[4]) if len(sys.argv) > 4 else 256
a, leaves = run("", steps, H, B)
b, _ = run(opts, steps, H, B)
names = {0: "params", 1: "adam_m", 2: "adam_v"}
nd = 0
for w in (0, 1, 2):
    for i in range(3):
        for name, off, shape in leaves:
            n = int(np.prod(shape))
            x, y = a[w][i][off:off + n], b[w][i][off:off + n]
            if not np.array_equal(x, y):
                d = np.abs(x.astype(np.float64) - y)
                idx = np.nonzero(x != y)[0]
                nd += 1
                print(f"{names[w]} member {i} {name} {shape}: {idx.size}/{n} differ, max {d.max():.3g}, first {idx[:8].tolist()}")
                if i == 0 and name.startswith("critic/Dense_0") and "--values" in sys.argv:
                    for j in idx[:6]:
                        print(f"    [{j}] {x[j]!r} vs {y[j]!r}  (params_a {a[0][i][off + j]!r})")
print("differing leaves:", nd)
