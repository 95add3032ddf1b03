"""Step rate right after setup, in chunks (developer tool, on the GPU box):

  python flow-q-learning_amd/csrc/tools/step_ramp.py [chunk] [n_chunks] [idle_s] [preheat_ms] [mem] [graph|eager]

(mem = 1: the preheat also streams HBM: device-to-device copies of a 1 GB buffer on a side
stream while the dominant kernel replays)

Builds the bench population (cube, 16 members, 1M rows), runs 5 warmup steps, then
times n_chunks back-to-back chunks of `chunk` steps (host-synchronised each), then
idles idle_s seconds and times 3 more chunks.  Shows how long the step rate takes
to reach its steady state (clocks, caches, first graph replays).
"""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "flow-q-learning_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from fqlpop import Population, PopulationConfig  # noqa: E402


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n_chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    idle = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    preheat_ms = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
    mem = len(sys.argv) > 5 and sys.argv[5] == "1"
    graph = not (len(sys.argv) > 6 and sys.argv[6] == "eager")  # eager: no hipGraph replays
    torch.cuda.set_device(0)
    wl = bench.WORKLOADS["cube"]
    data = bench.synthetic_dataset(1_000_000, wl["obs_dim"], wl["action_dim"])
    alphas, seeds = bench.population_values(16)
    pop = Population(PopulationConfig(obs_dim=wl["obs_dim"], action_dim=wl["action_dim"],
                                      batch_size=wl["batch_size"], use_graph=graph), alphas, seeds, device=0)
    pop.set_dataset(data)
    if preheat_ms > 0:  # as bench.py --preheat-ms
        us, _ = pop.time_dominant_kernel(1)
        if mem:
            src = torch.empty(256 << 20, dtype=torch.float32, device="cuda")
            dst = torch.empty_like(src)
            side = torch.cuda.Stream()
            with torch.cuda.stream(side):
                for _ in range(int(preheat_ms / 0.35)):  # ~2 GB moved per copy, ~0.35 ms at ~6 TB/s
                    dst.copy_(src)
        pop.time_dominant_kernel(max(1, int(preheat_ms * 1e3 / us)))
        torch.cuda.synchronize()
    pop.step(5)
    pop.sync()

    def timed(tag):
        t0 = time.perf_counter()
        pop.step(chunk)
        pop.sync()
        el = time.perf_counter() - t0
        c = bench.gpu_clock_power(0)
        print(f"{tag} {chunk} steps: {1e3 * el / chunk:.4f} ms/step  {16 * chunk / el:.1f} member-steps/s  "
              f"sclk {c['sclk_mhz']} mclk {c['mclk_mhz']} fclk {c['fclk_mhz']} {c['power_w']} W", flush=True)

    for i in range(n_chunks):
        timed(f"chunk {i:2d}")
    time.sleep(idle)
    for i in range(3):
        timed(f"after {idle:.1f} s idle, chunk {i}")
    pop.close()


if __name__ == "__main__":
    main()
