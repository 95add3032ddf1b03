"""North-star benchmark: FQL grad-steps/sec (whole node) over a 16-alpha population,
cube-single-play shapes (BASELINE.json config 2).

One "step" = one population update: every member samples its own minibatch on
device from the HBM-resident offline buffer and runs a full FQL ``update()``
(critic TD loss, BC flow-matching loss, 10-step Euler flow, one-step
distillation + Q loss, backward, Adam, target EMA).  ``value`` = member
grad-steps per second over all ranks.

Scaling (BASELINE north_star: "16-member alpha population at 1 GPU with >= 7x scaling at
8 GPUs"): by default the 16-member population is sharded over the N ranks (strong scaling,
16 / N members per GPU, ``--population``); ``--members M`` instead puts M members on every
GPU (weak scaling, M * N members in all).

  python bench.py [--gpus N --steps K --warmup W] [--population P | --members M]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py is its own
launcher: the parent (which makes no GPU call) starts N rank processes with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rank r on cuda:r over RCCL, and
exits with the first failing rank's status.  --share-device puts every rank on
cuda:0 over gloo (a rehearsal of the N-rank path on a one-GPU box).  A world size
that differs from --gpus is an error.

Rank 0 prints ONE JSON line.  Data is synthetic (no network): 1M transitions,
obs ~ N(0,1), act ~ U(-1+1e-5, 1-1e-5), next_obs = obs + 0.05 N(0,1),
reward in {-1, 0} with P(0) = 0.05, mask = 1 - (reward == 0).
"""
from __future__ import annotations

import argparse
import json
import os
import random
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "flow-q-learning_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MI355X_FP32_MFMA_PEAK_TFLOPS = 157.3  # /opt/skills/guides/MI355X_MICROARCH.md (f32 matrix = vector peak)

WORKLOADS = {
    "cube": dict(env="cube-single-play-singletask-task2-v0", obs_dim=28, action_dim=5, batch_size=256),
    "antsoccer": dict(env="antsoccer-arena-navigate-singletask-task4-v0", obs_dim=42, action_dim=8,
                      batch_size=1024),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synthetic_dataset(n_rows: int, obs_dim: int, action_dim: int, seed: int = 0) -> dict:
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((n_rows, obs_dim), dtype=np.float32)
    act = rng.uniform(-1 + 1e-5, 1 - 1e-5, (n_rows, action_dim)).astype(np.float32)
    nxt = obs + np.float32(0.05) * rng.standard_normal((n_rows, obs_dim), dtype=np.float32)
    rew = np.where(rng.uniform(size=n_rows) < 0.05, 0.0, -1.0).astype(np.float32)
    mask = (1.0 - (rew == 0.0)).astype(np.float32)
    return {"observations": obs, "actions": act, "rewards": rew, "masks": mask, "next_observations": nxt}


def population_values(n_total: int, seed: int = 0):
    """alpha = logspace(log10 3, log10 1000, n) and seeds = random.sample(range(10000), n)
    after random.seed(seed), as reference tune_alpha.py:40-46."""
    random.seed(seed)
    alphas = np.logspace(np.log10(3), np.log10(1000), num=n_total).tolist()
    seeds = random.sample(range(10000), n_total)
    return alphas, seeds


def host_cpu() -> dict:
    """Host core counts and CPU model (cpu_baseline labels)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = None
    return {"os_cpu_count": os.cpu_count(), "affinity_cpus": allowed, "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def _pci_sysfs(device_index: int):
    """sysfs directory of the PCI function behind cuda:<device_index> (None if unknown).
    torch.cuda.get_device_properties only reads the already-initialised device table."""
    try:
        pr = torch.cuda.get_device_properties(device_index)
        addr = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
    except Exception:
        return None
    d = os.path.join("/sys/bus/pci/devices", addr)
    return d if os.path.isdir(d) else None


def gpu_clock_power(device_index: int) -> dict:
    """Current shader, memory and fabric clocks (MHz), power (W) and power cap (W) of the GPU from sysfs /
    hwmon.  One read takes 0.3-0.9 ms on the MI355X boxes (read_ms; the SMU answers
    pp_dpm_*): the end read happens while the last steps are still queued, so the GPU does not
    idle for it.  Values the box does not expose are null."""
    t_rd = time.perf_counter()
    out = {"sclk_mhz": None, "mclk_mhz": None, "fclk_mhz": None, "power_w": None, "power_cap_w": None}
    d = _pci_sysfs(device_index)
    if d is None:
        out["error"] = "no sysfs PCI node for the device"
        return out

    def rd(path):
        try:
            with open(path) as f:
                return f.read()
        except OSError:
            return None

    for key, name in (("sclk_mhz", "pp_dpm_sclk"), ("mclk_mhz", "pp_dpm_mclk"), ("fclk_mhz", "pp_dpm_fclk")):
        txt = rd(os.path.join(d, name))  # the DPM level marked "*" is the current one
        for line in (txt or "").splitlines():
            if line.strip().endswith("*"):
                try:
                    out[key] = int(line.split(":")[1].strip().rstrip("*").strip().lower().rstrip("mhz"))
                except (IndexError, ValueError):
                    pass
    hw_root = os.path.join(d, "hwmon")
    for hw in sorted(os.listdir(hw_root)) if os.path.isdir(hw_root) else []:
        base = os.path.join(hw_root, hw)
        f = rd(os.path.join(base, "freq1_input"))
        if out["sclk_mhz"] is None and f and f.strip().isdigit():
            out["sclk_mhz"] = int(f) // 1_000_000
        for key, name in (("power_w", "power1_average"), ("power_w", "power1_input"), ("power_cap_w", "power1_cap")):
            v = rd(os.path.join(base, name))
            if out[key] is None and v and v.strip().isdigit():
                out[key] = round(int(v) / 1e6, 1)
    out["read_ms"] = round(1e3 * (time.perf_counter() - t_rd), 3)
    return out


CPU_LEG_CAP_S = 20.0  # the whole CPU leg, warm-up updates included (the driver's run must finish)


def _cgroup_cpu_quota():
    """CPUs granted by the cgroup CPU quota (cgroup v2 cpu.max, else v1 cfs_quota / period),
    rounded up; None when no quota is set or the files are unreadable."""
    def rd(p):
        try:
            with open(p) as f:
                return f.read().split()
        except OSError:
            return None

    v2 = rd("/sys/fs/cgroup/cpu.max")
    if v2 and len(v2) >= 2 and v2[0] != "max":
        try:
            return max(1, -(-int(v2[0]) // int(v2[1])))
        except ValueError:
            return None
    q, p = rd("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), rd("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
    if q and p:
        try:
            qi, pi = int(q[0]), int(p[0])
        except ValueError:
            return None
        if qi > 0 and pi > 0:
            return max(1, -(-qi // pi))
    return None


def cpu_allotment() -> dict:
    """The CPUs this process may actually keep busy: the smaller of sched_getaffinity and the
    cgroup CPU quota (the box's affinity mask and os.cpu_count() show the whole 256-CPU host;
    its cgroup quota is the job's share).  OMP_NUM_THREADS is recorded but does not cap the
    count: a launcher that exports OMP_NUM_THREADS=1 must not turn the CPU leg single-threaded
     while the host grants more CPUs."""
    host = host_cpu()
    quota = _cgroup_cpu_quota()
    cands = [c for c in (host["affinity_cpus"], quota) if c]
    host["cgroup_quota_cpus"] = quota
    host["effective_cpus"] = max(1, min(cands) if cands else (os.cpu_count() or 1))
    return host


def cpu_baseline(wl: dict, data: dict, budget_s: float, thread_counts=None) -> dict:
    """The oracle's float32 PyTorch-CPU restatement (kind "port") of one member's
    update on the same synthetic data, timed on this host's cores at the effective CPU
    allotment (cpu_allotment) and at 1 thread.  Hard wall budget: min(budget_s,
    CPU_LEG_CAP_S) for the whole leg, split over the thread counts; each count's warm-up
    update counts against its share, the timing loop stops at the share's deadline (so a
    count overruns it by at most one update), and a count whose warm-up update alone
    exceeds its share is abandoned and recorded as such.  The best completed count is the
    value.  ``thread_counts`` overrides the counts (tests)."""
    host = cpu_allotment()
    eff = host["effective_cpus"]
    counts = list(thread_counts) if thread_counts else ([eff, 1] if eff > 1 else [1])
    total = min(float(budget_s), CPU_LEG_CAP_S)
    share = total / len(counts)
    prev_threads = torch.get_num_threads()
    runs, abandoned = {}, {}
    longest = 0.0
    t_leg = time.perf_counter()
    try:
        for threads in counts:
            r = _cpu_rate(wl, data, share, threads)
            longest = max(longest, r["longest_update_s"])
            if r["steps"] > 0:
                runs[threads] = r
            else:
                abandoned[str(threads)] = r["note"]
    finally:
        torch.set_num_threads(prev_threads)
    leg_s = time.perf_counter() - t_leg
    B = wl["batch_size"]
    if not runs:
        return {"value": None, "unit": "member-grad-steps/s", "cores": None, "kind": "port", "host": host,
                "rates_by_threads": {}, "abandoned": abandoned, "leg_s": round(leg_s, 2),
                "longest_update_s": round(longest, 3), "budget_s": round(total, 2),
                "sample": f"no thread count finished an update within its {share:.1f} s share"}
    best = max(runs, key=lambda t: runs[t]["rate"])
    r = runs[best]
    return {"value": r["rate"], "unit": "member-grad-steps/s", "cores": best, "kind": "port", "host": host,
            "rates_by_threads": {str(t): round(x["rate"], 3) for t, x in runs.items()},
            "abandoned": abandoned, "leg_s": round(leg_s, 2), "budget_s": round(total, 2),
            "longest_update_s": round(longest, 3),
            "sample": f"{r['steps']} sequential update() steps of 1 member (alpha=10, B={B}, H=512) in "
                      f"{r['elapsed']:.1f} s after a {r['warmup_s']:.2f} s warm-up update, float32 PyTorch-CPU "
                      f"restatement (oracle/fql_torch.py), torch threads={best}: the best of "
                      f"{', '.join(str(t) for t in counts)} thread(s), {share:.1f} s wall budget each "
                      f"(effective CPUs {eff} = min of sched_getaffinity {host['affinity_cpus']} and cgroup quota "
                      f"{host['cgroup_quota_cpus']}; OMP_NUM_THREADS {host['omp_num_threads']} recorded, not a cap; "
                      f"os.cpu_count() {host['os_cpu_count']}). BASELINE C1 (1k steps) is timed, not extrapolated, "
                      f"by bench.py --c1 (profiles/round6*/c1_cpu_1k_steps.json)"}


def _cpu_rate(wl: dict, data: dict, budget_s: float, threads: int) -> dict:
    """Updates of one member at ``threads`` torch threads until ``budget_s`` of wall time
    (warm-up included) is spent.  steps == 0 means the warm-up update alone used the budget."""
    from oracle import fql_oracle as O
    from oracle.fql_torch import TorchFQL

    t_start = time.perf_counter()
    deadline = t_start + budget_s
    torch.set_num_threads(threads)
    cfg = O.OracleConfig(obs_dim=wl["obs_dim"], action_dim=wl["action_dim"], batch_size=wl["batch_size"],
                         alpha=10.0)
    agent = TorchFQL(cfg, O.cast_tree(O.init_params(cfg, 0), np.float32))
    rng = np.random.default_rng(1)
    B, A, N = cfg.batch_size, cfg.action_dim, data["observations"].shape[0]

    def draw():
        idx = rng.integers(0, N, B)
        b = {k: torch.from_numpy(np.ascontiguousarray(v[idx])) for k, v in data.items()}
        nz = {"z_next": torch.randn(B, A), "x0": torch.randn(B, A), "t": torch.rand(B, 1),
              "z_d": torch.randn(B, A), "z_metric": torch.randn(B, A)}
        return b, nz

    t_w = time.perf_counter()
    agent.update(*draw())  # warm-up
    warm = time.perf_counter() - t_w
    t0 = time.perf_counter()
    if t0 >= deadline:
        return {"rate": 0.0, "steps": 0, "elapsed": 0.0, "warmup_s": warm, "longest_update_s": warm,
                "note": f"abandoned: setup + warm-up update took {t0 - t_start:.2f} s > {budget_s:.2f} s share"}
    steps, el, longest = 0, 0.0, warm
    while True:
        t_u = time.perf_counter()
        agent.update(*draw())
        steps += 1
        now = time.perf_counter()
        longest = max(longest, now - t_u)
        el = now - t0
        if now >= deadline:
            break
    return {"rate": steps / el, "steps": steps, "elapsed": el, "warmup_s": warm, "longest_update_s": longest,
            "note": None}


def c1_cpu_run(steps: int, rows: int) -> dict:
    """BASELINE config 1 timed, not extrapolated: cube-single shapes, one
    member at alpha = 10, B = 256, H = 512 x 4, `steps` sequential update() calls on the host
    CPU only (no GPU call).  The reference runs this on CPU JAX, which is absent here; the
    float32 PyTorch restatement of the same update (oracle/fql_torch.py, kind "port") runs at
    the effective CPU allotment (cpu_allotment).  Minibatches are drawn from the synthetic
    1M-row buffer on the host, as the reference's task.sample does, inside the timed loop."""
    from oracle import fql_oracle as O
    from oracle.fql_torch import TorchFQL
    wl = WORKLOADS["cube"]
    host = cpu_allotment()
    threads = host["effective_cpus"]
    torch.set_num_threads(threads)
    data = synthetic_dataset(rows, wl["obs_dim"], wl["action_dim"])
    cfg = O.OracleConfig(obs_dim=wl["obs_dim"], action_dim=wl["action_dim"], batch_size=wl["batch_size"],
                         alpha=10.0)
    agent = TorchFQL(cfg, O.cast_tree(O.init_params(cfg, 0), np.float32))
    rng = np.random.default_rng(1)
    B, A, N = cfg.batch_size, cfg.action_dim, data["observations"].shape[0]

    def draw():
        idx = rng.integers(0, N, B)
        b = {k: torch.from_numpy(np.ascontiguousarray(v[idx])) for k, v in data.items()}
        nz = {"z_next": torch.randn(B, A), "x0": torch.randn(B, A), "t": torch.rand(B, 1),
              "z_d": torch.randn(B, A), "z_metric": torch.randn(B, A)}
        return b, nz

    t_w = time.perf_counter()
    agent.update(*draw())  # first call: allocator and thread-pool warm-up, not timed
    warm = time.perf_counter() - t_w
    t0 = time.perf_counter()
    last = None
    for _ in range(steps):
        last = agent.update(*draw())
    wall = time.perf_counter() - t0
    info = {k: float(v) for k, v in (last or {}).items()} if isinstance(last, dict) else {}
    return {"metric": f"BASELINE C1: wall time of {steps} FQL update() steps on the host CPU (no GPU)",
            "value": round(wall, 3), "unit": "s", "steps": steps, "higher_is_better": False,
            "member_grad_steps_per_s": round(steps / wall, 3), "threads": threads, "warmup_update_s": round(warm, 3),
            "kind": "port", "host": host, "dtype": "f32",
            "config": {"workload": f"{wl['env']} single alpha=10 update(), B={B}, H=512x4, obs {wl['obs_dim']}, "
                                   f"act {wl['action_dim']}, flow_steps 10", "rows": rows},
            "data": "synthetic (seeded numpy), host-sampled minibatches inside the timed loop",
            "finite": bool(all(np.isfinite(v) for v in info.values())) if info else None}


def eval_rollout_leg(pop, wl: dict, n_envs: int, steps: int, dev) -> dict:
    """World-model evaluation of every member (BASELINE config 5's eval; SURVEY.md
    8f rank 1): one fqlpop_rollout launch, 512-wide actor + BaselineStatePredictor
    (128, 256, 128) + TerminationPredictor (128, 256, 128), synthetic env model
    whose termination logit stays negative so every episode runs `steps` steps.
    Outside the timed region; reported beside the headline, not in `value`."""
    import envmodel as em
    D, A = wl["obs_dim"], wl["action_dim"]
    spec = em.EnvModelSpec(D, A)
    sp = em.init_state_predictor(spec, 0, scale=0.1)
    tp = em.init_termination_predictor(spec, 1, scale=0.0, bias=-1.0)
    pop.set_env_model(em.flatten_state_predictor(spec, sp), em.flatten_termination_predictor(spec, tp),
                      spec.sp_hidden, spec.tp_hidden)
    obs0 = np.random.default_rng(0).standard_normal((n_envs, D)).astype(np.float32)
    pop.rollout(obs0, 2, seed=1)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    succ, length = pop.rollout(obs0, steps, seed=2)
    el = time.perf_counter() - t0
    H = 512
    f_actor = 2.0 * ((D + A) * H + 3 * H * H + H * A)
    sd, td = spec.sp_dims(), spec.tp_dims()
    f_env = 2.0 * sum(sd[i] * sd[i + 1] for i in range(len(sd) - 1)) + 2.0 * sum(
        td[i] * td[i + 1] for i in range(len(td) - 1))
    env_steps = float(length.sum())
    return {"members": int(succ.shape[0]), "envs_per_member": n_envs, "max_episode_steps": steps,
            "ms": round(1000.0 * el, 3), "env_steps_per_s": round(env_steps / el, 1),
            "tflops": round(env_steps * (f_actor + f_env) / el / 1e12, 3),
            "episodes_all_full_length": bool(np.all(length == steps)),
            "note": "one launch, 16 envs per block, all steps on device (sample_actions + state predictor + "
                    "termination predictor); host-synchronised wall time incl. H2D of init obs"}


def envmodel_train_leg(wl: dict, data: dict, steps: int) -> dict:
    """Env-model training throughput (outside `value`): the
    baseline state predictor (128, 256, 128) and the termination predictor, B = 256,
    device-sampled from the same synthetic buffer, `steps` train_steps each."""
    import envmodel as em
    from envmodel.trainer import EnvModelTrainerConfig, StatePredictorTrainer, TerminationPredictorTrainer

    class _Loader:
        def __init__(self, ds):
            self.dataset = ds

    spec = em.EnvModelSpec(wl["obs_dim"], wl["action_dim"])
    ds = {k: data[k] for k in ("observations", "actions", "rewards", "next_observations")}
    out = {}
    ms_steps = max(10, steps // 20)
    for name, cls, params, cfg, n in (
            ("state_predictor", StatePredictorTrainer, em.init_state_predictor(spec, 0),
             EnvModelTrainerConfig(steps=steps, termination_weight=0.0), steps),
            ("termination_predictor", TerminationPredictorTrainer, em.init_termination_predictor(spec, 1),
             EnvModelTrainerConfig(steps=steps), steps),
            ("multistep_T256", StatePredictorTrainer, em.init_state_predictor(spec, 0),
             EnvModelTrainerConfig(steps=ms_steps, model="multistep", sequence_length=256,
                                   termination_weight=0.0), ms_steps)):
        n_ep = len(ds["observations"]) // 1000 * 1000  # multistep: whole 1000-row episodes
        tr = cls(spec, params, _Loader({k: v[:n_ep] for k, v in ds.items()} if cfg.model == "multistep" else ds),
                 None, cfg)
        tr.steps(min(20, n))
        tr.sync()
        t0 = time.perf_counter()
        tr.steps(n)
        tr.sync()
        el = time.perf_counter() - t0
        out[name] = {"train_steps_per_s": round(n / el, 1), "us_per_step": round(1e6 * el / n, 2),
                     "final_train_loss": round(tr.read_logs()["loss"], 6)}
        tr.close()
    out["note"] = ("B=256, hidden (128, 256, 128), Adam + cosine decay; two launches per train_step "
                   "(fused fwd/loss/bwd over 16-row blocks, partial-sum Adam); multistep: 256-step "
                   "windows of 1000-row episodes, termination_weight 0: backpropagation through time as "
                   "a forward and a backward sweep in one 1024-thread launch per 16 sequences, dW as a "
                   "GEMM over the stored records, then Adam (engine option em_seq_sweep; "
                   "profiles/round6b/em_multistep_ab_grouped.txt has termination_weight 1 too)")
    return out


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, argv: list) -> int:
    """Launcher for ``--gpus N`` without torch.distributed.run: N fresh rank processes
    (this parent makes no GPU call), rank r -> LOCAL_RANK r.  Rank 0 prints the JSON
    line.  If a rank fails, the others are terminated and its status is returned."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"bench.py: rank process {p.pid} exited with {code}; stopping the others")
                for q in procs:
                    q.terminate()
        time.sleep(0.1)
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--population", type=int, default=None,
                    help="members of the whole population, sharded round-robin over the ranks (strong "
                         "scaling; default 16, the north-star population)")
    ap.add_argument("--members", type=int, default=None,
                    help="members per GPU instead (weak scaling: members x N in all)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cube")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=100)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_dominant.json"),
                    help="HBM bytes per dominant-kernel launch measured by rocprofv3 --pmc passes "
                         "(csrc/tools/pmc_summary.py output); missing file -> traffic null")
    ap.add_argument("--kernel-times-json", default=os.path.join(ROOT, "profiles", "kernel_times.json"),
                    help="per-kernel in-step and serial launch times of the 16-member step (rocprofv3 stats, "
                         "csrc/tools/kernel_times.py output): the roofline's serial fraction and the in-step "
                         "top kernel; missing file -> those fields null")
    ap.add_argument("--preheat-ms", type=float, default=300.0,
                    help="replays of the dominant kernel alone before the warmup steps (GPU clock ramp); 0 = off")
    ap.add_argument("--preheat-kind", choices=("steps", "kernel"), default="steps",
                    help="steps: population steps of a second, throwaway population on the same device "
                         "(the timed population is untouched); kernel: replays of the dominant kernel alone")
    ap.add_argument("--no-probe", action="store_true",
                    help="time the step without the in-step timing nodes of the dominant kernel")
    ap.add_argument("--eval-envs", type=int, default=50, help="world-model rollout leg: envs per member "
                    "(reference eval_episodes); 0 disables the leg")
    ap.add_argument("--eval-steps", type=int, default=1000, help="world-model rollout leg: max_episode_steps")
    ap.add_argument("--envmodel-train-steps", type=int, default=2000,
                    help="env-model training leg: train_steps per model (0 disables the leg)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on cuda:0 over gloo (rehearse the N-rank path on one GPU)")
    ap.add_argument("--serial", action="store_true",
                    help="profiling: every launch of the step on one stream (engine option serial)")
    ap.add_argument("--engine-option", action="append", default=[], metavar="NAME=VALUE",
                    help="fqlpop_set_engine_option before the population is created (alternate schedules / "
                         "code paths with the same results; recorded in the JSON line)")
    ap.add_argument("--c1", action="store_true",
                    help="BASELINE config 1 only: --steps (default 1000 here) update() steps of one member on the "
                         "host CPU (no GPU call); prints its own JSON line")
    ap.add_argument("--diagnostic", action="store_true",
                    help="allow FQLPOP_* environment variables (developer A/B runs); they are recorded")
    args = ap.parse_args(argv)
    if args.population is not None and args.members is not None:
        ap.error("--population and --members are exclusive")

    fq_env = {k: v for k, v in os.environ.items() if k.startswith("FQLPOP_")}
    if fq_env and not args.diagnostic:
        log(f"bench.py: refusing to measure with {sorted(fq_env)} set (developer switches); "
            "unset them or pass --diagnostic")
        return 2
    if args.c1:
        steps = args.steps if "--steps" in (sys.argv[1:] if argv is None else list(argv)) else 1000
        print(json.dumps(c1_cpu_run(steps, args.rows)), flush=True)
        return 0
    if args.gpus < 1:
        log("bench.py: --gpus must be >= 1")
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: world size {world} (WORLD_SIZE) != --gpus {args.gpus}")
        return 2
    distributed = world > 1
    if not args.share_device and torch.cuda.device_count() < world:  # device_count: no GPU init
        log(f"bench.py: {world} ranks but {torch.cuda.device_count()} visible GPU(s); --share-device "
            "rehearses the N-rank path on one GPU")
        return 2
    dev_index = 0 if args.share_device else local_rank
    torch.cuda.set_device(dev_index)
    if distributed:
        if args.share_device:
            # gloo's rendezvous prints "[Gloo] Rank r is connected to ..." on stdout, which
            # carries only the JSON line: point fd 1 at stderr while it connects
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo")
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))

    from fqlpop import Population, PopulationConfig, set_engine_option
    engine_opts = {}
    for kv in args.engine_option:
        k, v = kv.split("=", 1)
        engine_opts[k] = int(v)
    if args.serial:
        engine_opts["serial"] = 1
    for k, v in engine_opts.items():
        set_engine_option(k, v)

    wl = WORKLOADS[args.workload]
    # dataset: generated on rank 0, broadcast over RCCL (xGMI) to every rank
    from fqlpop import distributed as D
    data = synthetic_dataset(args.rows, wl["obs_dim"], wl["action_dim"]) if rank == 0 else None
    dev = torch.device("cuda", dev_index)
    shapes = {"observations": (args.rows, wl["obs_dim"]), "actions": (args.rows, wl["action_dim"]),
              "rewards": (args.rows,), "masks": (args.rows,), "next_observations": (args.rows, wl["obs_dim"])}
    dev_data = D.broadcast_dataset(data, shapes, dev)
    torch.cuda.synchronize()

    weak = args.members is not None
    n_total = args.members * world if weak else (args.population or 16)
    if n_total < world:
        log(f"bench.py: a {n_total}-member population cannot give every one of {world} ranks a member")
        return 2
    alphas_all, seeds_all = population_values(n_total)
    alphas, seeds = D.shard(alphas_all, rank, world), D.shard(seeds_all, rank, world)
    pcfg = PopulationConfig(obs_dim=wl["obs_dim"], action_dim=wl["action_dim"], batch_size=wl["batch_size"],
                            use_graph=not args.no_graph)
    pop = Population(pcfg, alphas, seeds, device=dev_index)
    pop.set_dataset(dev_data)
    scratch = None
    if args.preheat_ms > 0 and args.preheat_kind == "steps":
        # a second population of the same shape (own parameters, optimiser state and dataset
        # copy): its steps warm the GPU; the timed population's state is never touched by them
        scratch = Population(pcfg, alphas, seeds, device=dev_index)
        scratch.set_dataset(dev_data)
    del dev_data
    torch.cuda.empty_cache()

    # every launch of the dominant kernel inside the timed steps stamps its
    # blocks' start/end (s_memrealtime); read_probe() reduces them per launch.  The
    # probe is on during the warmup too: its launches are separate hipGraphs (one per
    # stamp-slot set and parameter buffer), so they are captured and instantiated in
    # the warmup, not inside the timed region; set_probe() again resets the totals.
    # GPU clocks: after the idle setup (dataset generation on the host, uploads) the
    # chip needs ~50-100 ms of load to reach its steady clock; the first 20 steps
    # after 5 warmup steps ran 4-8 % slower than steady state (tools/step_ramp.py).
    # Replays of the dominant kernel alone (not steps; results discarded) bring it
    # there before the warmup steps, so a short --steps/--warmup run measures the
    # steady-state step, not the clock ramp.
    # The kernel replays still left a ramp that only the step's own mix of MFMA, L2 and HBM
    # work warms: the default preheat therefore steps a throwaway population
    # (same shapes and schedule) instead, and the W warmup steps of the timed population follow.
    preheat_ms, preheat_steps = 0.0, 0
    if args.preheat_ms > 0:
        t_ph = time.perf_counter()
        if scratch is not None:
            while 1e3 * (time.perf_counter() - t_ph) < args.preheat_ms:
                scratch.step(10)
                scratch.sync()
                preheat_steps += 10
        else:
            iso_us0, _ = pop.time_dominant_kernel(1)
            pop.time_dominant_kernel(max(1, int(args.preheat_ms * 1e3 / max(iso_us0, 1.0))))
        torch.cuda.synchronize()
        preheat_ms = 1e3 * (time.perf_counter() - t_ph)
    pop.set_probe(not args.no_probe)
    log(f"[rank {rank}] warmup {args.warmup} steps, {pop.n} members")
    pop.step(args.warmup)
    pop.sync()
    pop.set_probe(not args.no_probe)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    clk0 = gpu_clock_power(dev_index)
    t0 = time.perf_counter()
    chunk = max(1, min(100, args.steps))
    done = 0
    while done < args.steps:
        k = min(chunk, args.steps - done)
        pop.step(k)
        done += k
    clk1 = gpu_clock_power(dev_index)  # the last chunk is still running: the loaded clock
    pop.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if distributed:
        dist.barrier()
    el = D.max_over_ranks(el, None if args.share_device else dev)
    probe_us, probe_n, _ = pop.read_probe()
    pop.set_probe(False)
    info = pop.read_info_array()
    finite = bool(np.all(np.isfinite(info[:, :13])))

    member_steps = n_total * args.steps
    value = member_steps / el
    flops_ms = pop.flops_per_member_step

    # dominant kernel of the step (all members, one launch): the persistent
    # Euler flow (H = 512) or else the Euler hidden-layer GEMM
    kname, kflops, kbytes = pop.dominant_kernel_info()
    iso_us, _ = pop.time_dominant_kernel(args.kernel_iters)  # the same launch replayed alone
    _, _, (cc_event_us, cc_stamp_us) = pop.read_probe()     # stamp clock vs HIP events, one launch
    launch_us = probe_us if probe_n else iso_us
    achieved = kflops / (launch_us * 1e-6) / 1e12
    traffic, traffic_src = None, None
    if os.path.exists(args.pmc_json):
        with open(args.pmc_json) as f:
            pmc = json.load(f)
        # the counters were collected on one workload's launch (pmc_dominant.json "workload")
        if (pmc.get("kernel_regex") and pmc["kernel_regex"] in kname and pmc.get("members") == pop.n
                and pmc.get("workload", "cube") == args.workload):
            traffic = pmc["traffic_bytes_per_launch"]
            traffic_src = {"file": os.path.relpath(args.pmc_json, ROOT), "commit": pmc.get("commit"),
                           "date": pmc.get("date")}

    # the roofline's other views of the same kernel: alone (live replays
    # above), serial-stream launch and in-step top kernel by time (rocprofv3, kernel_times.json)
    serial_view, top_view = None, None
    if os.path.exists(args.kernel_times_json):
        with open(args.kernel_times_json) as f:
            kt = json.load(f)
        if kt.get("members") == pop.n and kt.get("workload", "cube") == args.workload:
            src = {"file": os.path.relpath(args.kernel_times_json, ROOT), "commit": kt.get("commit"),
                   "instep_source": kt.get("instep_source"), "serial_source": kt.get("serial_source")}
            kd = kt["kernels"].get(kname.split("(")[0])
            if kd and kd.get("serial_avg_us"):
                serial_view = {"serial_launch_us": kd["serial_avg_us"],
                               "frac": round(kflops / (kd["serial_avg_us"] * 1e-6) / 1e12 / MI355X_FP32_MFMA_PEAK_TFLOPS, 4),
                               "rocprof_in_step_launch_us": kd["in_step_avg_us"], "source": src}
            top_name = next(iter(kt["kernels"]))
            td = kt["kernels"][top_name]
            top_view = {"kernel": top_name, "launches_per_step": td["launches_per_step"],
                        "in_step_us_per_step": td["in_step_us_per_step"],
                        "serial_us_per_step": td.get("serial_us_per_step"), "stretch": td.get("stretch"),
                        "source": src}
    step_frac = flops_ms * value / 1e12 / (MI355X_FP32_MFMA_PEAK_TFLOPS * world)

    result = {
        # BASELINE.json's metric: the whole population (16 members by default) over all ranks
        "metric": f"FQL grad-steps/sec (whole node) over {n_total}-α population, "
                  + ("cube-single-v0" if args.workload == "cube" else "antsoccer"),
        "value": round(value, 2),
        "unit": "member-grad-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * el / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic ({args.rows / 1e6:g}M transitions of {args.workload} shape (obs {wl['obs_dim']}, act "
                f"{wl['action_dim']}), seeded numpy; random-init weights)",
        "config": {
            "workload": f"{wl['env']} {n_total}-alpha population update(), B={wl['batch_size']}, H=512x4, "
                        f"obs {wl['obs_dim']}, act {wl['action_dim']}, flow_steps 10",
            "population": n_total,
            "members_per_gpu": (args.members if weak else
                                (n_total // world if n_total % world == 0 else f"{n_total // world}-{-(-n_total // world)}")),
            "members_this_rank": pop.n,
            "global_batch": wl["batch_size"] * n_total,
            "population_steps_per_s": round(args.steps / el, 3),
            "gflop_per_member_step": round(flops_ms / 1e9, 4),
            "step_tflops": round(flops_ms * value / 1e12, 3),
            "step_mfma_frac": round(flops_ms * value / 1e12 / (MI355X_FP32_MFMA_PEAK_TFLOPS * world), 4),
            "parallelism": (f"weak: {args.members} members per GPU x {world} GPU(s)" if weak else
                            f"strong: a {n_total}-member population sharded round-robin over {world} GPU(s)")
                           + ", no data-path collective",
            "graph": not args.no_graph,
            "info_finite": finite,
            "share_device": bool(args.share_device),
            "serial_streams": bool(args.serial),
            "engine_options": engine_opts,
        },
        "gpu_clock": {"device": torch.cuda.get_device_name(dev_index), "start": clk0, "end": clk1,
                      "note": "sysfs pp_dpm_sclk / hwmon of this rank's GPU, read just before the clock "
                              "starts and before the final synchronize (GPU still busy)"},
        "roofline": {
            "bound": "mfma",
            "kernel": kname + (" (Euler flow steps 1..9 of all members: 16-column blocks, weights streamed, "
                               "activations LDS-resident)" if kname == "euler_flow_kernel" else
                               " (Euler-flow hidden layer y' = gelu(W^T x' + b), one launch per layer)"),
            "achieved": round(achieved, 3),
            "peak": MI355X_FP32_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / MI355X_FP32_MFMA_PEAK_TFLOPS, 4),
            "frac_in_step": round(achieved / MI355X_FP32_MFMA_PEAK_TFLOPS, 4),
            "frac_isolated": round(kflops / (iso_us * 1e-6) / 1e12 / MI355X_FP32_MFMA_PEAK_TFLOPS, 4),
            "frac_serial_stream": serial_view,
            "step_frac": round(step_frac, 4),
            "in_step_top_kernel": top_view,
            "fractions": "frac = frac_in_step: the dominant kernel's in-step launches (this run's stamps), "
                         "sharing the CUs with the other streams; frac_isolated: the same launch replayed alone "
                         "(this run); frac_serial_stream: its launch in a serial-stream step (rocprofv3, "
                         "kernel_times.json); step_frac: the whole step's flops / wall time / peak",
            "avg_launch_us": round(launch_us, 3),
            "launches_timed": probe_n,
            "isolated_launch_us": round(iso_us, 3),
            "timing": "in-step launches timed by per-block s_memrealtime stamps (100 MHz); cross-check on one "
                      f"isolated launch: HIP events {cc_event_us:.2f} us vs stamps {cc_stamp_us:.2f} us",
            "flops_per_launch": kflops,
            "algorithmic_bytes_per_launch": kbytes,
            "traffic": traffic,
            "traffic_source": traffic_src,
        },
        "cpu_baseline": None,
        "preheat": {"ms": round(preheat_ms, 1), "kind": args.preheat_kind if args.preheat_ms > 0 else None,
                    "steps": preheat_steps,
                    "what": ("population steps of a second, throwaway population of the same shape (own "
                             "parameters, optimiser state and dataset copy; the timed population is not "
                             "stepped by it)" if args.preheat_kind == "steps" else
                             "replays of the dominant kernel alone (no steps, results discarded)")
                            + " before the warmup steps, so the timed steps run at the steady GPU clock"},
    }
    if scratch is not None:
        scratch.close()
    if args.eval_envs > 0:
        result["eval_rollout"] = eval_rollout_leg(pop, wl, args.eval_envs, args.eval_steps, dev)
    if args.envmodel_train_steps > 0 and rank == 0:
        result["envmodel_train"] = envmodel_train_leg(wl, data, args.envmodel_train_steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log(f"[rank 0] cpu baseline ({args.cpu_baseline_seconds:.0f} s budget)")
        result["cpu_baseline"] = cpu_baseline(wl, data, args.cpu_baseline_seconds)
    if fq_env:
        result["diagnostic_env"] = fq_env
    if rank == 0:
        print(json.dumps(result), flush=True)
    pop.close()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
