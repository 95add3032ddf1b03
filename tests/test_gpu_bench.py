"""bench.py's JSON line (the driver's contract) on a short run of the real engine."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2", "--rows", "20000",
           "--no-cpu-baseline", "--eval-envs", "2", "--eval-steps", "20", "--envmodel-train-steps", "5",
           "--kernel-iters", "2", "--preheat-ms", "20"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "preheat"):
        assert k in d, k
    assert d["steps"] == 4 and d["warmup"] == 2 and d["n_gpus"] == 1
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]  # the north-star metric, verbatim
    # the default workload: the 16-member population sharded over the ranks (strong scaling)
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "strong"
    assert d["config"]["population"] == 16 and d["config"]["members_this_rank"] == 16
    assert d["config"]["info_finite"] is True
    assert abs(d["value"] - 16 * 1000.0 / d["ms_per_step"]) <= 1e-3 * d["value"] + 1.0
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "avg_launch_us", "launches_timed"):
        assert k in rf, k
    assert rf["launches_timed"] == 4  # one probed dominant launch per timed step
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert d["preheat"]["ms"] > 0


def _bench(args, env=None, timeout=400):
    e = dict(os.environ)
    for k in [k for k in e if k.startswith("FQLPOP_")]:
        del e[k]
    e.update(env or {})
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=e)


def test_bench_self_launches_ranks_sharing_the_device():
    """bench.py --gpus 2 without torch.distributed.run starts its own two rank processes
    (the parent makes no GPU call); --share-device puts both on cuda:0 over gloo.  The
    JSON line counts both ranks' members and is printed once."""
    r = _bench(["--gpus", "2", "--share-device", "--steps", "4", "--warmup", "2", "--rows", "20000",
                "--no-cpu-baseline", "--eval-envs", "0", "--envmodel-train-steps", "0", "--kernel-iters", "2",
                "--preheat-ms", "20", "--members", "4"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]  # stdout: the JSON line only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["share_device"] is True and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 256 * 4 * 2
    assert abs(d["value"] - 8 * 1000.0 / d["ms_per_step"]) <= 1e-3 * d["value"] + 1.0
    assert d["config"]["info_finite"] is True
    assert "gpu_clock" in d and "start" in d["gpu_clock"]


def test_production_library_ignores_timing_switches():
    """FQLPOP_SKIP (leave launches out) and FQLPOP_DW_MODE (drop optimiser phases) only
    exist in diagnostic builds: with them set, the production library's update still
    matches the oracle."""
    code = ("import sys; sys.path[:0] = [%r, %r]; import __graft_entry__ as g; g.smoke()"
            % (ROOT, os.path.join(ROOT, "flow-q-learning_amd")))
    e = dict(os.environ, FQLPOP_SKIP="255", FQLPOP_DW_MODE="1", FQLPOP_PIPE_EXP="1", FQLPOP_PHASE_PROBE="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "smoke ok" in r.stdout


def test_bench_population_is_sharded_over_ranks():
    """--population P (the default, P = 16): the P members are dealt round-robin to the
    ranks (strong scaling), the metric names the whole population, value counts P members."""
    r = _bench(["--gpus", "2", "--share-device", "--population", "6", "--steps", "4", "--warmup", "2", "--rows",
                "20000", "--no-cpu-baseline", "--eval-envs", "0", "--envmodel-train-steps", "0", "--kernel-iters",
                "2", "--preheat-ms", "20"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert d["scaling"] == "strong" and d["config"]["population"] == 6
    assert d["config"]["members_this_rank"] == 3 and d["config"]["members_per_gpu"] == 3
    assert "over 6-" in d["metric"]
    assert abs(d["value"] - 6 * 1000.0 / d["ms_per_step"]) <= 1e-3 * d["value"] + 1.0


def test_two_hardware_queues_smoke_and_bench():
    """GPU_MAX_HW_QUEUES=2 (a legal HIP runtime setting; the box defaults to 4) from the
    start of a fresh process: smoke() and a 16-member bench run complete.  Round 3 saw a
    crash inside the HIP runtime during the first graph captures under this setting."""
    code = ("import sys; sys.path[:0] = [%r, %r]; import __graft_entry__ as g; g.smoke()"
            % (ROOT, os.path.join(ROOT, "flow-q-learning_amd")))
    e = dict(os.environ, GPU_MAX_HW_QUEUES="2")
    for k in [k for k in e if k.startswith("FQLPOP_")]:
        del e[k]
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "smoke ok" in r.stdout
    r = _bench(["--steps", "4", "--warmup", "2", "--rows", "20000", "--no-cpu-baseline", "--eval-envs", "0",
                "--envmodel-train-steps", "0", "--kernel-iters", "2", "--preheat-ms", "20"],
               env={"GPU_MAX_HW_QUEUES": "2"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert d["config"]["info_finite"] is True and d["value"] > 0
