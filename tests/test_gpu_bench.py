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
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["info_finite"] is True
    assert abs(d["value"] - 16 * 1000.0 / d["ms_per_step"]) <= 1e-3 * d["value"] + 1.0
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "avg_launch_us", "launches_timed"):
        assert k in rf, k
    assert rf["launches_timed"] == 4  # one probed dominant launch per timed step
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert d["preheat"]["ms"] > 0
