"""bench.py's refusals, which happen before any GPU call (CPU tests), and the
production library's switch hygiene."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env):
    e = {k: v for k, v in os.environ.items() if not k.startswith("FQLPOP_")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True,
                          text=True, timeout=120, cwd=ROOT, env=e)


def test_bench_refuses_developer_switches():
    r = _bench(["--steps", "1"], {"FQLPOP_SKIP": "1"})
    assert r.returncode == 2 and "FQLPOP_SKIP" in r.stderr


def test_bench_refuses_world_size_mismatch():
    r = _bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "!= --gpus" in r.stderr


def test_production_library_reads_no_environment():
    """The shipped libfqlpop.so is not a diagnostic build and imports no getenv: the
    timing-only switches (FQLPOP_SKIP, FQLPOP_DW_MODE, FQLPOP_PIPE_EXP, FQLPOP_PHASE_PROBE)
    cannot reach it.  Alternate code paths go through fqlpop_set_engine_option."""
    import fqlpop
    assert not fqlpop.is_diagnostic_build()
    out = subprocess.run(["nm", "-D", "--undefined-only", fqlpop.LIB_PATH], capture_output=True, text=True)
    assert out.returncode == 0
    assert "getenv" not in out.stdout
    with open(fqlpop.LIB_PATH, "rb") as f:
        blob = f.read()
    for name in (b"FQLPOP_SKIP", b"FQLPOP_DW_MODE", b"FQLPOP_PIPE_EXP", b"FQLPOP_PHASE_PROBE"):
        assert name not in blob, name


def test_engine_options_validate_and_reset():
    import pytest
    import fqlpop
    fqlpop.set_engine_option("serial", 1)
    assert fqlpop.get_engine_option("serial") == 1
    fqlpop.reset_engine_options()
    assert fqlpop.get_engine_option("serial") == 0
    with pytest.raises(fqlpop.FqlpopError):
        fqlpop.set_engine_option("no_such_option", 1)
    with pytest.raises(fqlpop.FqlpopError):
        fqlpop.set_engine_option("streams", 7)


def test_removed_schedule_experiments_are_unknown_options():
    """The schedule experiments that measured slower were removed in round
    4: their names are no longer engine options, so no capture topology but the measured one
    can be selected."""
    import pytest
    import fqlpop
    for name in ("xstep", "bc_late", "fuse_dq", "early_join", "dw_stagger", "prio", "streams", "cdw_sb"):
        with pytest.raises(fqlpop.FqlpopError):
            fqlpop.set_engine_option(name, 1)
    fqlpop.reset_engine_options()


def test_split_option_values():
    """Engine option split: 0 (off), 1 (auto, the default), or 2 / 4 / 8 blocks per tile."""
    import pytest
    import fqlpop
    fqlpop.reset_engine_options()
    assert fqlpop.get_engine_option("split") == 1
    for v in (0, 2, 4, 8):
        fqlpop.set_engine_option("split", v)
        assert fqlpop.get_engine_option("split") == v
    for v in (3, 5, 6, 7, 9, -1):
        with pytest.raises(fqlpop.FqlpopError):
            fqlpop.set_engine_option("split", v)
    fqlpop.reset_engine_options()


def test_hw_queues_option_and_env_parse(monkeypatch):
    """hw_queues (the caller's GPU_MAX_HW_QUEUES): a validated engine option, and the value
    the Python layer reads from the environment (below 4 the step is captured on one stream)."""
    import pytest
    import fqlpop
    from fqlpop import _lib
    assert fqlpop.get_engine_option("hw_queues") == 4
    fqlpop.set_engine_option("hw_queues", 2)
    assert fqlpop.get_engine_option("hw_queues") == 2
    fqlpop.reset_engine_options()
    assert fqlpop.get_engine_option("hw_queues") == 4
    with pytest.raises(fqlpop.FqlpopError):
        fqlpop.set_engine_option("hw_queues", 0)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    assert _lib.hw_queues_from_env() == 2
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "junk")
    assert _lib.hw_queues_from_env() is None
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    assert _lib.hw_queues_from_env() is None


def test_population_passes_hw_queues_for_its_create_only(monkeypatch):
    """Population hands GPU_MAX_HW_QUEUES to the engine for its own fqlpop_create and then
    restores the process-wide option: a caller running the HIP runtime with 2
    queues gets the one-stream capture, and later populations do not inherit the value."""
    import fqlpop
    from fqlpop import Population, PopulationConfig, _lib
    lib = _lib.load_library()
    seen = []
    real = lib.fqlpop_create

    def fake_create(*a):
        seen.append(fqlpop.get_engine_option("hw_queues"))
        lib.fqlpop_last_error()  # (keeps the error text path alive)
        return -1

    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    monkeypatch.setattr(lib, "fqlpop_create", fake_create)
    try:
        fqlpop.set_engine_option("hw_queues", 8)
        try:
            Population(PopulationConfig(), [3.0], [1]).close()
        except fqlpop.FqlpopError:
            pass
        assert seen == [2]
        assert fqlpop.get_engine_option("hw_queues") == 8
    finally:
        monkeypatch.setattr(lib, "fqlpop_create", real)
        fqlpop.reset_engine_options()


def test_step_streams_never_exceed_hw_queues():
    """The hardware-queue invariant: the step is captured on 4 streams
    only with >= 4 hardware queues, else on one; serial is always one stream."""
    import fqlpop
    try:
        for q in range(1, 17):
            fqlpop.set_engine_option("hw_queues", q)
            for serial in (0, 1):
                fqlpop.set_engine_option("serial", serial)
                n = fqlpop.step_streams()
                assert n in (1, 4)
                assert n == 1 or n <= q
                assert n == (1 if serial or q < 4 else 4)
    finally:
        fqlpop.reset_engine_options()


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_cpu_allotment_takes_the_smallest_bound(monkeypatch):
    """The CPU leg's thread count is min(sched_getaffinity, cgroup quota): the GPU box's
    affinity mask shows 256 CPUs while the job's share is 16.  OMP_NUM_THREADS
    is recorded but is not a cap (OMP_NUM_THREADS=1 from a launcher must not make
    the baseline single-threaded)."""
    b = _bench_module()
    ncpu = len(os.sched_getaffinity(0))
    monkeypatch.setattr(b, "_cgroup_cpu_quota", lambda: None)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    got = b.cpu_allotment()
    assert got["effective_cpus"] == ncpu and got["omp_num_threads"] == "1"
    monkeypatch.setattr(b, "_cgroup_cpu_quota", lambda: 2)
    assert b.cpu_allotment()["effective_cpus"] == min(2, ncpu)
    monkeypatch.delenv("OMP_NUM_THREADS")
    monkeypatch.setattr(b, "_cgroup_cpu_quota", lambda: None)
    assert b.cpu_allotment()["effective_cpus"] == ncpu


def test_cpu_baseline_is_bounded_when_oversubscribed():
    """256 torch threads on this 8-CPU container (32x oversubscribed, the round-4 hang's
    shape): the leg returns within its wall budget plus one update, never loops on a step
    floor, and records what it measured or abandoned."""
    import time
    import torch
    b = _bench_module()
    wl = b.WORKLOADS["cube"]
    data = b.synthetic_dataset(4096, wl["obs_dim"], wl["action_dim"])
    prev = torch.get_num_threads()
    budget = 3.0
    t0 = time.perf_counter()
    out = b.cpu_baseline(wl, data, budget, thread_counts=[256])
    wall = time.perf_counter() - t0
    assert torch.get_num_threads() == prev
    one_update = out.get("longest_update_s") or 0.0
    assert wall <= budget + one_update + 1.0, (wall, out)
    assert out["leg_s"] <= wall + 0.01
    if out["value"] is None:
        assert "256" in out["abandoned"]
    else:
        assert out["cores"] == 256 and out["rates_by_threads"]["256"] > 0


def test_cpu_baseline_caps_the_whole_leg():
    """A requested budget above CPU_LEG_CAP_S is clamped to it."""
    b = _bench_module()
    wl = b.WORKLOADS["cube"]
    data = b.synthetic_dataset(4096, wl["obs_dim"], wl["action_dim"])
    b.CPU_LEG_CAP_S = 1.0
    out = b.cpu_baseline(wl, data, 1000.0, thread_counts=[2])
    assert out["budget_s"] == 1.0 and out["leg_s"] < 1.0 + out["longest_update_s"] + 1.0


def _plan(members, **cfg):
    from fqlpop import PopulationConfig, split_plan
    base = dict(obs_dim=28, action_dim=5, hidden_dims=(512,) * 4, batch_size=256)
    base.update(cfg)
    return split_plan(PopulationConfig(**base), members)


def test_split_plan_per_members_and_workload():
    """The split plan chosen from same-box A/B runs (DESIGN.md section 6,
    profiles/round5c, round5e): cube at 1-2 members splits every launch; at 2 members the
    critic's LN backward takes 4 blocks per tile (256 blocks, not 512); at 4 members the Euler
    flow runs at 4 blocks per tile; from 6 members nothing splits (the one-step backward at
    128 tiles measured 2.4 % slower split); the BC forward, target critic and critic forward
    run unsplit from 96 tiles (3-5 % faster), the one-step forward (the chain's first launch)
    splits up to 128.  antsoccer (B = 1024): one member splits the flow and the one-step
    backward, two members run unsplit.  The 4th-stream schedule (target critic and TD-column
    backward on sX) runs up to 256 tiles per step since round 5 (+1-4 % at 6-12 members and
    ant 2-4, neutral at 4 and 16, -1.1 % at ant 16: profiles/round5e/ab_small_sched_everywhere.txt,
    ab_4th_stream_ant16_cube3.txt)."""
    import fqlpop
    fqlpop.reset_engine_options()
    p = _plan(1)
    assert p["small_sched"] and p["euler_flow"] == 8 and p["critic_backward"] == 8 and p["critic_backward_td"] == 8
    assert p["onestep_backward"] == 8 and p["critic_forward"] == 4 and p["onestep_forward"] == 4
    p = _plan(2)
    assert p["small_sched"] and p["euler_flow"] == 8
    assert p["critic_backward"] == 4 and p["critic_backward_td"] == 4
    assert p["critic_forward"] == 1 and p["target_critic"] == 4 and p["onestep_backward"] == 8
    assert p["onestep_forward"] == 2 and p["bc_forward"] == 4
    p = _plan(4)
    assert p["small_sched"] and p["euler_flow"] == 4 and p["critic_backward_td"] == 1
    assert p["onestep_backward"] == 4 and p["critic_forward"] == 1 and p["critic_backward"] == 1
    assert p["bc_forward"] == 1 and p["target_critic"] == 1
    for m in (6, 8, 16):
        p = _plan(m)
        assert p["small_sched"] and all(p[s] == 1 for s in fqlpop.population.SPLIT_SITES), (m, p)
    p = _plan(1, obs_dim=42, action_dim=8, batch_size=1024)
    assert p["small_sched"] and p["euler_flow"] == 4 and p["critic_backward_td"] == 1
    assert p["bc_forward"] == 1 and p["target_critic"] == 1 and p["onestep_backward"] == 4
    p = _plan(2, obs_dim=42, action_dim=8, batch_size=1024)
    assert p["small_sched"] and all(p[s] == 1 for s in fqlpop.population.SPLIT_SITES), p
    # the 4th stream up to 256 tiles per step (cube 16 members: neutral; ant 16: -1.1 %)
    assert not _plan(16, obs_dim=42, action_dim=8, batch_size=1024)["small_sched"]
    assert not _plan(8, obs_dim=42, action_dim=8, batch_size=1024)["small_sched"]
    assert not _plan(17)["small_sched"]


def test_split_plan_follows_engine_options():
    import fqlpop
    try:
        fqlpop.set_engine_option("split", 0)
        p = _plan(1)
        assert p["small_sched"] and all(p[s] == 1 for s in fqlpop.population.SPLIT_SITES)
        fqlpop.reset_engine_options()
        fqlpop.set_engine_option("split_sites", 1 << 3)  # the Euler flow unsplit
        p = _plan(2)
        assert p["euler_flow"] == 1 and p["small_sched"] and p["onestep_forward"] > 1
        fqlpop.reset_engine_options()
        fqlpop.set_engine_option("small_sched", 0)  # three streams
        assert not _plan(2)["small_sched"] and not _plan(16)["small_sched"]
        fqlpop.reset_engine_options()
        fqlpop.set_engine_option("serial", 1)  # one stream: no 4th-stream schedule
        assert not _plan(2)["small_sched"]
    finally:
        fqlpop.reset_engine_options()


def test_cgroup_quota_parsing(monkeypatch, tmp_path):
    """cgroup v2 cpu.max ("quota period" or "max period") and v1 cfs_quota_us / cfs_period_us
    (-1 = none), rounded up to whole CPUs."""
    import builtins
    b = _bench_module()
    files = {}
    real_open = builtins.open

    def fake_open(p, *a, **k):
        if p in files:
            f = tmp_path / p.replace("/", "_")
            f.write_text(files[p])
            return real_open(f, *a, **k)
        if str(p).startswith("/sys/fs/cgroup"):
            raise OSError("absent")
        return real_open(p, *a, **k)

    monkeypatch.setattr(builtins, "open", fake_open)
    files.update({"/sys/fs/cgroup/cpu.max": "1600000 100000\n"})
    assert b._cgroup_cpu_quota() == 16
    files["/sys/fs/cgroup/cpu.max"] = "150000 100000\n"
    assert b._cgroup_cpu_quota() == 2
    files["/sys/fs/cgroup/cpu.max"] = "max 100000\n"
    assert b._cgroup_cpu_quota() is None
    del files["/sys/fs/cgroup/cpu.max"]
    files.update({"/sys/fs/cgroup/cpu/cpu.cfs_quota_us": "800000\n", "/sys/fs/cgroup/cpu/cpu.cfs_period_us": "100000\n"})
    assert b._cgroup_cpu_quota() == 8
    files["/sys/fs/cgroup/cpu/cpu.cfs_quota_us"] = "-1\n"
    assert b._cgroup_cpu_quota() is None
