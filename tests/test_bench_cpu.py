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


def test_population_passes_hw_queues_before_create(monkeypatch):
    """Population hands GPU_MAX_HW_QUEUES to the engine before fqlpop_create (here create
    then fails: no GPU in the CPU suite), so a caller running the HIP runtime with 2 queues
    gets the one-stream capture instead of the runtime's crash in hipGraphLaunch."""
    import fqlpop
    from fqlpop import Population, PopulationConfig
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    try:
        try:
            Population(PopulationConfig(), [3.0], [1]).close()  # (a GPU host: create succeeds)
        except fqlpop.FqlpopError:
            pass
        assert fqlpop.get_engine_option("hw_queues") == 2
    finally:
        fqlpop.reset_engine_options()
