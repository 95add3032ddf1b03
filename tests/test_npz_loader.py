"""task/offline_task_npz.py on small synthetic OGBench-style files (CPU)."""
import numpy as np
import pytest


def _raw_two_episodes(tmp_path, name="cube-single-play.npz", with_rewards=True):
    # two trajectories of 4 states each: s0..s3 (terminal on s3), then t0..t3
    obs = np.arange(8 * 3, dtype=np.float32).reshape(8, 3)
    act = np.linspace(-2, 2, 8 * 2, dtype=np.float32).reshape(8, 2)
    term = np.array([0, 0, 0, 1, 0, 0, 0, 1], np.float32)
    d = {"observations": obs, "actions": act, "terminals": term}
    if with_rewards:
        d["rewards"] = np.array([-1, -1, 0, -1, -1, 0, -1, -1], np.float32)
        d["masks"] = 1.0 - (d["rewards"] == 0)
    np.savez(tmp_path / name, **d)
    return d


def test_raw_layout_drops_terminal_rows_and_shifts_within_episodes(tmp_path):
    from task.offline_task_npz import load_npz_dataset
    raw = _raw_two_episodes(tmp_path)
    ds = load_npz_dataset(tmp_path / "cube-single-play.npz")
    keep = [0, 1, 2, 4, 5, 6]
    assert ds["observations"].shape == (6, 3)
    np.testing.assert_array_equal(ds["observations"], raw["observations"][keep])
    np.testing.assert_array_equal(ds["next_observations"], raw["observations"][[1, 2, 3, 5, 6, 7]])
    np.testing.assert_array_equal(ds["terminals"], [0, 0, 1, 0, 0, 1])
    np.testing.assert_array_equal(ds["rewards"], raw["rewards"][keep])
    np.testing.assert_array_equal(ds["masks"], raw["masks"][keep])
    assert np.all(np.abs(ds["actions"]) <= 1 - 1e-5)
    np.testing.assert_allclose(ds["actions"], np.clip(raw["actions"][keep], -1 + 1e-5, 1 - 1e-5))
    # no transition crosses the episode boundary: s2 -> s3 and t0 follows s3's episode end
    assert not np.any(np.all(ds["observations"] == raw["observations"][3], axis=1))


def test_transition_layout_used_as_is(tmp_path):
    from task.offline_task_npz import load_npz_dataset
    n = 5
    d = {"observations": np.ones((n, 3), np.float32), "next_observations": 2 * np.ones((n, 3), np.float32),
         "actions": np.zeros((n, 2), np.float32), "rewards": -np.ones(n, np.float32),
         "masks": np.ones(n, np.float32)}
    np.savez(tmp_path / "x.npz", **d)
    ds = load_npz_dataset(tmp_path / "x.npz")
    assert ds["observations"].shape == (n, 3) and np.all(ds["next_observations"] == 2)
    assert np.all(ds["terminals"] == 0)


def test_files_without_rewards_or_masks_are_refused(tmp_path):
    from task.offline_task_npz import load_npz_dataset
    _raw_two_episodes(tmp_path, with_rewards=False)
    with pytest.raises(ValueError, match="rewards"):
        load_npz_dataset(tmp_path / "cube-single-play.npz")


def test_task_finds_train_and_val_files(tmp_path):
    from task.offline_task_npz import OfflineTaskNpz
    _raw_two_episodes(tmp_path, "cube-single-play.npz")
    _raw_two_episodes(tmp_path, "cube-single-play-val.npz")
    task = OfflineTaskNpz("cube-single-play-singletask-task2-v0", tmp_path)
    b = task.sample("train", 16)
    assert b["observations"].shape == (16, 3) and set(b) >= {"rewards", "masks", "next_observations"}
    dd = task.device_datasets()
    assert dd["val"]["observations"].shape == (6, 3)
