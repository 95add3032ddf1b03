"""Train a world model on the GPU: the reference's train_env_model.py:1-137
(`--model baseline | termination_predictor`, same flags), over a local
OGBench-style .npz dataset (ogbench / wandb are absent: data must already be in
--data_directory; logs go to a CSV under --save_directory).

Saves ``<save_directory>/<env_name>/env_models/<model>.pt`` (flax
``to_bytes`` of the params tree, readable by utils/envmodel.py:load_model) and
``<model>_config.yaml``, as train_env_model.py:127-137 does.  ``multistep`` trains
the baseline cell through a ``--sequence_length`` scan (BPTT on the GPU) and saves
it under ``params/ScanCell_0/cell`` like flax's ``nn.scan`` tree.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import envmodel as em  # noqa: E402
from argparser import build_env_model_config_from_args, get_env_model_argparser  # noqa: E402
from envmodel.flax_msgpack import msgpack_serialize  # noqa: E402
from envmodel.trainer import StatePredictorTrainer, TerminationPredictorTrainer  # noqa: E402
from task.offline_task_npz import load_npz_dataset  # noqa: E402
from utils.logger import CsvLogger  # noqa: E402


class StepLoader:
    """utils/data_loader.py:47-52: uniform minibatches of single transitions."""

    def __init__(self, dataset: dict):
        self.dataset = {k: dataset[k] for k in ("observations", "actions", "rewards", "next_observations")}

    def sample(self, batch_size: int) -> dict:
        idx = np.random.randint(len(self.dataset["observations"]), size=batch_size)
        return {k: v[idx] for k, v in self.dataset.items()}


class MultistepLoader:
    """utils/data_loader.py:25-39: the dataset as [n / 1000][1000] episodes; a batch is
    batch_size windows of sequence_length steps (uniform episode, uniform start in
    [0, 1000 - sequence_length))."""

    episode_length = 1000

    def __init__(self, dataset: dict, sequence_length: int = 128):
        self.sequence_length = sequence_length
        n = len(dataset["observations"])
        if n % self.episode_length:
            raise ValueError(f"multistep: {n} rows is not a whole number of {self.episode_length}-step episodes")
        shape = (n // self.episode_length, self.episode_length)
        self.dataset = {k: np.asarray(dataset[k]).reshape(shape + np.shape(dataset[k])[1:])
                        for k in ("observations", "actions", "rewards", "next_observations")}

    def sample(self, batch_size: int) -> dict:
        ep = np.random.randint(len(self.dataset["observations"]), size=batch_size)
        start = np.random.randint(0, self.episode_length - self.sequence_length, size=batch_size)
        idx = start[:, None] + np.arange(self.sequence_length)
        return {k: v[ep[:, None], idx] for k, v in self.dataset.items()}


class _CsvRunLogger:
    """wandb.log stand-in: long-format CSV (step, key, value) -- train and val rows carry
    different keys, so a fixed-header CSV would drop some."""

    def __init__(self, path: Path):
        self.csv = CsvLogger(str(path))

    def log(self, row: dict, step: int):
        for k, v in row.items():
            self.csv.log({"key": k, "value": v}, step=step)


def main(argv=None):
    config = build_env_model_config_from_args(get_env_model_argparser().parse_args(argv))
    base = config.env_name.replace("-singletask", "").rsplit("-task", 1)[0]
    d = Path(config.data_directory)
    train = load_npz_dataset(d / f"{base}.npz")
    val_path = d / f"{base}-val.npz"
    val = load_npz_dataset(val_path) if val_path.exists() else train
    D, A = train["observations"].shape[-1], train["actions"].shape[-1]
    hidden = tuple(config.model_config.get("hidden_dims", em.DEFAULT_HIDDEN))
    save_dir = Path(config.save_directory) / config.env_name / "env_models"
    save_dir.mkdir(parents=True, exist_ok=True)
    logger = _CsvRunLogger(save_dir / f"{config.model}_log.csv")
    np.random.seed(config.seed)
    if config.model in ("baseline", "multistep"):
        spec = em.EnvModelSpec(D, A, hidden, em.DEFAULT_HIDDEN)
        tp = None
        if config.termination_weight > 0:  # utils/envmodel.py load_model("termination_predictor")
            tp = em.load_flax_msgpack(save_dir / "termination_predictor.pt")
            tp = tp.get("params", tp)
            n = sum(1 for k in tp if k.startswith("Dense_"))
            spec.tp_hidden = tuple(int(np.asarray(tp[f"Dense_{i}"]["kernel"]).shape[1]) for i in range(n - 1))
        if config.model == "multistep":
            loaders = (MultistepLoader(train, config.sequence_length), MultistepLoader(val, config.sequence_length))
        else:
            loaders = (StepLoader(train), StepLoader(val))
        trainer = StatePredictorTrainer(spec, em.init_state_predictor(spec, config.seed), *loaders, config,
                                        logger=logger, tp_params=tp)
    elif config.model == "termination_predictor":
        spec = em.EnvModelSpec(D, A, em.DEFAULT_HIDDEN, hidden)
        trainer = TerminationPredictorTrainer(spec, em.init_termination_predictor(spec, config.seed),
                                              StepLoader(train), StepLoader(val), config, logger=logger)
    else:
        raise ValueError(f"unknown model {config.model!r} (baseline, multistep, termination_predictor)")
    trainer.train()
    with open(save_dir / f"{config.model}_config.yaml", "w") as f:
        yaml.safe_dump({k: list(v) if isinstance(v, tuple) else v for k, v in config.model_config.items()}, f)
    with open(save_dir / f"{config.model}.pt", "wb") as f:
        params = trainer.params
        if config.model == "multistep":  # nn.scan(Cell) tree (envmodel/multistep.py:41-52)
            params = {"ScanCell_0": {"cell": params}}
        f.write(msgpack_serialize({"params": params}))
    trainer.close()
    return save_dir


if __name__ == "__main__":
    print(main())
