"""CSV (+ optional wandb) metric logging (reference utils/logger.py:12-144):
train.csv / val.csv / eval.csv per experiment and its config.yaml."""
from __future__ import annotations

import os
from dataclasses import asdict
from pathlib import Path

import yaml

try:  # wandb is optional (not installed in this image)
    import wandb  # type: ignore
except Exception:  # pragma: no cover
    wandb = None


class CsvLogger:
    def __init__(self, path, resume: bool = False):
        self.path = path
        os.makedirs(os.path.dirname(path), exist_ok=True)
        self.header = None
        if resume and os.path.exists(path) and os.path.getsize(path) > 0:
            with open(path) as f:
                self.header = f.readline().strip().split(",")
        self.file = open(path, "a" if resume else "w")

    def log(self, row: dict, step: int | None = None):
        row = dict(row)
        if step is not None:
            row["step"] = step
        if self.file is None:  # a stopped experiment that a strategy brought back appends
            self.file = open(self.path, "a")
        if self.header is None:
            self.header = list(row)
            self.file.write(",".join(self.header) + "\n")
        self.file.write(",".join(str(row.get(k, "")) for k in self.header) + "\n")
        self.file.flush()

    def close(self):
        if self.file is not None:
            self.file.close()
            self.file = None


class Logger:
    def __init__(self, save_directory: Path, env_name: str, experiment_name: str, config,
                 use_wandb: bool = False, state_dict: dict | None = None):
        root = Path(save_directory) / env_name / experiment_name
        resume = state_dict is not None
        self.train_logger = CsvLogger(root / "train.csv", resume=resume)
        self.val_logger = CsvLogger(root / "val.csv", resume=resume)
        self.eval_logger = CsvLogger(root / "eval.csv", resume=resume)
        cfg = asdict(config) if hasattr(config, "__dataclass_fields__") else dict(config)
        with open(root / "config.yaml", "w") as f:
            yaml.safe_dump({k: (list(v) if isinstance(v, tuple) else v) for k, v in cfg.items()}, f)
        self.wandb_run = None
        if use_wandb:
            if wandb is None:
                raise RuntimeError("--use_wandb requested but wandb is not installed")
            kwargs = dict(project="fql", name=f"{env_name}_{experiment_name}", config=cfg,
                          dir=str(save_directory), resume="allow")
            if state_dict is not None and state_dict.get("wandb_run"):
                kwargs["id"] = state_dict["wandb_run"]["id"]
            self.wandb_run = wandb.init(**kwargs)

    def state_dict(self) -> dict:
        return {"wandb_run": {"id": self.wandb_run.id} if self.wandb_run is not None else None}

    def log(self, data: dict, step: int, group: str):
        logger = {"train": self.train_logger, "val": self.val_logger, "eval": self.eval_logger}[group]
        logger.log(data, step=step)
        if self.wandb_run is not None:
            self.wandb_run.log({f"{group}/{k}": v for k, v in data.items()}, step=step)

    def close(self):
        for lg in (self.train_logger, self.val_logger, self.eval_logger):
            lg.close()
        if self.wandb_run is not None:
            self.wandb_run.finish()
