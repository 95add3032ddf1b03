"""Run configuration dataclasses.

Field names, defaults and types follow the reference's trainer/config.py:5-44
(AgentConfig, ExperimentConfig, TrainerConfig) so configs, checkpoints and the
argparser round-trip unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path


@dataclass
class AgentConfig:
    seed: int = 0
    agent_name: str = "fql"
    ob_dims: int | None = None
    action_dim: int | None = None
    lr: float = 3e-4
    batch_size: int = 256
    actor_hidden_dims: tuple = (512, 512, 512, 512)
    value_hidden_dims: tuple = (512, 512, 512, 512)
    layer_norm: bool = True
    actor_layer_norm: bool = False
    discount: float = 0.99
    tau: float = 0.005
    q_agg: str = "mean"
    alpha: float = 10.0
    flow_steps: int = 10
    normalize_q_loss: bool = False
    encoder: str | None = None


@dataclass(frozen=True)
class ExperimentConfig:
    """One population member: the tuned hyper-parameters (hashable: used as a
    dict key by Trainer and the HPO strategies)."""
    seed: int | None = None
    alpha: float | None = None


@dataclass
class TrainerConfig:
    seed: int = 0
    steps: int = 1_000_000
    log_interval: int = 5_000
    eval_interval: int = 100_000
    save_directory: Path = Path("exp/")
    data_directory: Path = Path("data/")
    use_wandb: bool = False
    env_name: str = "cube-single-play-singletask-task2-v0"
    agent: AgentConfig = field(default_factory=AgentConfig)
    eval_episodes: int = 50
    buffer_size: int = 2_000_000
