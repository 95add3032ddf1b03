"""Command-line flags -> TrainerConfig (reference argparser.py:9-169): trainer
fields as --name, agent fields namespaced as --agent.name.  Note (reference
argparser.py:83-85, kept): --agent.layer_norm is store_true, so the CLI
default is False although AgentConfig's is True; scripts pass it."""
from __future__ import annotations

import argparse
from ast import literal_eval
from pathlib import Path

from trainer.config import AgentConfig, TrainerConfig


def get_argparser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Trainer and Agent Configuration")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--steps", type=int, default=1_000_000)
    p.add_argument("--log_interval", type=int, default=5_000)
    p.add_argument("--eval_interval", type=int, default=100_000)
    p.add_argument("--save_directory", type=str, default="exp/")
    p.add_argument("--data_directory", type=str, default="data/")
    p.add_argument("--use_wandb", action="store_true")
    p.add_argument("--env_name", type=str, default="cube-single-play-singletask-task2-v0")
    p.add_argument("--eval_episodes", type=int, default=50)
    p.add_argument("--buffer_size", type=int, default=2_000_000)

    p.add_argument("--agent.seed", type=int, default=0)
    p.add_argument("--agent.agent_name", type=str, default="fql")
    p.add_argument("--agent.ob_dims", type=int, default=None)
    p.add_argument("--agent.action_dim", type=int, default=None)
    p.add_argument("--agent.lr", type=float, default=3e-4)
    p.add_argument("--agent.batch_size", type=int, default=256)
    p.add_argument("--agent.actor_hidden_dims", type=literal_eval, default="(512, 512, 512, 512)")
    p.add_argument("--agent.value_hidden_dims", type=literal_eval, default="(512, 512, 512, 512)")
    p.add_argument("--agent.layer_norm", action="store_true")
    p.add_argument("--agent.actor_layer_norm", action="store_true")
    p.add_argument("--agent.discount", type=float, default=0.99)
    p.add_argument("--agent.tau", type=float, default=0.005)
    p.add_argument("--agent.q_agg", type=str, default="mean")
    p.add_argument("--agent.alpha", type=float, default=10.0)
    p.add_argument("--agent.flow_steps", type=int, default=10)
    p.add_argument("--agent.normalize_q_loss", action="store_true")
    p.add_argument("--agent.encoder", type=str, default=None)
    p.add_argument("--single_experiment", action="store_true")
    p.add_argument("--job_id", type=int, default=0)
    return p


def build_config_from_args(args: argparse.Namespace) -> TrainerConfig:
    agent_kw, trainer_kw = {}, {}
    for key, value in vars(args).items():
        if key.startswith("agent."):
            agent_kw[key[len("agent."):]] = value
        else:
            trainer_kw[key] = value
    trainer_kw["save_directory"] = Path(trainer_kw["save_directory"])
    trainer_kw["data_directory"] = Path(trainer_kw["data_directory"])
    for k in ("actor_hidden_dims", "value_hidden_dims"):
        if isinstance(agent_kw.get(k), str):
            agent_kw[k] = literal_eval(agent_kw[k])
    agent = AgentConfig(**{k: v for k, v in agent_kw.items() if k in AgentConfig.__dataclass_fields__})
    return TrainerConfig(**{k: v for k, v in trainer_kw.items() if k in TrainerConfig.__dataclass_fields__},
                         agent=agent)


def get_env_model_argparser() -> argparse.ArgumentParser:
    """reference argparser.py:172-262 (train_env_model.py's flags)."""
    p = argparse.ArgumentParser(description="The configurations of the environment model.")
    p.add_argument("--model", type=str, default="baseline")
    p.add_argument("--model.hidden_dims", type=literal_eval, default=(128, 256, 128))
    p.add_argument("--model.latent_dim", type=int, default=4)
    p.add_argument("--true_termination_weight", type=float, default=30.0)
    p.add_argument("--termination_weight", type=float, default=1.0)
    p.add_argument("--reconstruction_weight", type=float, default=1.0)
    p.add_argument("--sequence_length", type=int, default=256)
    p.add_argument("--steps", type=int, default=20000)
    p.add_argument("--env_name", type=str, default="cube-single-play-singletask-task2-v0")
    p.add_argument("--init_learning_rate", type=float, default=1e-3)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--batch_size", type=int, default=256)
    p.add_argument("--val_batches", type=int, default=50)
    p.add_argument("--data_directory", type=str, default="data/")
    p.add_argument("--save_directory", type=str, default="exp/")
    return p


def build_env_model_config_from_args(args: argparse.Namespace):
    """reference argparser.py:265-290: --model.* flags into model_config, the rest
    filtered to the trainer config's fields."""
    from dataclasses import fields

    from envmodel.trainer import EnvModelTrainerConfig
    model_config, trainer_kw = {}, {}
    for k, v in vars(args).items():
        if k.startswith("model."):
            model_config[k[len("model."):]] = v
        else:
            trainer_kw[k] = v
    trainer_kw["save_directory"] = Path(trainer_kw["save_directory"])
    trainer_kw["data_directory"] = Path(trainer_kw["data_directory"])
    names = {f.name for f in fields(EnvModelTrainerConfig)}
    return EnvModelTrainerConfig(**{k: v for k, v in trainer_kw.items() if k in names}, model_config=model_config)
