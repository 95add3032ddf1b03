"""Restore a saved agent (reference utils/agent.py:9-41): config.yaml +
params.pkl written by Experiment.save_agent."""
from __future__ import annotations

import pickle
from pathlib import Path

import yaml

from fql.agents.fql import FQLAgent


def load_agent(agent_directory, sample_batch, agent_filename: str = "params", agent_extension: str = ".pkl"):
    agent_directory = Path(agent_directory)
    config_path = agent_directory / "config.yaml"
    if not config_path.exists():
        raise FileNotFoundError(f"Configuration file not found at {config_path}.")
    with open(config_path) as f:
        agent_config = yaml.safe_load(f)
    for k in ("actor_hidden_dims", "value_hidden_dims"):
        if k in agent_config and isinstance(agent_config[k], list):
            agent_config[k] = tuple(agent_config[k])
    agent = FQLAgent.create(agent_config["seed"], sample_batch["observations"], sample_batch["actions"],
                            agent_config)
    agent_path = agent_directory / (agent_filename + agent_extension)
    if not agent_path.exists():
        raise FileNotFoundError(f"Checkpoint not found at {agent_path}.")
    with open(agent_path, "rb") as f:  # a file this package wrote (Experiment.save_agent)
        state = pickle.load(f)
    return agent.from_state_dict(state["agent"])
