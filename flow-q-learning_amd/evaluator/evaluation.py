"""Episode evaluation loop (reference evaluator/evaluation.py:12-114): roll the
agent's one-step policy in the task's vectorised environments until every env
is done; average the final infos (``success``)."""
from __future__ import annotations

import random
from collections import defaultdict

import numpy as np


def supply_rng(f, seed: int = 0):
    """Feed a fresh integer seed to every call (JAX-key splitting stand-in)."""
    state = {"seed": int(seed)}

    def wrapped(*args, **kwargs):
        state["seed"] = (state["seed"] * 6364136223846793005 + 1442695040888963407) & (2**64 - 1)
        return f(*args, seed=state["seed"], **kwargs)

    return wrapped


def flatten(d, parent_key: str = "", sep: str = "."):
    out = {}
    for k, v in d.items():
        key = f"{parent_key}{sep}{k}" if parent_key else k
        if hasattr(v, "items"):
            out.update(flatten(v, key, sep))
        else:
            out[key] = v
    return out


def evaluate_agent(agent, env, seed: int | None = None, eval_temperature: float = 0):
    actor_fn = supply_rng(agent.sample_actions,
                          seed=seed if seed is not None else np.random.randint(0, 2**32))
    return evaluate_actor_fn(actor_fn, env, seed, eval_temperature)


def evaluate_actor_fn(actor_fn, env, seed: int | None = None, eval_temperature: float = 0):
    if seed is not None:
        random.seed(seed)
        np.random.seed(seed)
    stats = defaultdict(list)
    observations, _ = env.reset(seed=seed)
    done = np.zeros(len(observations), dtype=bool)
    transitions = []
    while not np.all(done):
        actions = np.clip(np.array(actor_fn(observations=observations, temperature=eval_temperature)), -1, 1)
        next_observations, _, terminated, truncated, infos = env.step(actions)
        invalid = np.array([info.get("invalid", False) for info in infos], dtype=bool)
        done = np.logical_or(np.logical_or(terminated, truncated), invalid)
        for i, info in enumerate(infos):
            if done[i] and not invalid[i]:
                for k, v in flatten(info).items():
                    stats[k].append(v)
        transitions.append((observations, actions, invalid))
        observations = next_observations
    return {k: float(np.mean(v)) for k, v in stats.items()}, transitions
