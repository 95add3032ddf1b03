"""One population member's training run (reference trainer/experiment.py:16-147).

Same surface as the reference Experiment -- ``train(num_steps) -> bool``,
``evaluate() -> float``, ``save_agent``, ``state_dict``, ``stop`` -- but the
agent is a slot of an HBM-resident population: when the task exposes its
dataset (``Task.device_datasets``) the update loop samples minibatches on
the GPU and runs ``log_interval``-sized chunks of updates per call into the
engine; otherwise it falls back to the reference loop
``batch = task.sample(...); agent.update(batch)``.
"""
from __future__ import annotations

import pickle
from copy import deepcopy
from dataclasses import asdict
from datetime import datetime
import random
from pathlib import Path

import numpy as np

from evaluator.evaluation import evaluate_agent
from fql.agents.fql import FQLAgent
from task.task import Task
from trainer.config import ExperimentConfig, TrainerConfig
from utils.logger import Logger


def agent_config_for(trainer_config: TrainerConfig, experiment_config: ExperimentConfig):
    """AgentConfig with the experiment's tuned fields applied (reference :32-41)."""
    tuned = [(f, v) for f, v in vars(experiment_config).items() if v is not None]
    cfg = deepcopy(trainer_config.agent)
    for f, v in tuned:
        if hasattr(cfg, f):
            setattr(cfg, f, v)
    return cfg, tuned


class Experiment:
    def __init__(self, task: Task, trainer_config: TrainerConfig, experiment_config: ExperimentConfig,
                 state_dict: dict | None = None, population=None, member: int | None = None):
        agent_config, tuned = agent_config_for(trainer_config, experiment_config)
        self.agent_config = agent_config
        example = task.sample("train", 1)
        self.agent = FQLAgent.create(agent_config.seed if experiment_config.seed is None else experiment_config.seed,
                                     example["observations"], example["actions"], asdict(agent_config),
                                     population=population, member=member)
        self.owns_population = population is None
        if self.owns_population:
            dd = task.device_datasets()
            if dd is not None:
                self.agent.population.set_dataset(dd["train"], "train")
                self.agent.population.set_dataset(dd["val"], "val")
        self.on_device = task.device_datasets() is not None

        if state_dict is None:
            name = "_".join(f"{f}_{v}" for f, v in tuned)
            self.experiment_name = f"{name}_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
            self.current_step = 0
        else:
            self.agent.from_state_dict(state_dict["agent"])
            self.experiment_name = state_dict["experiment_name"]
            self.current_step = state_dict["current_step"]

        self.logger = Logger(trainer_config.save_directory, trainer_config.env_name, self.experiment_name,
                             agent_config, use_wandb=trainer_config.use_wandb,
                             state_dict=state_dict["logger"] if state_dict else None)
        self.task = task
        self.steps = trainer_config.steps
        self.log_interval = trainer_config.log_interval
        self.save_directory = Path(trainer_config.save_directory)
        self.env_name = trainer_config.env_name

    # ------------------------------------------------------------------ io
    def state_dict(self) -> dict:
        return {"experiment_name": self.experiment_name, "logger": self.logger.state_dict(),
                "agent": self.agent.to_state_dict(), "current_step": self.current_step}

    def save_agent(self, checkpoint: bool = False):
        filename = f"checkpoint_{self.current_step}.pkl" if checkpoint else "params.pkl"
        path = self.save_directory / self.env_name / self.experiment_name / filename
        path.parent.mkdir(parents=True, exist_ok=True)
        with open(path, "wb") as f:
            pickle.dump({"agent": self.agent.to_state_dict()}, f)

    def stop(self):
        self.logger.close()

    # --------------------------------------------------------------- train
    def log_step(self, train_info: dict, val_info: dict):
        self.logger.log(train_info, step=self.current_step, group="train")
        self.logger.log(val_info, step=self.current_step, group="val")

    def train(self, num_steps: int) -> bool:
        """Run min(num_steps, steps left) updates; True once all steps are done."""
        num_steps = min(num_steps, self.steps - self.current_step)
        if self.on_device:
            train_population([self], num_steps)
        else:
            for _ in range(num_steps):
                self.current_step += 1
                batch = self.task.sample("train", self.agent.config["batch_size"])
                self.agent, info = self.agent.update(batch)
                if self.current_step % self.log_interval == 0:
                    val = self.task.sample("val", self.agent.config["batch_size"])
                    _, val_info = self.agent.total_loss(val, grad_params=None)
                    self.log_step(info, val_info)
        return self.current_step == self.steps

    def evaluate(self, eval_info: dict | None = None, seed: int | None = None) -> float:
        """Success rate of the agent (reference :120-126).  Tasks with an on-GPU
        world model (``evaluate_members``) roll the member on the device;
        ``eval_info`` passes a result the Trainer computed for a whole round.
        ``seed`` None draws the evaluation seed from np.random, as the reference does."""
        if eval_info is None:
            if hasattr(self.task, "evaluate_members") and self.agent.population is not None:
                seed = int(np.random.randint(0, 2**31 - 1)) if seed is None else int(seed)
                eval_info = self.task.evaluate_members(self.agent.population, [self.agent.member], seed)[
                    self.agent.member]
            elif seed is None:
                eval_info, _ = evaluate_agent(agent=self.agent, env=self.task)
            else:
                # evaluate_actor_fn re-seeds random / np.random when given a seed (reference
                # evaluator/evaluation.py:41-43); the reference's own evaluate() passes none
                # (trainer/experiment.py:121), so its global streams (task.sample's batches, the
                # checkpointed np_rng_state) never depend on the evaluations: keep them so here
                py_state, np_state = random.getstate(), np.random.get_state()
                try:
                    eval_info, _ = evaluate_agent(agent=self.agent, env=self.task, seed=seed)
                finally:
                    random.setstate(py_state)
                    np.random.set_state(np_state)
        self.logger.log(eval_info, step=self.current_step, group="eval")
        return eval_info.get("success", 0.0)


def train_population(experiments, num_steps: int) -> None:
    """Advance experiments that share one population in lock-step by num_steps
    updates, logging train/val info at every multiple of log_interval (the
    step numbers the reference logs at).  All must be at the same step."""
    if not experiments or num_steps <= 0:
        return
    pop = experiments[0].agent.population
    steps = {e.current_step for e in experiments}
    if len(steps) != 1:
        raise ValueError("lock-step training needs every experiment at the same step")
    mask = [False] * pop.n
    for e in experiments:
        mask[e.agent.member] = True
    pop.set_active(mask)
    cur = experiments[0].current_step
    target = cur + num_steps
    li = experiments[0].log_interval
    while cur < target:
        nxt = min(target, (cur // li + 1) * li)
        pop.step(nxt - cur)
        cur = nxt
        for e in experiments:
            e.current_step = cur
        if cur % li == 0:
            train_info = pop.read_info("train")
            val_info = pop.total_loss()
            for e in experiments:
                e.log_step(train_info[e.agent.member], val_info[e.agent.member])
