"""alpha-sweep driver (reference tune_alpha.py:14-95), same flags and flow:
alpha = logspace(log10 3, log10 1000, --number_of_alphas), seeds =
random.sample(range(10000), --number_of_seeds) after random.seed(--seed);
--single_experiment --job_id=i runs one (alpha, seed) to completion with a
checkpoint every eval_interval; otherwise an Identity-strategy Trainer trains
the whole population (here: all members together on the GPU) and writes
<save>/<env>/checkpoint.pkl.  --strategy successive_halving selects halving.

Data: --task synthetic (default; SURVEY.md 8d transitions + a toy evaluation
env), --task npz (local OGBench .npz files under --data_directory) or --task
simulated (candidates scored by world-model rollouts on the GPU).

Multi-GPU (BASELINE configs 4 / 5): launched by torch.distributed.run with one
process per GPU (``python -m torch.distributed.run --nproc-per-node 8
--master-addr 127.0.0.1 tune_alpha.py ...``), the population is sharded over the
ranks by trainer.distributed_trainer.DistributedTrainer (RCCL over xGMI gathers
the scores and moves members after pruning); rank 0 writes the checkpoint.
"""
from __future__ import annotations

import itertools
import os
import pickle
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from argparser import build_config_from_args, get_argparser  # noqa: E402
from hpo.identity import Identity  # noqa: E402
from hpo.successive_halving import SuccessiveHalving  # noqa: E402
from trainer.config import ExperimentConfig  # noqa: E402
from trainer.experiment import Experiment  # noqa: E402
from trainer.trainer import Trainer  # noqa: E402


def make_task(args, config):
    if args.task == "simulated":
        # world-model evaluation on the GPU (BASELINE config 5): the reference's env-model files
        # under <save>/<env>/env_models if present, else a seeded synthetic model
        from task.offline_task_simulated import OfflineTaskWithSimulatedEvaluations
        env_dir = config.save_directory / config.env_name / "env_models"
        return OfflineTaskWithSimulatedEvaluations(
            config.env_name, model=args.env_model, save_directory=config.save_directory if env_dir.exists() else None,
            n_rows=args.synthetic_rows, num_evaluation_envs=config.eval_episodes,
            max_episode_steps=args.max_episode_steps, seed=config.seed)
    if args.task == "npz":
        from task.offline_task_npz import OfflineTaskNpz
        return OfflineTaskNpz(config.env_name, config.data_directory)
    from task.offline_task_synthetic import OfflineTaskSynthetic
    return OfflineTaskSynthetic(config.env_name, n_rows=args.synthetic_rows,
                                num_evaluation_envs=min(config.eval_episodes, 64), seed=config.seed)


def main(argv=None):
    parser = get_argparser()
    parser.add_argument("--max_evaluations", type=int, default=200)
    parser.add_argument("--number_of_seeds", type=int, default=1)
    parser.add_argument("--number_of_alphas", type=int, default=1)
    parser.add_argument("--task", choices=("synthetic", "npz", "simulated"), default="synthetic")
    parser.add_argument("--env_model", choices=("baseline", "multistep"), default="multistep")
    parser.add_argument("--max_episode_steps", type=int, default=1000)
    parser.add_argument("--synthetic_rows", type=int, default=100_000)
    parser.add_argument("--strategy", choices=("identity", "successive_halving"), default="identity")
    parser.add_argument("--fraction", type=float, default=0.5)
    parser.add_argument("--history_length", type=int, default=1)
    # SuccessiveHalving's evaluation horizon E (hpo/successive_halving.py milestones).  The
    # reference passes --max_evaluations, which Trainer.train spends per candidate: with N
    # candidates evaluated every round the milestones (in evaluations per candidate, >= h)
    # are then out of reach for N >= 8 at h = 4.  The reference's StrategyEvaluator counts E in
    # rounds (steps / eval_interval); --halving_horizon selects that reading.  Default: the
    # reference wiring.
    parser.add_argument("--halving_horizon", type=int, default=None)
    args = parser.parse_args(argv)
    config = build_config_from_args(args)
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    device = 0
    if world_size > 1 and not args.single_experiment:
        import torch
        import torch.distributed as dist
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        n_dev = torch.cuda.device_count()
        if n_dev >= world_size:  # one GPU per rank: RCCL (the "nccl" backend) over xGMI
            device = local_rank
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:  # fewer GPUs than ranks (a rehearsal on a small box): ranks share GPUs, gloo
            device = local_rank % max(n_dev, 1)
            dist.init_process_group("gloo")

    random.seed(config.seed)
    np.random.seed(config.seed)
    alpha_values = np.logspace(np.log10(3), np.log10(1000), num=args.number_of_alphas).tolist()
    seeds = random.sample(range(10000), args.number_of_seeds)
    combinations = list(itertools.product(alpha_values, seeds))
    task = make_task(args, config)

    if args.single_experiment:
        alpha, seed = combinations[args.job_id]
        experiment = Experiment(task, config, ExperimentConfig(seed=seed, alpha=alpha))
        done = False
        while not done:
            done = experiment.train(config.eval_interval)
            experiment.save_agent(checkpoint=True)
        experiment.stop()
        return

    configs = [ExperimentConfig(seed=seed, alpha=alpha) for alpha, seed in combinations]
    ckpt = config.save_directory / config.env_name / "checkpoint.pkl"
    state = {}
    if ckpt.exists():
        with open(ckpt, "rb") as f:  # written by this script
            state = pickle.load(f)
    if args.strategy == "identity":
        strategy = Identity(population=configs, total_evaluations=0, state_dict=state.get("strategy"))
    else:
        horizon = args.max_evaluations if args.halving_horizon is None else args.halving_horizon
        strategy = SuccessiveHalving(population=set(configs), total_evaluations=horizon,
                                     fraction=args.fraction, history_length=args.history_length,
                                     state_dict=state.get("strategy"))
    if world_size > 1:
        from trainer.distributed_trainer import DistributedTrainer
        trainer = DistributedTrainer(task, strategy, config, state_dict=state.get("trainer"), device=device)
    else:
        trainer = Trainer(task, strategy, config, state_dict=state.get("trainer"))
    trainer.train(max_evaluations=args.max_evaluations)
    trainer_state = trainer.state_dict()  # collective under DistributedTrainer (rank 0 gets it)
    if trainer_state is not None:
        ckpt.parent.mkdir(parents=True, exist_ok=True)
        with open(ckpt, "wb") as f:
            pickle.dump({"trainer": trainer_state, "strategy": trainer.strategy.state_dict()}, f)
    if world_size > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
