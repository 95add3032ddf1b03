"""`FQLAgent` drop-in backed by the HIP population engine.

Replaces [EXT] ``fql/agents/fql.py`` (MazenAmria/fql fork of seohongpark/fql,
un-vendored submodule, reference .gitmodules:1-4) at the call sites the
reference uses:

* ``FQLAgent.create(seed, ex_observations, ex_actions, config)``
  (reference trainer/experiment.py:44-49, utils/agent.py:24-29)
* ``agent.update(batch) -> (agent, info)``          (trainer/experiment.py:109)
* ``agent.total_loss(batch, grad_params=None)``     (trainer/experiment.py:115)
* ``agent.sample_actions(observations=, seed=, temperature=)``
  (evaluator/evaluation.py:58-64,94)
* ``agent.config["batch_size"]``                    (trainer/experiment.py:108,114)
* ``to_state_dict`` / ``from_state_dict`` in place of flax.serialization
  (trainer/experiment.py:61-63,92,135; utils/agent.py:35)

Differences, by design: the agent is a handle on one member of an
HBM-resident population (``fqlpop.Population``), so ``update`` mutates in
place and returns ``self`` (the reference returns a new immutable agent and
the caller rebinds -- the same call pattern works); noise is drawn on device
from Philox keyed by (seed, update count) instead of JAX threefry.
"""
from __future__ import annotations

import numpy as np

from fql.utils.serialization import flat_to_flax, flax_to_flat, is_flax_layout
from fqlpop import Population, PopulationConfig
from fqlpop._lib import TRAIN_INFO_KEYS, VAL_INFO_KEYS


def _sampler_key(seed: int, alpha: float) -> int:
    """The device sampler's member key (runtime.cpp sample_key: splitmix64 finaliser of
    seed ^ (bits(float32 alpha) << 32 | 0x9E3779B9))."""
    m = (1 << 64) - 1
    ab = int(np.array([alpha], dtype=np.float32).view(np.uint32)[0])
    z = (int(seed) ^ ((ab << 32) | 0x9E3779B9)) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _as_seed(seed) -> int:
    """Accept an int or a (JAX-style) uint32 key array."""
    if seed is None:
        return 0
    if isinstance(seed, (int, np.integer)):
        return int(seed)
    arr = np.asarray(seed).astype(np.uint64).reshape(-1)
    out = 0
    for v in arr:
        out = (out * 0x9E3779B97F4A7C15 + int(v)) & (2**64 - 1)
    return out


class FQLAgent:
    def __init__(self, population: Population, member: int, config: dict):
        self.population = population
        self.member = int(member)
        self.config = dict(config)

    # ------------------------------------------------------------ creation
    @classmethod
    def create(cls, seed, ex_observations, ex_actions, config: dict, population: Population | None = None,
               member: int | None = None):
        ex_obs = np.asarray(ex_observations)
        ex_act = np.asarray(ex_actions)
        cfg = dict(config)
        cfg["ob_dims"] = ex_obs.shape[1:]
        cfg["action_dim"] = int(ex_act.shape[-1])
        if population is None:
            pcfg = PopulationConfig.from_agent_config(cfg, int(ex_obs.shape[-1]), int(ex_act.shape[-1]))
            population = Population(pcfg, [float(cfg.get("alpha", 10.0))], [int(seed)])
            member = 0
        return cls(population, member, cfg)

    # ------------------------------------------------------------ hot path
    def _only_me(self):
        pop = self.population
        if not (pop.active.sum() == 1 and pop.active[self.member]):
            mask = np.zeros(pop.n, dtype=bool)
            mask[self.member] = True
            pop.set_active(mask)

    def update(self, batch: dict):
        """One FQL update on a host minibatch; returns (self, info)."""
        self._only_me()
        self.population.step_injected([batch])
        info = self.population.read_info("train")[self.member]
        return self, info

    def total_loss(self, batch: dict, grad_params=None, rng=None):
        """Losses on ``batch`` without updating; returns (loss, info) with the
        10 critic/ and actor/ keys."""
        self._only_me()
        info = self.population.total_loss([batch])[self.member]
        return info["critic/critic_loss"] + info["actor/actor_loss"], info

    def sample_actions(self, observations, seed=None, temperature: float = 1.0):
        return self.population.sample_actions(self.member, observations, seed=_as_seed(seed))

    # ----------------------------------------------------------- state dict
    def to_state_dict(self) -> dict:
        """``flax.serialization.to_state_dict(agent)`` layout (fql/utils/serialization.py):
        {rng, network: {step, params: {modules_<net>: ...}, opt_state}}.  ``rng`` holds the
        member's device sampler key (Philox, keyed by seed and alpha) as two uint32 words."""
        pop = self.population
        key = _sampler_key(int(pop.seeds[self.member]), float(pop.alphas[self.member]))
        return flat_to_flax(pop.state_dict(self.member), rng=[key & 0xFFFFFFFF, key >> 32])

    def from_state_dict(self, sd: dict):
        """Accepts the flax layout or the engine's flat member state (older checkpoints)."""
        flat = flax_to_flat(sd) if is_flax_layout(sd) else sd
        self.population.load_state_dict(self.member, flat)
        return self

    @property
    def step(self) -> int:
        return self.population.get_count(self.member)


__all__ = ["FQLAgent", "TRAIN_INFO_KEYS", "VAL_INFO_KEYS"]
