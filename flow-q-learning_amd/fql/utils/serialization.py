"""The agent state dict in the layout of ``flax.serialization.to_state_dict(FQLAgent)``.

The reference exchanges agents through flax's state dicts
(trainer/experiment.py:61-63,92,135 pickle ``{"agent": to_state_dict(agent)}``;
utils/agent.py:35 ``from_state_dict``).  Upstream FQL [EXT, fql/agents/fql.py,
fql/utils/flax_utils.py; the fork's commit is not recorded, so this layout is
**unpinned**: no file in the reference holds a saved agent] makes that dict:

    {"rng": uint32[2],                                  # FQLAgent.rng (a JAX PRNG key)
     "network": {                                       # flax_utils.TrainState
        "step": int,                                    # apply_gradients calls
        "params": {                                     # ModuleDict(modules=...)
           "modules_actor_bc_flow":      {"mlp": MLP},          # ActorVectorField.mlp
           "modules_actor_onestep_flow": {"mlp": MLP},
           "modules_critic":             {"value_net": MLP},    # Value.value_net (ensemblize:
           "modules_target_critic":      {"value_net": MLP}},   #  leading axis num_qs)
        "opt_state": {"0": {"count": int32, "mu": params, "nu": params},  # optax.adam =
                      "1": {}}}}                                          # chain(scale_by_adam, scale)

with MLP = {"Dense_i": {"kernel": [in, out], "bias": [out]}, "LayerNorm_i": {"scale", "bias"}}.
``config`` is a non-pytree field and is not in the dict.

The engine's own member state (``fqlpop.Population.state_dict``) is flat:
``{"params": {net: {"Dense_0/kernel": ...}}, "opt_state": {"count", "mu", "nu"}, "alpha",
"seed"}``.  ``flat_to_flax`` / ``flax_to_flat`` convert both ways; ``from_state_dict``
accepts either, so checkpoints written before this layout still load.
"""
from __future__ import annotations

import numpy as np

# engine net name -> (ModuleDict key, the module's attribute holding the MLP)
MODULES = {
    "actor_bc_flow": ("modules_actor_bc_flow", "mlp"),
    "actor_onestep_flow": ("modules_actor_onestep_flow", "mlp"),
    "critic": ("modules_critic", "value_net"),
    "target_critic": ("modules_target_critic", "value_net"),
}
_NET_OF = {v[0]: (k, v[1]) for k, v in MODULES.items()}


def is_flax_layout(sd: dict) -> bool:
    return isinstance(sd, dict) and "network" in sd


def params_to_flax(tree: dict) -> dict:
    """{net: {"Dense_0/kernel": a}} -> {"modules_<net>": {mlp|value_net: {"Dense_0": {"kernel": a}}}}."""
    out = {}
    for net, leaves in tree.items():
        mod, attr = MODULES[net]
        inner = {}
        for name, arr in leaves.items():
            layer, leaf = name.split("/")
            inner.setdefault(layer, {})[leaf] = np.asarray(arr)
        out[mod] = {attr: inner}
    return out


def params_from_flax(tree: dict) -> dict:
    out = {}
    for mod, body in tree.items():
        if mod not in _NET_OF:
            raise KeyError(f"unexpected module {mod!r} in the flax params tree")
        net, attr = _NET_OF[mod]
        if set(body) != {attr}:
            raise KeyError(f"{mod}: expected the single submodule {attr!r}, got {sorted(body)}")
        out[net] = {f"{layer}/{leaf}": np.asarray(arr) for layer, leaves in body[attr].items()
                    for leaf, arr in leaves.items()}
    return out


def flat_to_flax(sd: dict, rng=None) -> dict:
    """Engine member state -> the upstream FQLAgent state-dict layout."""
    count = int(sd["opt_state"]["count"])
    if rng is None:
        rng = np.zeros(2, np.uint32)
    return {"rng": np.asarray(rng, dtype=np.uint32).reshape(2),
            "network": {"step": count,
                        "params": params_to_flax(sd["params"]),
                        "opt_state": {"0": {"count": np.asarray(count, dtype=np.int32),
                                            "mu": params_to_flax(sd["opt_state"]["mu"]),
                                            "nu": params_to_flax(sd["opt_state"]["nu"])},
                                      "1": {}}}}


def flax_to_flat(sd: dict) -> dict:
    """The upstream FQLAgent state-dict layout -> engine member state (no alpha / seed:
    those live in the agent's config, which flax does not serialise)."""
    net = sd["network"]
    adam = net["opt_state"]["0"]
    count = int(np.asarray(adam["count"]))
    if int(net["step"]) != count:
        raise ValueError(f"TrainState.step {int(net['step'])} != adam count {count}")
    return {"params": params_from_flax(net["params"]),
            "opt_state": {"count": count, "mu": params_from_flax(adam["mu"]), "nu": params_from_flax(adam["nu"])}}


def params_of(sd: dict) -> dict:
    """{net: {"Dense_0/kernel": ...}} parameters of a state dict in either layout."""
    return params_from_flax(sd["network"]["params"]) if is_flax_layout(sd) else sd["params"]


def to_state_dict(agent) -> dict:
    return agent.to_state_dict()


def from_state_dict(agent, state_dict: dict):
    return agent.from_state_dict(state_dict)
