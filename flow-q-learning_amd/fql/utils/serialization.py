"""flax.serialization stand-ins for the agent (reference trainer/experiment.py:61-63,92,135)."""


def to_state_dict(agent) -> dict:
    return agent.to_state_dict()


def from_state_dict(agent, state_dict: dict):
    return agent.from_state_dict(state_dict)
