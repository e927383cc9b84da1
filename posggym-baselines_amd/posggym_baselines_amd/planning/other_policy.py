"""Other-agent policies inside search — ``other_policy.py:10-154``.

POMCP models every other agent as uniform random; the engine samples their
actions in-kernel from the agent's action-space stream.
"""
import abc
from typing import Dict, Optional


class OtherAgentPolicy(abc.ABC):
    def __init__(self, model, agent_id: str):
        self.model = model
        self.agent_id = agent_id

    @abc.abstractmethod
    def sample_initial_state(self):
        ...

    @abc.abstractmethod
    def get_next_state(self, action, obs, state):
        ...

    @abc.abstractmethod
    def sample_action(self, state):
        ...

    @abc.abstractmethod
    def get_pi(self, state) -> Dict[int, float]:
        ...

    def get_state_from_history(self, initial_state, history):
        state = initial_state
        for a, o in history:
            state = self.get_next_state(a, o, state)
        return state

    def close(self):
        pass


class RandomOtherAgentPolicy(OtherAgentPolicy):
    def __init__(self, model, agent_id: str):
        super().__init__(model, agent_id)
        self._action_space = model.action_spaces[agent_id]

    def sample_initial_state(self):
        return {}

    def get_next_state(self, action: Optional[int], obs, state):
        return {}

    def sample_action(self, state) -> int:
        return self._action_space.sample()

    def get_pi(self, state) -> Dict[int, float]:
        n = self._action_space.n
        return {a: 1.0 / n for a in range(n)}
