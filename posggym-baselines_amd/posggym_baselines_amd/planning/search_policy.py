"""Search (rollout / prior) policies — ``search_policy.py:16-185``.

The GPU engine runs the uniform random policy in-kernel (``RandomSearchPolicy``:
``sample_action`` = ``Discrete.sample``, uniform ``get_pi``, no value) and a
``SearchPolicyWrapper`` of a fixed-distribution policy (planning/policies.py:
node priors and rollouts, planning/ipomcp.py).  Neural / posggym.agents search
policies are out of scope for this build and are rejected by the
planners.
"""
import abc
from typing import Dict, Optional


class SearchPolicy(abc.ABC):
    def __init__(self, model, agent_id: str, policy_id: str):
        self.model = model
        self.agent_id = agent_id
        self.policy_id = policy_id

    @abc.abstractmethod
    def get_initial_state(self):
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

    @abc.abstractmethod
    def get_value(self, state) -> float:
        ...

    def get_state_from_history(self, initial_state, history):
        state = initial_state
        for a, o in history:
            state = self.get_next_state(a, o, state)
        return state

    def close(self):
        pass


class RandomSearchPolicy(SearchPolicy):
    """Uniform random rollout policy (runs inside the search kernel)."""

    def __init__(self, model, agent_id: str):
        super().__init__(model, agent_id, "RandomSearchPolicy")
        self._action_space = model.action_spaces[agent_id]

    def get_initial_state(self):
        return {}

    def get_next_state(self, action: Optional[int], obs, state):
        return {}

    def sample_action(self, state) -> int:
        return self._action_space.sample()

    def get_pi(self, state) -> Dict[int, float]:
        n = self._action_space.n
        return {a: 1.0 / n for a in range(n)}

    def get_value(self, state) -> float:
        raise NotImplementedError("RandomSearchPolicy does not support value estimates.")


class SearchPolicyWrapper(SearchPolicy):
    """A posggym.agents ``Policy`` as a search policy (``search_policy.py:188-224``)."""

    def __init__(self, policy):
        super().__init__(policy.model, policy.agent_id, policy.policy_id)
        self.policy = policy

    def get_initial_state(self):
        return self.policy.get_initial_state()

    def get_next_state(self, action, obs, state):
        return self.policy.get_next_state(action, obs, state)

    def sample_action(self, state):
        return self.policy.sample_action(state)

    def get_pi(self, state):
        # search_policy.py:214-220: the policy's probs dict, missing actions as 0.0
        pi = self.policy.get_pi(state).probs
        n = self.policy.model.action_spaces[self.policy.agent_id].n
        if len(pi) != n:
            for a in range(n):
                if a not in pi:
                    pi[a] = 0.0
        return pi

    def get_value(self, state):
        return self.policy.get_value(state)

    def close(self):
        self.policy.close()


def load_posggym_agents_search_policy(model, agent_id: str, policy_id: str):
    """``search_policy.py:226-232``: needs posggym.agents (absent from this build)."""
    raise NotImplementedError("posggym.agents policies are not available to the MI355X engine")


class PPOLSTMSearchPolicy(SearchPolicy):
    """``search_policy.py:235-290``: a PPO-LSTM network as search policy --
    neural inference on the search path, out of this build's scope."""

    def __new__(cls, *args, **kwargs):
        raise NotImplementedError("PPO-LSTM search policies are out of the GPU engine's scope")
