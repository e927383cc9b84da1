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


class OtherAgentMixturePolicy(OtherAgentPolicy):
    """Mixture over the other agent's policies (``other_policy.py:155-216``):
    one policy per episode, drawn uniformly by ``sample_initial_state`` and kept
    in the state.  POTMMCP runs it on the GPU when every policy is a
    ``FixedDistributionPolicy`` (planning/policies.py); the particle's policy
    index is drawn on the MIXTURE stream there."""

    def __init__(self, model, agent_id: str, policies: Dict[str, object]):
        super().__init__(model, agent_id)
        assert len(model.possible_agents) == 2, "Currently only supports 2 agents"
        self.policies = policies
        self.action_space = list(range(model.action_spaces[agent_id].n))

    def sample_initial_state(self):
        import random
        policy_id = random.choice(list(self.policies))
        return {"policy_id": policy_id,
                "policy_state": self.policies[policy_id].get_initial_state()}

    def get_next_state(self, action, obs, state):
        pid = state["policy_id"]
        return {"policy_id": pid,
                "policy_state": self.policies[pid].get_next_state(action, obs,
                                                                  state["policy_state"])}

    def sample_action(self, state):
        return self.policies[state["policy_id"]].sample_action(state["policy_state"])

    def get_pi(self, state):
        pi = self.policies[state["policy_id"]].get_pi(state["policy_state"]).probs
        if len(pi) != len(self.action_space):
            for a in self.action_space:
                if a not in pi:
                    pi[a] = 0.0
        return pi

    def close(self):
        for p in self.policies.values():
            p.close()

    @staticmethod
    def load_posggym_agents_policy(model, agent_id, policy_dist):
        raise NotImplementedError("posggym.agents policies are not available to the MI355X engine")
