"""POTMMCP API surface (``potmmcp.py:18-459``) -- not on the GPU path.

POTMMCP searches with a meta-policy over posggym.agents policies (PPO-LSTM
networks in the reference's experiments): every simulation samples one of them
(``sample_policy``, ``potmmcp.py:381-389``) for its rollout / prior, and every
tree node keeps the networks' recurrent states.  That is neural inference on
the search path -- a different (MFMA) roofline, out of this build's scope
(DESIGN.md §9).  The classes below keep the reference's import surface and the
meta-policy's host arithmetic; constructing the planner raises
``NotImplementedError`` instead of running a CPU fallback.
"""
import random
from typing import Dict, Optional

from posggym_baselines_amd.planning.search_policy import SearchPolicy, SearchPolicyWrapper


class POTMMCPMetaPolicy(SearchPolicy):
    """``potmmcp.py:304-459``: other-agent policy id -> distribution over the
    ego's policies."""

    def __init__(self, model, agent_id: str, policies: Dict[str, object],
                 meta_policy: Dict[str, Dict[str, float]]):
        super().__init__(model, agent_id, "POTMMCPMetaPolicy")
        assert len(model.possible_agents) == 2, "Currently only supports 2 agents"
        assert len(meta_policy) > 0
        for dist in meta_policy.values():
            assert all(k in policies for k in dist)
            assert abs(sum(dist.values()) - 1) < 1e-6
        self.other_agent_id = [i for i in model.possible_agents if i != agent_id][0]
        self.policies = policies
        self.meta_policy = meta_policy
        self.action_space = list(range(model.action_spaces[agent_id].n))

    def get_initial_state(self):
        return {k: pi.get_initial_state() for k, pi in self.policies.items()}

    def get_next_state(self, action, obs, state):
        return {k: self.policies[k].get_next_state(action, obs, s) for k, s in state.items()}

    def sample_action(self, state):
        raise NotImplementedError("POTMMCPMetaPolicy does not support action sampling; "
                                  "use sample_policy")

    def get_pi(self, state):
        raise NotImplementedError("POTMMCPMetaPolicy does not support get_pi; use sample_policy")

    def get_value(self, state):
        raise NotImplementedError("POTMMCPMetaPolicy does not support value estimates")

    def sample_policy(self, other_agent_policy_state):
        dist = self.meta_policy[other_agent_policy_state[self.other_agent_id]["policy_id"]]
        pid = random.choices(list(dist), weights=list(dist.values()), k=1)[0]
        return SearchPolicyWrapper(self.policies[pid])

    def get_expected_action_probs(self, other_agent_policy_dist: Optional[Dict[str, float]],
                                  policy_state) -> Dict[int, float]:
        """Action prior under a distribution over the other agent's policies
        (uniform when None), ``potmmcp.py:391-431``."""
        if other_agent_policy_dist is None:
            other_agent_policy_dist = {k: 1.0 / len(self.meta_policy) for k in self.meta_policy}
        expected = {k: 0.0 for k in self.policies}
        for oid, prob in other_agent_policy_dist.items():
            for pid, mp in self.meta_policy[oid].items():
                expected[pid] += prob * mp
        total = sum(expected.values())
        for k in expected:
            expected[k] /= total
        dist = {a: 0.0 for a in self.action_space}
        for pid, pp in expected.items():
            pi = self.policies[pid].get_pi(policy_state[pid])
            for a, ap in getattr(pi, "probs", pi).items():
                dist[a] += pp * ap
        s = sum(dist.values())
        return {a: v / s for a, v in dist.items()}


class POTMMCP:
    """``potmmcp.py:18-301`` -- rejected: its search policies are networks."""

    def __init__(self, model, agent_id, config, other_agent_policies, search_policy):
        raise NotImplementedError(
            "POTMMCP searches with posggym.agents (neural) meta-policies; the MI355X engine "
            "runs POMCP / I-NTMCP / IPOMCP with random policies (DESIGN.md §9)")
