"""POTMMCP drop-in (``potmmcp.py:18-459``) on the GPU engine, for non-neural
policies.

POTMMCP searches with a meta-policy over the ego's policies: every simulation
draws one of them from the meta-policy row of its particle's other-agent
policy (``sample_policy``, ``potmmcp.py:381-389``) and uses it for the
rollout and for the prior of the nodes it creates; every obs node keeps
``action_probs`` (PUCB's prior), moved towards the simulation's policy on
every arrival at an existing child (``potmmcp.py:255-264``).  The other agent
is an ``OtherAgentMixturePolicy``: each particle carries the policy it was
sampled with (``other_policy.py:178-183``).

The engine runs this in the search kernel (``k_search`` with TM = 1,
``include/pomcp.h`` ``pomcp_set_type_policies``) when every policy has an
action distribution that does not depend on its history -- the
``FixedDistributionPolicy`` type of ``planning/policies.py`` (uniform
included).  Policies with recurrent state (posggym.agents networks in the
reference's experiments) are neural inference on the search path and raise
``NotImplementedError``.
"""
import dataclasses
import random
from typing import Dict, Optional

from posggym_baselines_amd import _native as N
from posggym_baselines_amd.planning.config import MCTSConfig
from posggym_baselines_amd.planning.other_policy import OtherAgentMixturePolicy
from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
from posggym_baselines_amd.planning.pomcp import POMCP, RootView
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


class POTMMCP(POMCP):
    """``potmmcp.py:18-301`` on the GPU: ``POTMMCP(model, agent_id, config,
    other_agent_policies, search_policy)`` with ``other_agent_policies`` =
    {other agent: ``OtherAgentMixturePolicy``} and ``search_policy`` a
    ``POTMMCPMetaPolicy``, every policy of both a ``FixedDistributionPolicy``.
    Bit-exact with the reference planner (tests/golden/potmmcp_*.json).
    ``root.action_probs`` is the root's prior after the last search."""

    def __init__(self, model, agent_id, config: MCTSConfig, other_agent_policies,
                 search_policy: "POTMMCPMetaPolicy", *, num_sims: Optional[int] = None,
                 process_group=None):
        assert len(model.possible_agents) == 2, "Currently only supports 2 agents"
        if not isinstance(search_policy, POTMMCPMetaPolicy):
            raise NotImplementedError("POTMMCP searches with a POTMMCPMetaPolicy")
        other = [i for i in model.possible_agents if i != agent_id][0]
        mix = other_agent_policies.get(other)
        for pol in list(search_policy.policies.values()) + list(getattr(mix, "policies", {}).values()):
            if not isinstance(pol, FixedDistributionPolicy):
                raise NotImplementedError(
                    f"policy {getattr(pol, 'policy_id', pol)!r}: the engine runs fixed-distribution "
                    "policies (planning/policies.py); recurrent / neural policies are out of scope")
        if not isinstance(mix, OtherAgentMixturePolicy):
            raise NotImplementedError("POTMMCP's other agent must be an OtherAgentMixturePolicy")
        if config.state_belief_only:
            # the reference draws the other agent's action from its particle's
            # policy state (mcts.py:602-615); with state_belief_only it passes {}
            # and OtherAgentMixturePolicy raises KeyError('policy_id')
            raise ValueError("POTMMCP needs state_belief_only=False (particles carry the "
                             "other agent's policy)")
        self.type_policies = type_policy_tables(model, agent_id, search_policy, mix)
        self._init_planner(model, agent_id, config, search_policy, dict(other_agent_policies),
                           num_sims, process_group, type_policies=self.type_policies)
        self.root = RootViewTM()

    def reset(self):
        super().reset()
        self.root = RootViewTM()

    def update(self, action, obs):
        super().update(action, obs)
        if not isinstance(self.root, RootViewTM):
            self.root = RootViewTM(**dataclasses.asdict(self.root))

    def get_action(self):
        action = super().get_action()
        if not self.root.is_absorbing:
            prior = self._engine.root_prior(0)
            self.root = RootViewTM(**{**dataclasses.asdict(self.root),
                                      "action_probs": {a: p for a, p in enumerate(prior)}})
        return action

    def root_policies(self, replica: int = 0):
        """The other agent's policy id of every root particle (belief order)."""
        ids = list(self.other_agent_policies[
            [i for i in self.model.possible_agents if i != self.agent_id][0]].policies)
        return [ids[j] for j in self._engine.root_policies(replica)]

    def __str__(self):
        return "POTMMCP"


@dataclasses.dataclass
class RootViewTM(RootView):
    action_probs: dict = dataclasses.field(default_factory=dict)


def type_policy_tables(model, agent_id, meta: "POTMMCPMetaPolicy", mix) -> N.PomcpTypePolicies:
    """``pomcp_type_policies`` of a meta-policy over fixed-distribution ego
    policies and a mixture over fixed-distribution other-agent policies: index
    order = the dicts' order (what ``random.choice`` / ``random.choices`` see)."""
    A = model.action_spaces[agent_id].n
    ego_ids, oth_ids = list(meta.policies), list(mix.policies)
    if len(ego_ids) > N.POMCP_MAX_TYPE_POLICIES or len(oth_ids) > N.POMCP_MAX_TYPE_POLICIES:
        raise NotImplementedError("at most 8 ego and 8 other-agent policies")
    tp = N.PomcpTypePolicies()
    tp.num_ego, tp.num_other = len(ego_ids), len(oth_ids)
    for k, pid in enumerate(ego_ids):
        pi = meta.policies[pid].get_pi({}).probs
        for a in range(A):
            tp.ego_pi[k][a] = float(pi.get(a, 0.0))
    for j, oid in enumerate(oth_ids):
        pi = mix.policies[oid].get_pi({}).probs
        for a in range(A):
            tp.other_pi[j][a] = float(pi.get(a, 0.0))
        if oid not in meta.meta_policy:
            raise ValueError(f"meta_policy has no entry for the other agent's policy {oid!r}")
        row = meta.meta_policy[oid]
        tp.meta_len[j] = len(row)
        for i, (eid, w) in enumerate(row.items()):
            tp.meta_policy[j][i] = ego_ids.index(eid)
            tp.meta_weight[j][i] = float(w)
    prior = meta.get_expected_action_probs(None, meta.get_initial_state())
    for a in range(A):
        tp.expected_prior[a] = float(prior[a])
    return tp
