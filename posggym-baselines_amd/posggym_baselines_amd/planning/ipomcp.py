"""``MCTS`` / I-POMCP drop-ins: ``mcts.py:22-91`` (the base planner with the
other agents' policies given by the caller) and ``ipomcp.py:11-38`` (which
only forwards them to ``MCTS``), on the GPU POMCP engine.

The reference searches with the other agents' actions drawn from those
policies (``mcts.py:602-615``) -- from each particle's policy state when
``state_belief_only=False`` (``HistoryPolicyState``, ``belief.py:12-30``) --
and with the search policy's prior on every node it creates (``mcts.py:621-645``)
and its actions in the rollouts (``mcts.py:405-452``).

On the engine:
  * random policies on both sides (``RandomSearchPolicy``,
    ``RandomOtherAgentPolicy``, ``other_policy.py:132-154``) are the plain POMCP
    kernel: the random other agent's policy state is ``{}`` whatever the
    history, so carrying the histories changes no draw and no statistic
    (``tests/golden/ipomcp_*.json``, the reference IPOMCP with
    ``state_belief_only=False``);
  * fixed-distribution policies (``planning/policies.py``) run on the
    type-based machinery of the search kernel (``pomcp_type_policies``): a
    search policy ``SearchPolicyWrapper(FixedDistributionPolicy)`` gives every
    node its prior (PUCB's, and its N = 0 draw) and draws the rollouts; the
    other agent is a stateless ``FixedDistributionPolicy``
    (``state_belief_only=True``) or an ``OtherAgentMixturePolicy`` over them
    (``state_belief_only=False``: each particle draws its policy at the initial
    update and keeps it, ``other_policy.py:180-185``).  The moving average of
    a child's ``action_probs`` (``mcts.py:358-367``) adds ``(pi - p) / visits``
    where both are the search policy's fixed ``pi``: an exact identity, which
    the engine's prior lines reproduce bit for bit
    (``tests/golden/mcts_*.json``, made by the real reference planners).
History-dependent (posggym.agents network / PPO) policies are outside the GPU
path and raise ``NotImplementedError``.
"""
import dataclasses
from typing import Dict, Optional

from posggym_baselines_amd import _native as N
from posggym_baselines_amd.planning.config import MCTSConfig
from posggym_baselines_amd.planning.other_policy import (OtherAgentMixturePolicy,
                                                          OtherAgentPolicy,
                                                          RandomOtherAgentPolicy)
from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
from posggym_baselines_amd.planning.pomcp import POMCP
from posggym_baselines_amd.planning.search_policy import (RandomSearchPolicy, SearchPolicy,
                                                           SearchPolicyWrapper)


def _named(policy, name) -> bool:
    # ours, or the reference's class of the same name
    return type(policy).__name__ == name


def _is_random_other(policy) -> bool:
    return isinstance(policy, RandomOtherAgentPolicy) or _named(policy, "RandomOtherAgentPolicy")


def _is_random_search(policy) -> bool:
    return isinstance(policy, RandomSearchPolicy) or _named(policy, "RandomSearchPolicy")


def _fixed_probs(policy, A):
    """The action distribution of a fixed-distribution policy, action order."""
    if not isinstance(policy, FixedDistributionPolicy):
        raise NotImplementedError(
            f"policy {getattr(policy, 'policy_id', policy)!r}: the engine runs fixed-distribution "
            "policies (planning/policies.py); recurrent / neural policies are out of scope")
    pi = policy.get_pi(policy.get_initial_state()).probs
    if list(pi) != list(range(len(pi))):
        raise NotImplementedError("random.choices over a prior in an order other than the "
                                  "actions' is not supported")
    return [float(pi.get(a, 0.0)) for a in range(A)]


def search_policy_probs(model, agent_id, search_policy):
    """None for the uniform random search policy, else its fixed action
    distribution (``SearchPolicyWrapper(FixedDistributionPolicy)``)."""
    if _is_random_search(search_policy):
        return None
    A = model.action_spaces[agent_id].n
    inner = getattr(search_policy, "policy", None)
    if (isinstance(search_policy, SearchPolicyWrapper) or _named(search_policy, "SearchPolicyWrapper")) \
            and inner is not None:
        return _fixed_probs(inner, A)
    if isinstance(search_policy, FixedDistributionPolicy):
        return _fixed_probs(search_policy, A)
    raise NotImplementedError(
        "the GPU engine runs the uniform random search policy or a fixed-distribution one "
        f"(SearchPolicyWrapper(FixedDistributionPolicy)); {type(search_policy).__name__} is not "
        "supported")


def base_type_tables(model, agent_id, config, other_agent_policies, search_policy):
    """``pomcp_type_policies`` of the base planner with these policies, or None
    when both sides are uniform random (the plain POMCP kernel)."""
    A = model.action_spaces[agent_id].n
    others = [i for i in model.possible_agents if i != agent_id]
    if len(others) != 1:
        raise NotImplementedError("the engine plans for two-agent environments")
    other = other_agent_policies[others[0]]
    sp = search_policy_probs(model, agent_id, search_policy)
    ego_pi = [1.0 / A] * A if sp is None else sp   # RandomSearchPolicy.get_pi
    oth, mixture = [], False
    if _is_random_other(other):
        oth = [[1.0 / A] * A]
    elif isinstance(other, OtherAgentMixturePolicy) or _named(other, "OtherAgentMixturePolicy"):
        mixture = True
        oth = [_fixed_probs(p, A) for p in other.policies.values()]
        if config.state_belief_only:
            # mcts.py:609-610 passes {} and OtherAgentMixturePolicy.sample_action
            # raises KeyError('policy_id') in the reference
            raise ValueError("an OtherAgentMixturePolicy needs state_belief_only=False (the "
                             "particles carry the other agent's policy)")
    else:
        oth = [_fixed_probs(other, A)]
        if not config.state_belief_only:
            # mcts.py:205-210 calls other_agent_policies[j].sample_initial_state(),
            # which a posggym.agents-style policy does not have
            raise ValueError(f"{type(other).__name__} as the other agent's policy needs "
                             "state_belief_only=True (it has no sample_initial_state)")
    if sp is None and _is_random_other(other):
        return None
    if len(oth) > N.POMCP_MAX_TYPE_POLICIES:
        raise NotImplementedError("at most 8 other-agent policies")
    tp = N.PomcpTypePolicies()
    tp.num_ego, tp.num_other = 1, len(oth)
    for a in range(A):
        tp.ego_pi[0][a] = ego_pi[a]
        tp.expected_prior[a] = ego_pi[a]   # the prior of every node: get_pi of the search policy
    for j, pi in enumerate(oth):
        for a in range(A):
            tp.other_pi[j][a] = pi[a]
        tp.meta_len[j] = 1
        tp.meta_policy[j][0] = 0
        tp.meta_weight[j][0] = 1.0
    tp.no_meta_draw = 1
    tp.no_mixture_draw = 0 if mixture else 1
    tp.ego_uniform = 1 if sp is None else 0
    tp.other_uniform = 1 if _is_random_other(other) else 0
    return tp


class MCTS(POMCP):
    """Base multi-agent MCTS planner (``mcts.py:22-91``)."""

    def __init__(self, model, agent_id: str, config: MCTSConfig,
                 other_agent_policies: Dict[str, OtherAgentPolicy], search_policy: SearchPolicy,
                 *, num_sims: Optional[int] = None, process_group=None):
        expected = {i for i in model.possible_agents if i != agent_id}
        if set(other_agent_policies) != expected:
            raise AssertionError(
                f"other_agent_policies must cover agents {sorted(expected)}, "
                f"got {sorted(other_agent_policies)}")
        tables = base_type_tables(model, agent_id, config, other_agent_policies, search_policy)
        engine_cfg = config
        if tables is None:
            # random policies: the plain kernel; histories in the particles would
            # change nothing (module docstring)
            engine_cfg = dataclasses.replace(config, state_belief_only=True)
        self.type_policies = tables
        self._init_planner(model, agent_id, engine_cfg, search_policy, dict(other_agent_policies),
                           num_sims, process_group, type_policies=tables)
        self.config = config

    def root_prior(self, replica: int = 0):
        """The root's ``ObsNode.action_probs`` (fixed-distribution search policy)."""
        if self.type_policies is None:
            n = len(self.action_space)
            return {a: 1.0 / n for a in range(n)}
        return {a: p for a, p in enumerate(self._engine.root_prior(replica))}

    def __str__(self):
        return "MCTS"


class IPOMCP(MCTS):
    """Interactive POMCP with known other-agent policies (``ipomcp.py:11-38``)."""

    def __str__(self):
        return "IPOMCP"
