"""Non-neural ``posggym.agents``-style policies the engine can run on the GPU.

POTMMCP (``potmmcp.py:18-301``) searches with a meta-policy over the ego's
policies and models the other agent as a mixture over its policies
(``other_policy.py:155-216``).  The reference's experiments plug in
posggym.agents networks; the engine takes policies whose action distribution
does not depend on the history -- a fixed distribution per policy (uniform
included) -- so that every simulation's policy draws, rollouts and node priors
run in the search kernel.  ``FixedDistributionPolicy`` has the interface the
reference calls on a ``posggym.agents.policy.Policy``: ``policy_id``,
``get_initial_state``, ``get_next_state``, ``get_pi(state).probs``,
``sample_action``, ``get_value``, ``close``.

``sample_action`` draws like ``random.choices(range(n), weights=probs)``
(CPython's cumulative-weight bisection) on ``self.rng``; the engine makes the
same draw on the acting agent's action stream (stream 8 + agent index), one
32-bit word per action.
"""
import random
from typing import Dict, Sequence


class ActionDistribution:
    """``posggym.agents.utils.action_distributions.DiscreteActionDistribution``-like:
    ``probs`` is a fresh ``{action: probability}`` dict in action order."""

    def __init__(self, probs: Dict[int, float]):
        self.probs = probs


class FixedDistributionPolicy:
    """A stateless policy with a fixed action distribution."""

    def __init__(self, model, agent_id: str, policy_id: str, probs: Sequence[float],
                 rng=None):
        n = model.action_spaces[agent_id].n
        probs = [float(p) for p in probs]
        if len(probs) != n:
            raise ValueError(f"{policy_id}: {len(probs)} probabilities for {n} actions")
        if any(p < 0.0 for p in probs) or not sum(probs) > 0.0:
            raise ValueError(f"{policy_id}: probabilities must be >= 0 with a positive sum")
        self.model = model
        self.agent_id = agent_id
        self.policy_id = policy_id
        self.probs = probs
        self.rng = rng if rng is not None else random.Random()

    @classmethod
    def uniform(cls, model, agent_id: str, policy_id: str = "uniform", rng=None):
        n = model.action_spaces[agent_id].n
        return cls(model, agent_id, policy_id, [1.0 / n] * n, rng)

    def get_initial_state(self):
        return {}

    def get_next_state(self, action, obs, state):
        return {}

    def get_pi(self, state) -> ActionDistribution:
        return ActionDistribution({a: p for a, p in enumerate(self.probs)})

    def sample_action(self, state) -> int:
        return self.rng.choices(range(len(self.probs)), weights=self.probs, k=1)[0]

    def get_value(self, state) -> float:
        raise NotImplementedError(f"{self.policy_id} has no value estimates")

    def close(self):
        pass


def cumulative(weights: Sequence[float]):
    """``random.choices``' cumulative weights (``itertools.accumulate``) and its
    ``total = cum_weights[-1] + 0.0``: the exact doubles the device bisects."""
    cum, acc = [], None
    for w in weights:
        acc = float(w) if acc is None else acc + float(w)
        cum.append(acc)
    return cum, cum[-1] + 0.0
