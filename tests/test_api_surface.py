"""The drop-in exports the reference's planning API (``planning/__init__.py:1-18``)
and rejects what is out of the GPU engine's scope loudly; no GPU needed."""
from types import SimpleNamespace

import pytest

import posggym_baselines_amd.planning as P

# every name the reference's posggym_baselines/planning/__init__.py exports
REFERENCE_EXPORTS = ["MCTSConfig", "INTMCP", "IPOMCP", "MCTS", "OtherAgentMixturePolicy",
                     "OtherAgentPolicy", "RandomOtherAgentPolicy", "POMCP", "POTMMCP",
                     "POTMMCPMetaPolicy", "PPOLSTMSearchPolicy", "RandomSearchPolicy",
                     "SearchPolicy", "SearchPolicyWrapper", "load_posggym_agents_search_policy"]


def test_reference_exports_exist():
    for name in REFERENCE_EXPORTS:
        assert hasattr(P, name), name


class _Pi:
    """A posggym.agents-like policy with a fixed action distribution."""

    def __init__(self, probs):
        self.probs = probs

    def get_initial_state(self):
        return {}

    def get_next_state(self, action, obs, state):
        return {}

    def get_pi(self, state):
        return SimpleNamespace(probs=self.probs)


def test_potmmcp_meta_policy_expected_action_probs():
    from posggym_baselines_amd.envs import DrivingModel
    m = DrivingModel()
    pols = {"a": _Pi({0: 1.0, 1: 0.0, 2: 0.0, 3: 0.0, 4: 0.0}),
            "b": _Pi({0: 0.0, 1: 0.5, 2: 0.5, 3: 0.0, 4: 0.0})}
    meta = P.POTMMCPMetaPolicy(m, "0", pols, {"x": {"a": 1.0}, "y": {"a": 0.5, "b": 0.5}})
    probs = meta.get_expected_action_probs(None, meta.get_initial_state())
    assert probs == pytest.approx({0: 0.75, 1: 0.125, 2: 0.125, 3: 0.0, 4: 0.0})
    with pytest.raises(NotImplementedError):
        meta.sample_action({})
    with pytest.raises(NotImplementedError):   # history-dependent / neural policies
        P.POTMMCP(m, "0", None, {}, meta)


def test_neural_policies_rejected():
    with pytest.raises(NotImplementedError):
        P.load_posggym_agents_search_policy(None, "0", "PPO")
    with pytest.raises(NotImplementedError):
        P.PPOLSTMSearchPolicy(None, "0", "PPO")
