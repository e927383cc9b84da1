"""POTMMCP host side (no GPU): the fixed-distribution policy's draw is the
engine's (random.choices over the policy's cumulative weights on its agent's
action stream), the policy tables handed to pomcp_set_type_policies follow the
dicts' order, the meta-policy's expected prior equals the reference's bit for
bit, and unsupported setups raise before any device work."""
import pytest

from golden_util import load


def _model():
    from posggym_baselines_amd.envs import DrivingModel
    return DrivingModel()


def test_fixed_policy_draw_is_choices_over_cumulative_weights():
    from oracle.rng import S_ACT_BASE, StreamRandom, Streams
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy, cumulative
    probs = [0.05, 0.7, 0.05, 0.1, 0.1]
    s1, s2 = Streams(5, 3), Streams(5, 3)
    pol = FixedDistributionPolicy(_model(), "1", "fast", probs, StreamRandom(s1, S_ACT_BASE + 1))
    cum, total = cumulative(probs)
    for _ in range(2000):
        u = s2.u32(S_ACT_BASE + 1)
        x = u * (1.0 / 4294967296.0) * total
        exp = next((i for i in range(len(probs) - 1) if x < cum[i]), len(probs) - 1)
        assert pol.sample_action({}) == exp
    assert pol.get_pi({}).probs == dict(enumerate(probs))
    with pytest.raises(NotImplementedError):
        pol.get_value({})


def _planner_parts(spec, ego="0"):
    from posggym_baselines_amd.planning import OtherAgentMixturePolicy, POTMMCPMetaPolicy
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
    m = _model()
    other = "1" if ego == "0" else "0"
    ego_p = {k: FixedDistributionPolicy(m, ego, k, v) for k, v in spec["ego"].items()}
    oth_p = {k: FixedDistributionPolicy(m, other, k, v) for k, v in spec["other"].items()}
    return m, POTMMCPMetaPolicy(m, ego, ego_p, spec["meta"]), OtherAgentMixturePolicy(m, other, oth_p)


def test_type_policy_tables_follow_dict_order():
    from posggym_baselines_amd.planning.potmmcp import type_policy_tables
    spec = load("potmmcp_ucb_ego1")["spec"]
    m, meta, mix = _planner_parts(spec, ego="1")
    tp = type_policy_tables(m, "1", meta, mix)
    ego_ids, oth_ids = list(spec["ego"]), list(spec["other"])
    assert (tp.num_ego, tp.num_other) == (len(ego_ids), len(oth_ids))
    for k, e in enumerate(ego_ids):
        assert list(tp.ego_pi[k][:5]) == spec["ego"][e]
    for j, o in enumerate(oth_ids):
        assert list(tp.other_pi[j][:5]) == spec["other"][o]
        row = spec["meta"][o]
        assert tp.meta_len[j] == len(row)
        assert [tp.meta_policy[j][i] for i in range(len(row))] == [ego_ids.index(e) for e in row]
        assert [tp.meta_weight[j][i] for i in range(len(row))] == list(row.values())
    exp = meta.get_expected_action_probs(None, meta.get_initial_state())
    assert list(tp.expected_prior[:5]) == [exp[a] for a in range(5)]


@pytest.mark.parametrize("case", ["potmmcp_pucb", "potmmcp_ucb_ego1"])
def test_expected_prior_equals_reference(case):
    """potmmcp.py:391-431 restated in planning/potmmcp.py: the same doubles as
    the reference meta-policy (container only: needs /root/reference)."""
    from oracle.ref_harness import import_reference, potmmcp_policies, reference_available
    if not reference_available():
        pytest.skip("reference not available")
    P = import_reference()
    data = load(case)
    ego = data["ego"]
    m, meta, _ = _planner_parts(data["spec"], ego=ego)
    from oracle.envs import make_model
    from oracle.rng import Streams
    rm = make_model("Driving-v1", Streams(0, 0))
    ego_pols, _, rmeta = potmmcp_policies(rm, ego, data["spec"])
    ref = P.POTMMCPMetaPolicy(rm, ego, ego_pols, rmeta)
    exp = ref.get_expected_action_probs(None, ref.get_initial_state())
    got = meta.get_expected_action_probs(None, meta.get_initial_state())
    assert list(got.values()) == list(exp.values())
    assert list(got) == list(exp)


def test_potmmcp_rejects_before_device_work():
    from posggym_baselines_amd.planning import MCTSConfig, POTMMCP, RandomOtherAgentPolicy
    spec = load("potmmcp_pucb")["spec"]
    m, meta, mix = _planner_parts(spec)
    cfg = MCTSConfig(discount=0.95, search_time_limit=0.1, c=1.4, truncated=False,
                     action_selection="pucb", epsilon=0.92, seed=0, state_belief_only=True,
                     num_sims=16)
    with pytest.raises(ValueError):          # particles must carry the other's policy
        POTMMCP(m, "0", cfg, {"1": mix}, meta)
    with pytest.raises(NotImplementedError):  # the other agent must be a mixture
        POTMMCP(m, "0", cfg, {"1": RandomOtherAgentPolicy(m, "1")}, meta)

    class Recurrent:   # a history-dependent (e.g. network) policy
        policy_id = "rnn"
    meta.policies["rnn"] = Recurrent()
    with pytest.raises(NotImplementedError):
        POTMMCP(m, "0", cfg, {"1": mix}, meta)


def test_base_planner_type_tables():
    """MCTS / IPOMCP / POMCP with fixed-distribution policies (planning/ipomcp.py
    base_type_tables): one ego policy (the search policy, no sample_policy
    draw), the node prior = its get_pi, the other agent's policies and draw
    kinds; random policies on both sides stay on the plain kernel; the
    reference's own failures (mixture with state_belief_only=True, a stateless
    policy with state_belief_only=False) are raised up front."""
    import pytest
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import (MCTSConfig, OtherAgentMixturePolicy,
                                                RandomOtherAgentPolicy, RandomSearchPolicy)
    from posggym_baselines_amd.planning.ipomcp import base_type_tables
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
    from posggym_baselines_amd.planning.search_policy import SearchPolicyWrapper
    m = DrivingModel()
    cfg = MCTSConfig(discount=0.95, search_time_limit=0.1, c=1.4, truncated=False, seed=0,
                     state_belief_only=True)
    cfg_h = MCTSConfig(discount=0.95, search_time_limit=0.1, c=1.4, truncated=False, seed=0,
                       state_belief_only=False)
    fs = SearchPolicyWrapper(FixedDistributionPolicy(m, "0", "s", [0.1, 0.5, 0.1, 0.2, 0.1]))
    rnd_o = {"1": RandomOtherAgentPolicy(m, "1")}
    assert base_type_tables(m, "0", cfg, rnd_o, RandomSearchPolicy(m, "0")) is None
    tp = base_type_tables(m, "0", cfg, rnd_o, fs)
    assert (tp.num_ego, tp.num_other, tp.no_meta_draw, tp.no_mixture_draw, tp.ego_uniform,
            tp.other_uniform) == (1, 1, 1, 1, 0, 1)
    assert list(tp.ego_pi[0])[:5] == list(tp.expected_prior)[:5] == [0.1, 0.5, 0.1, 0.2, 0.1]
    mix = OtherAgentMixturePolicy(m, "1", {"a": FixedDistributionPolicy(m, "1", "a", [0.2] * 5),
                                           "b": FixedDistributionPolicy(m, "1", "b",
                                                                        [0, 1, 0, 0, 0])})
    tp = base_type_tables(m, "0", cfg_h, {"1": mix}, RandomSearchPolicy(m, "0"))
    assert (tp.num_other, tp.no_mixture_draw, tp.ego_uniform, tp.other_uniform) == (2, 0, 1, 0)
    assert list(tp.ego_pi[0])[:5] == [1.0 / 5] * 5 and list(tp.other_pi[1])[:5] == [0, 1, 0, 0, 0]
    with pytest.raises(ValueError):
        base_type_tables(m, "0", cfg, {"1": mix}, fs)
    fixed = {"1": FixedDistributionPolicy(m, "1", "f", [0.3, 0.1, 0.1, 0.4, 0.1])}
    tp = base_type_tables(m, "0", cfg, fixed, RandomSearchPolicy(m, "0"))
    assert (tp.no_mixture_draw, tp.other_uniform, list(tp.other_pi[0])[:5]) == \
        (1, 0, [0.3, 0.1, 0.1, 0.4, 0.1])
    with pytest.raises(ValueError):
        base_type_tables(m, "0", cfg_h, fixed, fs)
