"""GPU parity of the base planner with non-random policies (SURVEY §8(a) a6,
a11, a17; mcts.py:22-739, ipomcp.py:11-38, pomcp.py:9-35): a fixed-distribution
search policy (node priors mcts.py:621-645, the child-side moving average
mcts.py:358-367, rollouts mcts.py:405-452) and other agents drawn per particle
from an ``OtherAgentMixturePolicy`` or a stateless fixed-distribution policy
(mcts.py:602-615).  Every step record of the reference goldens
(tests/golden/mcts_*.json, made by the real reference MCTS / IPOMCP / POMCP:
root statistics, the root's action_probs, the root belief with each particle's
other-agent policy) must match bit for bit."""
import pytest

from golden_util import load
from oracle.episode import run_episode
from test_gpu_potmmcp import _record

pytestmark = pytest.mark.gpu

MCTS_CASES = ["mcts_pomcp_fs_pucb", "mcts_pomcp_fs_ucb", "mcts_ipomcp_mix_pucb",
              "mcts_ipomcp_fs_mix_ucb_ego1", "mcts_fixed_other_pucb", "mcts_pe_fs_ucb",
              "mcts_pe_mix_pucb"]


def make_planner(data, cfg, model):
    """The drop-in planner of a golden case, built from the build's policies."""
    from gpu_util import product_config
    from posggym_baselines_amd.planning import (IPOMCP, MCTS, POMCP, OtherAgentMixturePolicy,
                                                RandomOtherAgentPolicy, RandomSearchPolicy)
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
    from posggym_baselines_amd.planning.search_policy import SearchPolicyWrapper
    ego, spec = data["ego"], data["spec"]
    other = [i for i in model.possible_agents if i != ego][0]
    if spec["search"] is None:
        search = RandomSearchPolicy(model, ego)
    else:
        search = SearchPolicyWrapper(FixedDistributionPolicy(model, ego, "search", spec["search"]))
    o = spec["other"]
    if o["kind"] == "random":
        others = {other: RandomOtherAgentPolicy(model, other)}
    elif o["kind"] == "fixed":
        others = {other: FixedDistributionPolicy(model, other, "fixed", o["probs"])}
    else:
        others = {other: OtherAgentMixturePolicy(
            model, other, {k: FixedDistributionPolicy(model, other, k, v)
                           for k, v in o["policies"].items()})}
    config = product_config(cfg, data["num_sims"])
    if data["planner"] == "POMCP":
        return POMCP(model, ego, config, search)
    return {"MCTS": MCTS, "IPOMCP": IPOMCP}[data["planner"]](model, ego, config, others, search)


@pytest.mark.parametrize("case", MCTS_CASES)
def test_gpu_base_planner_policies_match_reference_goldens(case):
    from gpu_util import product_model
    data = load(case)
    ego = data["ego"]
    for ep in data["episodes"]:
        model = product_model(data["env"])
        planner = make_planner(data, ep["config"], model)
        assert planner.type_policies is not None   # the type-based kernel runs it
        planner.reset()
        A = model.action_spaces[ego].n
        records = []

        def step(obs):
            searched = not planner.root.is_absorbing
            a = planner.step(obs)
            if not searched:
                records.append({"searched": False, "action": int(a)})
            else:
                records.append(_record(planner, planner._engine, 0, A, a,
                                       planner.step_statistics["num_sims"]))
            return a

        trace = run_episode(step, ep["env_seed"], ego=ego, max_steps=data["max_steps"],
                            env=data["env"])
        planner.close()
        assert len(records) == len(ep["records"]), case
        for t, (got, exp) in enumerate(zip(records, ep["records"])):
            assert got == exp, f"{case} env_seed {ep['env_seed']} step {t}"
        assert trace == ep["trace"]
