"""Helpers to load the committed golden fixtures (tests/golden/*.json)."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EPISODE_CASES = ["c1_ucb", "c1_pucb", "uniform", "deep_ucb", "known_bounds", "ego1_ucb",
                 "large_first_step", "pe_evader_ucb", "pe_pursuer_pucb"]


def case_env(data):
    return data.get("env", "Driving-v1")


def case_max_steps(case, data):
    if case == "large_first_step":
        return 1
    return 100 if case_env(data) == "PursuitEvasion-v1" else 50


def load(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


def cfg_kwargs(cfg):
    kw = dict(cfg)
    if kw.get("known_bounds") is not None:
        kw["known_bounds"] = tuple(kw["known_bounds"])
    return kw


# reference IPOMCP (ipomcp.py:11-38), random other agents, state_belief_only=False:
# the same records as POMCP (tests/golden/make_golden.py IPOMCP_CASES)
IPOMCP_CASES = ["ipomcp_ucb", "ipomcp_pucb_ego1"]

INTMCP_CASES = ["intmcp_ucb", "intmcp_ego1", "intmcp_uniform", "intmcp_deep", "intmcp_pe"]

# I-NTMCP nesting_level=0 (tests/golden/make_golden.py INTMCP0_CASES): a single
# level-0 tree whose other agent acts uniformly (intmcp.py:750-753)
INTMCP0_CASES = ["intmcp0_ucb", "intmcp0_ego1_uniform", "intmcp0_deep", "intmcp0_pe"]

# I-NTMCP with fixed-distribution search policies (make_golden.py INTMCP_SP_CASES)
INTMCP_SP_CASES = ["intmcp_sp_ucb", "intmcp0_sp_ego1", "intmcp_sp_pe", "intmcp2_sp_ucb"]

# I-NTMCP nesting_level=2 (make_golden.py INTMCP2_CASES): three trees
INTMCP2_CASES = ["intmcp2_ucb", "intmcp2_ego1_uniform", "intmcp2_pe"]

# I-NTMCP nesting_level=3 (make_golden.py INTMCP3_CASES): four trees
INTMCP3_CASES = ["intmcp3_ucb", "intmcp3_pe"]

# I-NTMCP nesting_level=4 / 5 (make_golden.py INTMCP45_CASES): five / six trees
INTMCP45_CASES = ["intmcp4_ucb", "intmcp4_pe", "intmcp5_ucb"]


def search_probs(data):
    """A golden's {level: {agent: probs}} with integer levels (None if absent)."""
    sp = data.get("search_probs")
    return None if sp is None else {int(lv): v for lv, v in sp.items()}
