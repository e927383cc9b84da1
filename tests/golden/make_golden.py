"""Generate the golden fixtures under tests/golden/ (container-only).

Runs the REAL reference planner (``oracle/ref_harness.py``: stub-imported
``posggym_baselines.planning``, injected RNG streams, fake clock) on the build's
Driving-v1 restatement and writes its per-step records.  Every case is also
run through the oracle restatement (``oracle/pomcp.py``) and the script aborts
if the two disagree anywhere, so the committed fixtures pin the oracle.

Usage:  python tests/golden/make_golden.py
"""
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.ref_harness import (  # noqa: E402
    import_reference, reference_available, reference_episode, reference_intmcp_episode,
    reference_mcts_episode, reference_potmmcp_episode)
from oracle.run import oracle_episode, oracle_intmcp_episode  # noqa: E402

SQRT2 = math.sqrt(2)
# tests/planning/test_pomcp.py:38-50 (config 1 of BASELINE.json)
TEST_CFG = dict(discount=0.95, search_time_limit=0.1, c=SQRT2, truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, seed=0, state_belief_only=True)

CASES = {
    # name: (cfg overrides, num_sims, [(planner seed, env seed)], ego, max_steps[, env])
    "c1_ucb": ({}, 128, [(0, 0), (1, 1), (2, 2)], "0", 50),
    "c1_pucb": ({"action_selection": "pucb"}, 128, [(0, 3), (4, 4)], "0", 50),
    "uniform": ({"action_selection": "uniform"}, 64, [(5, 5)], "0", 50),
    "deep_ucb": ({"discount": 0.99, "epsilon": 0.01}, 48, [(6, 2)], "0", 50),
    "known_bounds": ({"known_bounds": (-1.0, 1.0)}, 96, [(7, 7)], "0", 50),
    "ego1_ucb": ({}, 96, [(8, 8)], "1", 50),
    "large_first_step": ({}, 2048, [(9, 9), (10, 10)], "0", 1),
    # BASELINE config 3: PursuitEvasion-v1 (16x16, max_obs_distance 12, progress reward)
    "pe_evader_ucb": ({}, 128, [(11, 11), (12, 12)], "0", 100, "PursuitEvasion-v1"),
    "pe_pursuer_pucb": ({"action_selection": "pucb"}, 96, [(13, 13)], "1", 100,
                        "PursuitEvasion-v1"),
}


# IPOMCP (ipomcp.py:11-38) with random other-agent policies and histories in
# the particles (state_belief_only=False): the reference must produce exactly
# the POMCP oracle's records (the other agents' random policies are stateless)
IPOMCP_CASES = {
    "ipomcp_ucb": ({"state_belief_only": False}, 128, [(20, 20), (21, 21)], "0", 50),
    "ipomcp_pucb_ego1": ({"state_belief_only": False, "action_selection": "pucb"}, 96,
                         [(22, 22)], "1", 50),
}


def run_case(name, cases=CASES, planner_cls="POMCP"):
    over, num_sims, pairs, ego, max_steps = cases[name][:5]
    env = cases[name][5] if len(cases[name]) > 5 else "Driving-v1"
    out = {"case": name, "env": env, "num_sims": num_sims, "ego": ego, "episodes": []}
    if planner_cls != "POMCP":
        out["planner"] = planner_cls
    for seed, env_seed in pairs:
        cfg = dict(TEST_CFG)
        cfg.update(over)
        cfg["seed"] = seed
        tr, rr = reference_episode(cfg, num_sims, env_seed, ego=ego, max_steps=max_steps, env=env,
                                   planner_cls=planner_cls)
        to, ro = oracle_episode(dict(cfg, state_belief_only=True), num_sims, env_seed, ego=ego,
                                max_steps=max_steps, env=env)
        if tr != to or rr != ro:
            raise SystemExit(f"oracle disagrees with reference in case {name} seed {seed}")
        cfg_json = dict(cfg)
        if cfg_json["known_bounds"] is not None:
            cfg_json["known_bounds"] = list(cfg_json["known_bounds"])
        out["episodes"].append({"config": cfg_json, "env_seed": env_seed,
                                "trace": tr, "records": rr})
    return out


# BASELINE config 5: I-NTMCP nesting_level=1 (tests/planning/test_intmcp.py:34-71:
# search_time_limit = 0.1 * (nesting_level + 1), state_belief_only=False); the
# simulation count is per nesting level
INTMCP_CFG = dict(TEST_CFG, search_time_limit=0.2, state_belief_only=False)
INTMCP_CASES = {
    "intmcp_ucb": ({}, 64, [(0, 0), (1, 1)], "0", 50, "Driving-v1"),
    "intmcp_ego1": ({}, 48, [(2, 2)], "1", 50, "Driving-v1"),
    "intmcp_uniform": ({"action_selection": "uniform"}, 32, [(3, 3)], "0", 50, "Driving-v1"),
    "intmcp_deep": ({"discount": 0.99, "epsilon": 0.01}, 16, [(4, 4)], "0", 20, "Driving-v1"),
    "intmcp_pe": ({}, 48, [(5, 5)], "0", 100, "PursuitEvasion-v1"),
}


# I-NTMCP nesting_level=0 (intmcp.py:950-994 with no nested planner: the other
# agent acts by the planner's own self._rng.choice, intmcp.py:750-753);
# search_time_limit = 0.1 * (nesting_level + 1) as tests/planning/test_intmcp.py
INTMCP0_CFG = dict(TEST_CFG, search_time_limit=0.1, state_belief_only=False)
INTMCP0_CASES = {
    "intmcp0_ucb": ({}, 64, [(40, 40), (41, 41)], "0", 50, "Driving-v1"),
    "intmcp0_ego1_uniform": ({"action_selection": "uniform"}, 48, [(42, 42)], "1", 50,
                             "Driving-v1"),
    "intmcp0_deep": ({"discount": 0.99, "epsilon": 0.01}, 16, [(43, 43)], "0", 20, "Driving-v1"),
    "intmcp0_pe": ({}, 48, [(44, 44)], "0", 100, "PursuitEvasion-v1"),
}


# I-NTMCP nesting_level=2: the ego's level-2 tree over the other agent's
# level-1 planner over the ego's level-0 planner (intmcp.py:950-994 recursion,
# _nested_sim dispatch intmcp.py:434-436); search_time_limit = 0.1 * 3
INTMCP2_CFG = dict(TEST_CFG, search_time_limit=0.3, state_belief_only=False)
INTMCP2_CASES = {
    "intmcp2_ucb": ({}, 32, [(60, 60)], "0", 25, "Driving-v1"),
    "intmcp2_ego1_uniform": ({"action_selection": "uniform"}, 24, [(61, 61)], "1", 20,
                             "Driving-v1"),
    "intmcp2_pe": ({}, 24, [(62, 62)], "1", 30, "PursuitEvasion-v1"),
}


# I-NTMCP nesting_level=3: a chain of four planners, the ego's level-3 tree over
# the other agent's level-2, the ego's level-1 and the other agent's level-0
# (the same recursion); search_time_limit = 0.1 * 4
INTMCP3_CFG = dict(TEST_CFG, search_time_limit=0.4, state_belief_only=False)
INTMCP3_CASES = {
    "intmcp3_ucb": ({}, 16, [(70, 70)], "0", 12, "Driving-v1"),
    "intmcp3_pe": ({}, 12, [(71, 71)], "1", 15, "PursuitEvasion-v1"),
}


# I-NTMCP nesting_level=4 and 5: chains of five and six planners (the same
# recursion, intmcp.py:949-994); search_time_limit = 0.1 * (nesting_level + 1).
# Level 5's middle planners of levels 4 draw on the streams past the agents'
# action streams (oracle/intmcp.py belief_stream).
INTMCP4_CFG = dict(TEST_CFG, search_time_limit=0.5, state_belief_only=False)
INTMCP5_CFG = dict(TEST_CFG, search_time_limit=0.6, state_belief_only=False)
INTMCP45_CASES = {
    # name: (nesting level, cfg overrides, num_sims, [(seed, env_seed)], ego, max_steps, env)
    "intmcp4_ucb": (4, {}, 12, [(80, 80)], "0", 8, "Driving-v1"),
    "intmcp4_pe": (4, {}, 10, [(81, 81)], "1", 10, "PursuitEvasion-v1"),
    "intmcp5_ucb": (5, {}, 8, [(82, 82)], "1", 6, "Driving-v1"),
}


# I-NTMCP with caller-supplied search policies (intmcp.py:956-971):
# {level: {agent: probs}} -> SearchPolicyWrapper(FixedDistributionPolicy) on
# the agent's action stream, RandomSearchPolicy for the agents left out.
# (nesting level, search_probs, num_sims, [(seed, env_seed)], ego, max_steps, env)
INTMCP_SP_CASES = {
    "intmcp_sp_ucb": (1, {1: {"0": [0.1, 0.4, 0.2, 0.2, 0.1], "1": [0.5, 0.1, 0.1, 0.2, 0.1]},
                          0: {"1": [0.05, 0.05, 0.3, 0.3, 0.3]}},
                      48, [(50, 50)], "0", 30, "Driving-v1"),
    "intmcp0_sp_ego1": (0, {0: {"1": [0.1, 0.4, 0.2, 0.2, 0.1], "0": [0.3, 0.0, 0.1, 0.5, 0.1]}},
                        48, [(51, 51)], "1", 50, "Driving-v1"),
    "intmcp_sp_pe": (1, {1: {"1": [0.25, 0.25, 0.4, 0.1]},
                         0: {"0": [0.1, 0.2, 0.3, 0.4], "1": [0.7, 0.1, 0.1, 0.1]}},
                     32, [(52, 52)], "1", 100, "PursuitEvasion-v1"),
    "intmcp2_sp_ucb": (2, {2: {"0": [0.1, 0.4, 0.2, 0.2, 0.1]},
                           1: {"0": [0.2, 0.2, 0.2, 0.3, 0.1], "1": [0.5, 0.1, 0.1, 0.2, 0.1]},
                           0: {"1": [0.05, 0.05, 0.3, 0.3, 0.3]}},
                       24, [(66, 66)], "0", 20, "Driving-v1"),
}


def run_intmcp_case(name):
    sp = None
    if name in INTMCP_SP_CASES:
        level, sp, num_sims, pairs, ego, max_steps, env = INTMCP_SP_CASES[name]
        over, base = {}, (INTMCP0_CFG, INTMCP_CFG, INTMCP2_CFG, INTMCP3_CFG)[level]
    elif name in INTMCP45_CASES:
        level, over, num_sims, pairs, ego, max_steps, env = INTMCP45_CASES[name]
        base = INTMCP4_CFG if level == 4 else INTMCP5_CFG
    elif name in INTMCP3_CASES:
        over, num_sims, pairs, ego, max_steps, env = INTMCP3_CASES[name]
        base, level = INTMCP3_CFG, 3
    elif name in INTMCP2_CASES:
        over, num_sims, pairs, ego, max_steps, env = INTMCP2_CASES[name]
        base, level = INTMCP2_CFG, 2
    elif name in INTMCP0_CASES:
        over, num_sims, pairs, ego, max_steps, env = INTMCP0_CASES[name]
        base, level = INTMCP0_CFG, 0
    else:
        over, num_sims, pairs, ego, max_steps, env = INTMCP_CASES[name]
        base, level = INTMCP_CFG, 1
    out = {"case": name, "env": env, "num_sims": num_sims, "ego": ego, "max_steps": max_steps,
           "episodes": []}
    if level != 1:
        out["nesting_level"] = level
    if sp is not None:   # JSON keys are strings: levels as "0" / "1"
        out["search_probs"] = {str(lv): v for lv, v in sp.items()}
    for seed, env_seed in pairs:
        cfg = dict(base)
        cfg.update(over)
        cfg["seed"] = seed
        tr, rr = reference_intmcp_episode(cfg, num_sims, env_seed, ego=ego, max_steps=max_steps,
                                          env=env, nesting_level=level, search_probs=sp)
        to, ro = oracle_intmcp_episode(cfg, num_sims, env_seed, ego=ego, max_steps=max_steps,
                                       env=env, nesting_level=level, search_probs=sp)
        if tr != to or rr != ro:
            raise SystemExit(f"oracle disagrees with reference in case {name} seed {seed}")
        if sp is not None:   # the policies must matter: the random-policy run differs
            _, r0 = oracle_intmcp_episode(cfg, num_sims, env_seed, ego=ego, max_steps=max_steps,
                                          env=env, nesting_level=level)
            if r0 == ro:
                raise SystemExit(f"case {name}: the search policies change no record")
        out["episodes"].append({"config": dict(cfg), "env_seed": env_seed, "trace": tr,
                                "records": rr})
    return out


# POTMMCP (potmmcp.py:18-301) with fixed-distribution policies (planning/
# policies.py): ego policies of the meta-policy, the other agent's mixture
# policies, meta_policy[other][ego] weights (dict order matters: it is
# random.choices' order).  No oracle restatement: the GPU tests compare against
# these reference records directly.
POTMMCP_SPECS = {
    "A": {"ego": {"u": [0.2] * 5, "acc": [0.1, 0.5, 0.1, 0.2, 0.1],
                  "stay": [0.6, 0.1, 0.1, 0.1, 0.1]},
          "other": {"o_u": [0.2] * 5, "o_fast": [0.05, 0.7, 0.05, 0.1, 0.1]},
          "meta": {"o_u": {"u": 0.5, "acc": 0.25, "stay": 0.25}, "o_fast": {"stay": 0.7, "u": 0.3}}},
    # zero-probability actions and a deterministic other-agent policy
    "B": {"ego": {"a": [0.2] * 5, "b": [0.0, 0.0, 0.5, 0.5, 0.0]},
          "other": {"x": [0.3, 0.1, 0.1, 0.4, 0.1], "y": [0.2] * 5, "z": [0.0, 1.0, 0.0, 0.0, 0.0]},
          "meta": {"x": {"b": 1.0}, "y": {"a": 0.5, "b": 0.5}, "z": {"a": 1.0}}},
    "PE": {"ego": {"u": [0.25] * 4, "fw": [0.7, 0.1, 0.1, 0.1]},
           "other": {"u": [0.25] * 4, "side": [0.1, 0.4, 0.4, 0.1]},
           "meta": {"u": {"u": 0.5, "fw": 0.5}, "side": {"fw": 1.0}}},
}
POTMMCP_CFG = dict(TEST_CFG, state_belief_only=False)
POTMMCP_CASES = {
    # name: (cfg overrides, spec, num_sims, [(planner seed, env seed)], ego, max_steps, env)
    "potmmcp_pucb": ({"action_selection": "pucb"}, "A", 64, [(30, 30), (31, 31)], "0", 50,
                     "Driving-v1"),
    "potmmcp_ucb_ego1": ({}, "B", 48, [(32, 32)], "1", 50, "Driving-v1"),
    "potmmcp_pe_pucb": ({"action_selection": "pucb"}, "PE", 48, [(33, 33)], "0", 100,
                        "PursuitEvasion-v1"),
}
# batched trees: the first step of trees 0..5 (keys (seed, k)), one episode each
POTMMCP_TREES = ({"action_selection": "pucb"}, "A", 96, 34, 34, 6)


def run_potmmcp_case(name):
    over, spec, num_sims, pairs, ego, max_steps, env = POTMMCP_CASES[name]
    out = {"case": name, "env": env, "num_sims": num_sims, "ego": ego, "max_steps": max_steps,
           "spec": POTMMCP_SPECS[spec], "episodes": []}
    for seed, env_seed in pairs:
        cfg = dict(POTMMCP_CFG, **over)
        cfg["seed"] = seed
        tr, rr = reference_potmmcp_episode(cfg, num_sims, env_seed, POTMMCP_SPECS[spec], ego=ego,
                                           max_steps=max_steps, env=env)
        out["episodes"].append({"config": dict(cfg), "env_seed": env_seed, "trace": tr,
                                "records": rr})
    return out


def run_potmmcp_trees():
    over, spec, num_sims, seed, env_seed, n = POTMMCP_TREES
    cfg = dict(POTMMCP_CFG, **over)
    cfg["seed"] = seed
    out = {"case": "potmmcp_trees", "env": "Driving-v1", "num_sims": num_sims, "ego": "0",
           "spec": POTMMCP_SPECS[spec], "config": dict(cfg), "env_seed": env_seed, "trees": []}
    for k in range(n):
        tr, rr = reference_potmmcp_episode(cfg, num_sims, env_seed, POTMMCP_SPECS[spec], tree=k,
                                           max_steps=2)
        out["trees"].append({"tree": k, "trace": tr, "records": rr})
    return out


# The base planner (MCTS / IPOMCP / POMCP, mcts.py:22-739) with non-random
# policies (fixed distributions, planning/policies.py): a search policy whose
# prior seeds every node (mcts.py:621-645) and drives the rollouts, other
# agents drawn per particle from a mixture's policy state (mcts.py:602-615).
# No oracle restatement: the GPU tests compare against these reference records.
MCTS_SPECS = {
    "fs": {"search": [0.1, 0.5, 0.1, 0.2, 0.1], "other": {"kind": "random"}},
    "mix": {"search": None,
            "other": {"kind": "mixture", "policies": {"o_u": [0.2] * 5,
                                                      "o_fast": [0.05, 0.7, 0.05, 0.1, 0.1]}}},
    "fs_mix": {"search": [0.0, 0.0, 0.5, 0.5, 0.0],
               "other": {"kind": "mixture", "policies": {"x": [0.3, 0.1, 0.1, 0.4, 0.1],
                                                         "z": [0.0, 1.0, 0.0, 0.0, 0.0],
                                                         "y": [0.2] * 5}}},
    "fixed_other": {"search": [0.6, 0.1, 0.1, 0.1, 0.1],
                    "other": {"kind": "fixed", "probs": [0.3, 0.1, 0.1, 0.4, 0.1]}},
    "pe_fs": {"search": [0.7, 0.1, 0.1, 0.1], "other": {"kind": "random"}},
    "pe_mix": {"search": None,
               "other": {"kind": "mixture", "policies": {"u": [0.25] * 4,
                                                         "side": [0.1, 0.4, 0.4, 0.1]}}},
}
MCTS_CASES = {
    # name: (planner class, cfg overrides, spec, num_sims, [(planner seed, env seed)], ego,
    #        max_steps, env)
    "mcts_pomcp_fs_pucb": ("POMCP", {"action_selection": "pucb"}, "fs", 64, [(40, 40), (41, 41)],
                           "0", 50, "Driving-v1"),
    "mcts_pomcp_fs_ucb": ("POMCP", {}, "fs", 64, [(42, 42)], "0", 50, "Driving-v1"),
    "mcts_ipomcp_mix_pucb": ("IPOMCP", {"action_selection": "pucb", "state_belief_only": False},
                             "mix", 64, [(43, 43), (44, 44)], "0", 50, "Driving-v1"),
    "mcts_ipomcp_fs_mix_ucb_ego1": ("IPOMCP", {"state_belief_only": False}, "fs_mix", 48,
                                    [(45, 45)], "1", 50, "Driving-v1"),
    "mcts_fixed_other_pucb": ("MCTS", {"action_selection": "pucb"}, "fixed_other", 48,
                              [(46, 46)], "0", 50, "Driving-v1"),
    "mcts_pe_fs_ucb": ("POMCP", {}, "pe_fs", 48, [(47, 47)], "0", 100, "PursuitEvasion-v1"),
    "mcts_pe_mix_pucb": ("IPOMCP", {"action_selection": "pucb", "state_belief_only": False},
                         "pe_mix", 48, [(48, 48)], "1", 100, "PursuitEvasion-v1"),
}


def run_mcts_case(name):
    cls, over, spec, num_sims, pairs, ego, max_steps, env = MCTS_CASES[name]
    out = {"case": name, "planner": cls, "env": env, "num_sims": num_sims, "ego": ego,
           "max_steps": max_steps, "spec": MCTS_SPECS[spec], "episodes": []}
    for seed, env_seed in pairs:
        cfg = dict(TEST_CFG, **over)
        cfg["seed"] = seed
        tr, rr = reference_mcts_episode(cfg, num_sims, env_seed, MCTS_SPECS[spec], ego=ego,
                                        max_steps=max_steps, env=env, planner_cls=cls)
        out["episodes"].append({"config": dict(cfg), "env_seed": env_seed, "trace": tr,
                                "records": rr})
    return out


def config_kats():
    """MCTSConfig derived fields (config.py:47-55) from the reference itself."""
    P = import_reference()
    rows = []
    for T in (0.1, 0.5, 1.0, 5.0, 20.0):
        for g, eps in ((0.95, 0.92), (0.99, 0.01), (0.9, 0.5), (0.0, 0.5), (1.0, 0.3)):
            for prop in (1.0 / 16, 0.0, 0.5):
                row = {"search_time_limit": T, "discount": g, "epsilon": eps,
                       "extra_particles_prop": prop}
                try:
                    c = P.MCTSConfig(discount=g, search_time_limit=T, c=1.0, truncated=False,
                                     epsilon=eps, extra_particles_prop=prop)
                    row.update(num_particles=c.num_particles, extra_particles=c.extra_particles,
                               depth_limit=c.depth_limit)
                except Exception as ex:  # e.g. discount == 1.0 -> log(1) == 0
                    row["raises"] = type(ex).__name__
                rows.append(row)
    return rows


def tracker_sequences():
    """Scripted ``step_statistics`` sequences for ``PlanningStatTracker``
    (utils.py:45-144): NaN steps (an absorbing root reports NaN search
    statistics), keys missing from a step (``.get(k, np.nan)``, utils.py:82),
    ``mem_usage`` reduced by max, an empty episode (``reset_episode`` with no
    steps is a no-op, utils.py:98-99) and ``track_overall=False``."""
    nan = float("nan")
    keys = ["search_time", "update_time", "reinvigoration_time", "evaluation_time",
            "policy_calls", "inference_time", "search_depth", "num_sims", "mem_usage",
            "min_value", "max_value"]

    def full(i, j):
        return {k: 0.125 * (i + 1) + 0.01 * j * (n + 1) - (0.3 if k == "min_value" else 0.0)
                for n, k in enumerate(keys)}

    eps = []
    # 1: plain steps
    eps.append([full(0, j) for j in range(4)])
    # 2: a NaN step in the middle (absorbing root) and one with missing keys
    e = [full(1, j) for j in range(5)]
    e[2] = dict(e[2], search_time=nan, num_sims=nan, min_value=nan, max_value=nan)
    e[3] = {"search_time": 0.5, "mem_usage": 7.0, "num_sims": 33.0}
    eps.append(e)
    # 3: empty episode (reset with no steps)
    eps.append([])
    # 4: every step NaN for some keys, mem_usage falling then rising
    e = [dict(full(2, j), mem_usage=m, search_depth=nan) for j, m in enumerate((9.0, 3.0, 12.5))]
    eps.append(e)
    # 5: a single step with only mem_usage
    eps.append([{"mem_usage": 2.0}])
    return eps


def _enc(v):
    """JSON form of a tracker value: hex float, 'nan' or a list of them."""
    import numpy as np
    if isinstance(v, (list, tuple, np.ndarray)):
        return [_enc(x) for x in v]
    v = float(v)
    return "nan" if math.isnan(v) else v.hex()


def planning_stat_tracker():
    """Run the reference ``PlanningStatTracker`` over tracker_sequences():
    get_episode() after every step, get() after every reset_episode()."""
    import_reference()
    from posggym_baselines.planning.utils import PlanningStatTracker

    class _Planner:
        step_statistics = {}

    out = []
    for track_overall in (True, False):
        pl = _Planner()
        tr = PlanningStatTracker(pl, track_overall=track_overall)
        log = {"track_overall": track_overall, "episodes": []}
        for ep in tracker_sequences():
            rec = {"steps": [{k: _enc(v) for k, v in st.items()} for st in ep],
                   "get_episode": [], "get": None}
            for st in ep:
                pl.step_statistics = dict(st)
                tr.step()
                rec["get_episode"].append({k: _enc(v) for k, v in tr.get_episode().items()})
            tr.reset_episode()
            rec["get"] = {k: _enc(v) for k, v in tr.get().items()}
            rec["num_episodes"] = tr._num_episodes
            rec["all_steps"] = list(tr._all_steps)
            log["episodes"].append(rec)
        out.append(log)
    return out


def config_checks():
    """MCTSConfig.__post_init__ assertions and normalisation (config.py:33-45)
    from the reference: which argument sets raise, and the lower-cased
    ``action_selection``."""
    P = import_reference()
    base = dict(discount=0.95, search_time_limit=0.1, c=1.0, truncated=False)
    cases = [
        {}, {"discount": -0.01}, {"discount": 1.01}, {"discount": 0.0}, {"search_time_limit": 0.0},
        {"search_time_limit": -1.0}, {"c": 0.0}, {"c": -1.0}, {"pucb_exploration_fraction": -0.1},
        {"pucb_exploration_fraction": 1.0}, {"pucb_exploration_fraction": 1.1},
        {"extra_particles_prop": 1.5}, {"extra_particles_prop": -0.5}, {"epsilon": 0.0},
        {"epsilon": 1.0}, {"epsilon": 0.999}, {"action_selection": "UCB"},
        {"action_selection": "Uniform"}, {"action_selection": "PUCB"}, {"action_selection": "greedy"},
        {"search_time_limit": 0.001}, {"search_time_limit": 0.015, "extra_particles_prop": 1.0},
    ]
    rows = []
    for over in cases:
        kw = dict(base, **over)
        row = {"kwargs": kw}
        try:
            c = P.MCTSConfig(**kw)
            row.update(action_selection=c.action_selection, num_particles=c.num_particles,
                       extra_particles=c.extra_particles, depth_limit=c.depth_limit)
        except Exception as ex:
            row["raises"] = type(ex).__name__
        rows.append(row)
    return rows


def _write(out_dir, name, data):
    with open(os.path.join(out_dir, f"{name}.json"), "w") as f:
        json.dump(data, f, separators=(",", ":"))


def main(only=None, out_dir=HERE):
    """only: None (every fixture), "ipomcp", "potmmcp", "mcts", "meta" (config +
    tracker fixtures only) or a list of I-NTMCP case names."""
    if not reference_available():
        raise SystemExit("reference not available (container-only script)")
    os.makedirs(out_dir, exist_ok=True)
    for name in CASES if only is None else ():
        data = run_case(name)
        _write(out_dir, name, data)
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    for name in IPOMCP_CASES if only in (None, "ipomcp") else ():
        data = run_case(name, IPOMCP_CASES, "IPOMCP")
        _write(out_dir, name, data)
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    for name in (list(INTMCP_CASES) + list(INTMCP0_CASES) + list(INTMCP2_CASES)
                 + list(INTMCP3_CASES) + list(INTMCP45_CASES) + list(INTMCP_SP_CASES) if only is None
                 else (only if isinstance(only, list) else ())):
        data = run_intmcp_case(name)
        _write(out_dir, name, data)
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    for name in POTMMCP_CASES if only in (None, "potmmcp") else ():
        data = run_potmmcp_case(name)
        _write(out_dir, name, data)
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    if only in (None, "potmmcp"):
        _write(out_dir, "potmmcp_trees", run_potmmcp_trees())
        print("potmmcp_trees written")
    for name in MCTS_CASES if only in (None, "mcts") else ():
        data = run_mcts_case(name)
        _write(out_dir, name, data)
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    if only in (None, "meta"):
        _write(out_dir, "config_kats", config_kats())
        _write(out_dir, "config_checks", config_checks())
        _write(out_dir, "planning_stat_tracker", planning_stat_tracker())
        print("config_kats, config_checks, planning_stat_tracker written")


if __name__ == "__main__":
    # --out DIR: write there instead of tests/golden/ (the CPU test regenerates
    # into a temporary directory and compares byte for byte);
    # --ipomcp: only the IPOMCP fixtures; --meta: only the config / tracker
    # fixtures; --intmcp NAME...: only the named I-NTMCP fixtures
    argv = list(sys.argv[1:])
    out = HERE
    if "--out" in argv:
        i = argv.index("--out")
        out = argv[i + 1]
        del argv[i:i + 2]
    if "--ipomcp" in argv:
        main(only="ipomcp", out_dir=out)
    elif "--potmmcp" in argv:
        main(only="potmmcp", out_dir=out)
    elif "--mcts" in argv:
        main(only="mcts", out_dir=out)
    elif "--meta" in argv:
        main(only="meta", out_dir=out)
    elif "--intmcp" in argv:
        main(only=argv[argv.index("--intmcp") + 1:], out_dir=out)
    else:
        main(out_dir=out)
