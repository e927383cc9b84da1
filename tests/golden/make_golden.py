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
    import_reference, reference_available, reference_episode, reference_intmcp_episode)
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
},
                        16, [(2, 2)], "0", 50, "Driving-v1"),
    "intmcp_depleted_pe": ({"extra_particles_prop": 1.0,
                            "reinvigoration_sample_limit_factor": 0.45, "action_selection": "uniform"},
                           16, [(5, 5)], "1", 100, "PursuitEvasion-v1"),
}


def run_intmcp_case(name):
    over, num_sims, pairs, ego, max_steps, env = INTMCP_CASES[name]
    out = {"case": name, "env": env, "num_sims": num_sims, "ego": ego, "max_steps": max_steps,
           "episodes": []}
    for seed, env_seed in pairs:
        cfg = dict(INTMCP_CFG)
        cfg.update(over)
        cfg["seed"] = seed
        tr, rr = reference_intmcp_episode(cfg, num_sims, env_seed, ego=ego, max_steps=max_steps,
                                          env=env)
        to, ro = oracle_intmcp_episode(cfg, num_sims, env_seed, ego=ego, max_steps=max_steps,
                                       env=env)
        if tr != to or rr != ro:
            raise SystemExit(f"oracle disagrees with reference in case {name} seed {seed}")
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


def main(only=None):
    if not reference_available():
        raise SystemExit("reference not available (container-only script)")
    for name in CASES if only is None else ():
        data = run_case(name)
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    for name in IPOMCP_CASES if only in (None, "ipomcp") else ():
        data = run_case(name, IPOMCP_CASES, "IPOMCP")
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    for name in INTMCP_CASES if only is None else (only if isinstance(only, list) else ()):
        data = run_intmcp_case(name)
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        n = sum(len(e["records"]) for e in data["episodes"])
        print(f"{name}: {len(data['episodes'])} episodes, {n} records")
    if only is None:
        with open(os.path.join(HERE, "config_kats.json"), "w") as f:
            json.dump(config_kats(), f, separators=(",", ":"))
        print("config_kats written")


if __name__ == "__main__":
    # --ipomcp: (re)generate only the IPOMCP fixtures; --intmcp NAME...: only
    # the named I-NTMCP fixtures
    if "--ipomcp" in sys.argv:
        main(only="ipomcp")
    elif "--intmcp" in sys.argv:
        main(only=sys.argv[sys.argv.index("--intmcp") + 1:])
    else:
        main()
