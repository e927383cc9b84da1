"""Per-pair digests of oracle I-NTMCP episodes for the GPU suite's batched tests.

The GPU tests run hundreds of planner pairs in one engine and must compare
EVERY pair with the oracle (oracle/intmcp.py, itself pinned to the real
reference by tests/golden/intmcp_*.json).  Running the pure-Python oracle for
all of them inside the GPU session would take minutes, so this script runs it
here, on all host cores, and commits one SHA-1 per pair of that pair's step
records (oracle/run.py oracle_intmcp_episode, canonical JSON).  The GPU tests
hash their own records the same way (`record_digest`) and, on a mismatch, rerun
the oracle for that pair to show the difference; `tests/test_oracle.py` checks
a sample of the digests against the oracle on the CPU.

    python tests/golden/make_oracle_digests.py      (writes oracle_digests.json)
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for _p in (ROOT, os.path.join(ROOT, "posggym-baselines_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

OUT = os.path.join(HERE, "oracle_digests.json")

BASE_CFG = dict(discount=0.95, search_time_limit=0.1, c=2 ** 0.5, truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, seed=3, state_belief_only=False)

# name -> workload: env, ego, selection, pairs (tree key b, env seed seed0 + b),
# simulations per level, real steps (tests/test_gpu_intmcp.py)
CASES = {
    "im_drv_ucb_48": dict(env="Driving-v1", ego="0", sel="ucb", pairs=1100, seed0=500,
                          sims=48, steps=4),
    "im_pe_uniform_48": dict(env="PursuitEvasion-v1", ego="1", sel="uniform", pairs=150,
                             seed0=500, sims=48, steps=4),
    "im_drv_ucb_256": dict(env="Driving-v1", ego="0", sel="ucb", pairs=130, seed0=900,
                           sims=256, steps=3),
    "im_pe_ucb_256": dict(env="PursuitEvasion-v1", ego="0", sel="ucb", pairs=130, seed0=900,
                          sims=256, steps=3),
}


def record_digest(records) -> str:
    """SHA-1 of a pair's step records in canonical JSON (numpy scalars as ints)."""
    txt = json.dumps(records, sort_keys=True, separators=(",", ":"), default=int)
    return hashlib.sha1(txt.encode()).hexdigest()


def case_cfg(case):
    return dict(BASE_CFG, action_selection=case["sel"])


def oracle_pair(case, b):
    from oracle.run import oracle_intmcp_episode
    _, recs = oracle_intmcp_episode(case_cfg(case), case["sims"], case["seed0"] + b,
                                    ego=case["ego"], tree=b, max_steps=case["steps"],
                                    env=case["env"])
    return recs


def _job(arg):
    name, b = arg
    return name, b, record_digest(oracle_pair(CASES[name], b))


def main():
    jobs = [(n, b) for n, c in CASES.items() for b in range(c["pairs"])]
    out = {n: dict(c, digests=[None] * c["pairs"]) for n, c in CASES.items()}
    with mp.get_context("fork").Pool(os.cpu_count() or 1) as pool:
        for n, b, d in pool.imap_unordered(_job, jobs, chunksize=8):
            out[n]["digests"][b] = d
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", OUT, {n: len(c["digests"]) for n, c in out.items()})


if __name__ == "__main__":
    main()
