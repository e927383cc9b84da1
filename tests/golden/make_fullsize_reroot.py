"""Generate tests/golden/fullsize_reroot.json (container-only).

Full-size re-root parity (BASELINE configs 2 and 3 at their benchmarked size):
3-step episodes at num_sims = 65,536 -- the initial update, then two re-roots
of a 65,536-simulation tree (mcts.py:229-263: the chosen child's subtree kept,
its particles the new root belief, mcts.py:651-700 reinvigoration) -- for two
planners per environment (Driving-v1 ego "0", PursuitEvasion-v1 ego "1").

Every episode is run twice: by the oracle restatement (oracle/pomcp.py) and by
the REAL reference planner (oracle/ref_harness.py: stub-imported, injected
RNG, fake clock); the script aborts unless the two agree record for record, so
the fixture is the reference's own output at the benchmarked size.  The oracle
run also counts, before each re-root, the particle records of the kept
subtree's cut-off nodes (the children beyond the depth limit, which the lane
kernel defers to the re-root's k_compact_log): the test asserts there are more
than one materialisation chunk's worth of them.

Usage:  python tests/golden/make_fullsize_reroot.py   (about 2 minutes on 8 cores)
"""
import json
import math
import os
import sys
from multiprocessing import get_context

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

SQRT2 = math.sqrt(2)
TEST_CFG = dict(discount=0.95, search_time_limit=0.1, c=SQRT2, truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, seed=0, state_belief_only=True)
NUM_SIMS = 65536
STEPS = 3
# env -> (ego, [env seeds]); tree b of the engine = planner b (oracle Streams tree b)
CASES = {"Driving-v1": ("0", [1000, 1001]), "PursuitEvasion-v1": ("1", [2000, 2001])}


def kept_cutoff_records(p, action, obs):
    """Particle records of the cut-off nodes (relative depth depth_limit) under
    the child (action, obs) of the oracle's root, i.e. the deferred records the
    re-root keeps and materialises."""
    root = p.root
    b = p.on_block[root]
    if b < 0 or action is None:
        return 0
    child = p.children.get((b * p.A + action, p.model.pack_obs(obs)))
    if child is None:
        return 0
    by_an = {}
    for (an, _), c in p.children.items():
        by_an.setdefault(an, []).append(c)
    level, n = [child], 0
    for _ in range(p.cfg.depth_limit):
        nxt = []
        for node in level:
            blk = p.on_block[node]
            if blk < 0:
                continue
            for a in range(p.A):
                nxt.extend(by_an.get(blk * p.A + a, ()))
        level = nxt
    for node in level:
        n += len(p.belief[node])
    return n


def run_oracle(job):
    from oracle.episode import run_episode
    from oracle.run import make_oracle, oracle_record
    env, ego, seed, tree = job
    p = make_oracle(TEST_CFG, NUM_SIMS, ego=ego, tree=tree, env=env)
    records, kept = [], []

    def step(obs):
        searched = not p.on_abs[p.root]
        if p.on_t[p.root] > 0:
            kept.append(kept_cutoff_records(p, p.last_action, obs))
        a = p.step(obs)
        records.append(oracle_record(p, searched, a))
        return a

    trace = run_episode(step, seed, ego=ego, max_steps=STEPS, env=env)
    return trace, records, kept


def run_reference(job):
    from oracle.ref_harness import reference_episode
    env, ego, seed, tree = job
    return reference_episode(TEST_CFG, NUM_SIMS, seed, ego=ego, tree=tree, max_steps=STEPS,
                             env=env)


def main(out=os.path.join(HERE, "fullsize_reroot.json")):
    from oracle.ref_harness import reference_available
    if not reference_available():
        raise SystemExit("reference not available (container-only script)")
    jobs = [(env, ego, s, tree) for env, (ego, seeds) in CASES.items()
            for tree, s in enumerate(seeds)]
    with get_context("fork").Pool(min(8, 2 * len(jobs))) as pool:
        ro = pool.map_async(run_oracle, jobs)
        rr = pool.map_async(run_reference, jobs)
        oracle_out, ref_out = ro.get(), rr.get()
    data = {"num_sims": NUM_SIMS, "steps": STEPS, "config": TEST_CFG, "cases": []}
    for job, (to, rec_o, kept), (tr, rec_r) in zip(jobs, oracle_out, ref_out):
        env, ego, seed, tree = job
        if to != tr or rec_o != rec_r:
            raise SystemExit(f"oracle disagrees with the reference: {job}")
        if tr["len"] < STEPS or not all(r["searched"] and r.get("num_sims") for r in rec_r):
            raise SystemExit(f"episode {job} ends before {STEPS} searched steps: pick another seed")
        data["cases"].append({"env": env, "ego": ego, "env_seed": seed, "tree": tree,
                              "trace": tr, "records": rec_r, "kept_cutoff_records": kept})
        print(env, ego, seed, [r["belief_size"] for r in rec_r], "kept cut-off records", kept)
    with open(out, "w") as f:
        json.dump(data, f, separators=(",", ":"))


if __name__ == "__main__":
    main(*sys.argv[1:2])
