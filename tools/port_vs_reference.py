"""Re-measure the CPU baseline's tie to the real reference:
the oracle port (oracle/pomcp.py, the bench's cpu_baseline) and the real
reference planner (stub-imported from /root/reference, oracle/ref_harness.py)
timed on the same workload on one core each -- get_action of `--sims`
simulations on the synthetic roots of bench.py (env seed 1000 + b) -- and the
chosen actions checked equal.  Writes profiles/port_vs_reference.json, which
bench.py reports beside its cpu_baseline (the reference cannot run on the GPU
box).  Container-only (needs /root/reference):

    python tools/port_vs_reference.py [--sims 8192 --trees 4 --out PATH]
"""
import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, state_belief_only=True, seed=0)


def _cpu_name():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def time_port(sims, b):
    from oracle.episode import run_episode
    from oracle.run import make_oracle
    p = make_oracle(CFG, sims, tree=b)
    out = {}

    def step(obs):
        p.update(None, obs)
        t0 = time.perf_counter()
        out["a"] = p.get_action()
        out["t"] = time.perf_counter() - t0
        return out["a"]

    run_episode(step, 1000 + b, max_steps=1)
    return out["t"], out["a"]


def time_reference(sims, b):
    from oracle.envs import make_model
    from oracle.episode import run_episode
    from oracle.ref_harness import make_reference_pomcp
    from oracle.rng import Streams
    streams = Streams(CFG["seed"], b)
    model = make_model("Driving-v1", streams)
    p = make_reference_pomcp(model, "0", CFG, sims, streams)
    p.reset()
    out = {}

    def step(obs):
        p.update(None, obs)
        t0 = time.perf_counter()
        out["a"] = p.get_action()
        out["t"] = time.perf_counter() - t0
        return out["a"]

    run_episode(step, 1000 + b, max_steps=1)
    p.close()
    return out["t"], out["a"]


def measure(sims, trees):
    from oracle.ref_harness import reference_available
    if not reference_available():
        raise SystemExit("the reference is not available here (container-only)")
    tp = tr = 0.0
    for b in range(trees):
        t, a = time_port(sims, b)
        u, r = time_reference(sims, b)
        if a != r:
            raise SystemExit(f"root {b}: port chose {a}, reference {r}")
        tp, tr = tp + t, tr + u
    port, ref = sims * trees / tp, sims * trees / tr
    return {"port_sims_per_s": port, "reference_sims_per_s": ref,
            "port_vs_reference_speed": port / ref, "sims": sims, "trees": trees, "cores": 1,
            "workload": "get_action only, Driving-v1 synthetic roots (env seed 1000+b), "
                        "ucb c=sqrt2 gamma=0.95 depth_limit=2, one process",
            "cpu": _cpu_name(), "python": platform.python_version(),
            "measured": time.strftime("%Y-%m-%d %H:%M:%S")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sims", type=int, default=8192)
    ap.add_argument("--trees", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "port_vs_reference.json"))
    a = ap.parse_args()
    r = measure(a.sims, a.trees)
    if a.out != "-":
        with open(a.out, "w") as f:
            json.dump(r, f, indent=1)
            f.write("\n")
    print(json.dumps(r))


if __name__ == "__main__":
    main()
