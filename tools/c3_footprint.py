"""Per-tree footprint of the C3 update()-inclusive workload (bench.py
run_pomcp(update_step=True)): one search of 65,536 simulations from the
synthetic PursuitEvasion-v1 / Driving-v1 roots, the environment's answer and
update(); prints the distribution of the re-rooted belief sizes, blocks and log
records in use before / after the re-root (sizes the arenas)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "posggym-baselines_amd"))


def probe(env, B=1024, S=65536, seed=0):
    import math
    from posggym_baselines_amd.envs import DrivingModel, PursuitEvasionModel
    from posggym_baselines_amd.planning import BatchedPOMCP, MCTSConfig
    from posggym_baselines_amd.planning.engine import plan_capacities
    cfg = MCTSConfig(seed=seed, num_sims=S, discount=0.95, search_time_limit=0.1, c=math.sqrt(2),
                     truncated=False, action_selection="ucb", epsilon=0.92)
    model = PursuitEvasionModel() if env == "PursuitEvasion-v1" else DrivingModel()
    caps = plan_capacities(cfg, model.spec.max_episode_steps, S, 1, reroot=True, max_blocks=512,
                           overflow_slots=1024, num_actions=model.action_spaces["0"].n)
    bp = BatchedPOMCP(model, "0", cfg, B, S, capacities=caps)
    bp.init_synthetic(1000)
    acts = bp.search()
    st = bp.engine.root_stats()
    blocks = np.array([s.n_blocks for s in st])
    logs = np.array([s.n_log for s in st])
    bp.engine.update(acts, bp.engine.synthetic_step(1000, acts))
    bp.engine.search(1, fetch=False)
    st = bp.engine.root_stats()
    bel = np.array([s.belief_size for s in st])
    blocks2 = np.array([s.n_blocks for s in st])
    bp.close()
    q = lambda a: {k: int(v) for k, v in zip(("min", "p50", "p99", "max"),
                                              np.percentile(a, [0, 50, 99, 100]))}
    print(env, "B", B, "S", S, "caps", caps, flush=True)
    print("  blocks after search", q(blocks), " log records", q(logs))
    print("  re-rooted belief", q(bel), " blocks after re-root + 1 sim", q(blocks2), flush=True)


if __name__ == "__main__":
    for env in (sys.argv[1:] or ["PursuitEvasion-v1", "Driving-v1"]):
        probe(env)
