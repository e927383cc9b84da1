"""I-NTMCP time per nesting level (diagnostics; run on the GPU box).

One get_action of `--sims` simulations per level on `--pairs` synthetic
Driving-v1 pairs, launched as the level-0 simulations (the other agent's
tree) and then the level-1 simulations (the ego's tree, which also steps the
other agent's history through the level-0 tree), each timed separately.

    python tools/intmcp_levels.py [--pairs B --sims S]
"""
import argparse
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=16384)
    ap.add_argument("--sims", type=int, default=256)
    ap.add_argument("--arena", default=None, help="NODES,STATS,LOG per tree (default worst case)")
    args = ap.parse_args()
    import torch
    torch.cuda.init()   # before the engine's library touches HIP
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import BatchedINTMCP, MCTSConfig
    from posggym_baselines_amd.planning.intmcp import plan_intmcp_capacities
    cfg = MCTSConfig(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
                     action_selection="ucb", epsilon=0.92, seed=0, state_belief_only=False,
                     num_sims=args.sims)
    model = DrivingModel()
    caps = plan_intmcp_capacities(cfg, 50, args.sims, 3, 5)
    if args.arena:
        caps.max_nodes, caps.max_stats, caps.max_log = (int(x) for x in args.arena.split(","))
        caps.hash_slots = 1 << max(4, (2 * caps.max_nodes - 1).bit_length())
    print("capacities", caps, flush=True)
    bp = BatchedINTMCP(model, "0", cfg, args.pairs, args.sims, capacities=caps)
    bp.init_synthetic(1000)
    eng = bp.engine
    sync = torch.cuda.synchronize   # (root_stats() copies per pair: too slow to time with)
    for rep in range(2):
        sync()
        t0 = time.perf_counter()
        eng.search_levels(args.sims, 0, N.INTMCP_BEGIN)
        sync()
        t1 = time.perf_counter()
        eng.search_levels(0, args.sims, N.INTMCP_FINAL)
        sync()
        t2 = time.perf_counter()
        n = args.pairs * args.sims
        print(f"rep {rep}: level 0 {1e3 * (t1 - t0):.1f} ms ({n / (t1 - t0) / 1e6:.0f} M sims/s), "
              f"level 1 {1e3 * (t2 - t1):.1f} ms ({n / (t2 - t1) / 1e6:.0f} M sims/s)", flush=True)
        if rep == 0:
            bp.close()
            bp = BatchedINTMCP(model, "0", cfg, args.pairs, args.sims, capacities=caps)
            bp.init_synthetic(1000)
            eng = bp.engine
    bp.close()


if __name__ == "__main__":
    main()
