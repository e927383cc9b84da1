"""Per-step update / search times of a wall-clock INTMCP (or, with `pomcp` as
the second argument, POMCP) episode (diagnostics):
    python tools/dbg/wallclock_times.py TIME_LIMIT [pomcp|intmcp] [MAX_STEPS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd"), os.path.join(ROOT, "tests")]


def main():
    import torch
    torch.cuda.init()
    from gpu_util import product_model
    from oracle.episode import run_episode
    from posggym_baselines_amd.planning import INTMCP, MCTSConfig, POMCP, RandomSearchPolicy
    from test_gpu_intmcp import TEST_CFG
    tl = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
    pomcp = len(sys.argv) > 2 and sys.argv[2] == "pomcp"
    model = product_model("Driving-v1")
    t0 = time.time()
    cfg = MCTSConfig(**dict(TEST_CFG, search_time_limit=tl, state_belief_only=pomcp))
    planner = (POMCP(model, "0", cfg, RandomSearchPolicy(model, "0")) if pomcp
               else INTMCP.initialize(model, "0", cfg, 1, None))
    t1 = time.time()
    planner.reset()
    print(f"init {t1 - t0:.2f} s, reset {time.time() - t1:.2f} s", flush=True)

    def step(obs):
        t = time.time()
        a = planner.step(obs)
        st = planner.step_statistics
        extra = "" if pomcp else (f" nodes {list(planner._engine.root_stats()[0].n_nodes)} log "
                                  f"{list(planner._engine.root_stats()[0].n_log)}")
        print(f"step {time.time() - t:.2f} s: update {st['update_time']:.3f} search "
              f"{st['search_time']:.3f} sims {st['num_sims']} arena_full "
              f"{st.get('arena_full')}" + extra, flush=True)
        return a

    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    run_episode(step, 41, max_steps=steps)
    planner.close()


if __name__ == "__main__":
    main()
