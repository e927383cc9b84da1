"""Debug: a wall-clock (search_time_limit=1.0) Driving-v1 episode, printing per
step the simulations, arena headroom and usage (run on the GPU box).
usage: POMCP_SEARCH_KERNEL=wave python tools/dbg/wallclock_wave.py"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd"), os.path.join(ROOT, "tests")]
from gpu_util import product_model  # noqa: E402
from oracle.episode import run_episode  # noqa: E402
from posggym_baselines_amd.planning import MCTSConfig, POMCP, RandomSearchPolicy  # noqa: E402

TEST_CFG = dict(discount=0.95, search_time_limit=1.0, c=math.sqrt(2), truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, seed=0, state_belief_only=True)
model = product_model("Driving-v1")
planner = POMCP(model, "0", MCTSConfig(**TEST_CFG), RandomSearchPolicy(model, "0"))
planner.reset()
eng = planner._engine
print("kernel", eng.search_kernel(), "caps", eng.capacities, "ceiling", eng.wall_clock_sims, flush=True)


def step(obs):
    a = planner.step(obs)
    st = planner.step_statistics
    import ctypes as C
    nb, nl = C.c_int32(), C.c_int32()
    eng._lib.pomcp_arena_usage(eng._ctx, C.byref(nb), C.byref(nl))
    print("t", planner.root.t, "sims", st.get("num_sims"), "full", st.get("arena_full"),
          "time %.3f" % st.get("search_time", 0), "blocks", nb.value, "log", nl.value,
          "room", eng.headroom(), flush=True)
    return a


run_episode(step, 31, max_steps=50)
planner.close()
