"""Debug: arena use around updates with small arenas (run on the GPU box)."""
import math
import sys
sys.path[:0] = ["/root/repo", "/root/repo/posggym-baselines_amd", "/root/repo/tests"]
import numpy as np
from gpu_util import _arena_usage, product_config
from oracle.driving import DrivingModel as EnvModel, pack_obs
from oracle.episode import ENV_TREE_BASE
from oracle.rng import S_ENV_POLICY_BASE, Streams
from posggym_baselines_amd.envs import DrivingModel
from posggym_baselines_amd.planning import BatchedPOMCP, MCTSConfig
from posggym_baselines_amd.planning.engine import plan_capacities

CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, seed=0, state_belief_only=True)
S, steps, B = 64, 8, int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = MCTSConfig(num_sims=S, **CFG)
caps = plan_capacities(cfg, 50, S, 8, num_actions=5, overflow_slots=64)
print("caps", caps)
bp = BatchedPOMCP(DrivingModel(), "0", product_config(CFG, S), B, S, searches=steps, reroot=True,
                  capacities=caps)
envs = []
for s in range(7000, 7000 + B):
    es = Streams(s, ENV_TREE_BASE)
    env = EnvModel(es)
    st = env.sample_initial_state()
    envs.append([es, env, st, env.sample_initial_obs(st)])
last = np.full(B, -1, dtype=np.int32)
for t in range(steps):
    keys = np.array([pack_obs(e[3]["0"]) for e in envs], dtype=np.uint64)
    u0 = _arena_usage(bp.engine)
    bp.engine.update(last, keys)
    u1 = _arena_usage(bp.engine)
    actions = bp.search()
    st = bp.engine.root_stats()
    print(t, "before", u0, "after", u1, "post-search tree0 blocks/log", st[0].n_blocks, st[0].n_log,
          "max", max(s.n_blocks for s in st), max(s.n_log for s in st),
          "root visits", st[0].root_visits, flush=True)
    for b in range(B):
        es, env, s_, obs = envs[b]
        acts = {"0": int(actions[b]), "1": es.randint(S_ENV_POLICY_BASE + 1, 5)}
        ts = env.step(s_, acts)
        envs[b][2], envs[b][3] = ts.state, ts.observations
    last = actions.astype(np.int32)
