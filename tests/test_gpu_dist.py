"""Root-parallel POMCP across ranks on real hardware (BASELINE config 4's code
path): two processes on one GPU, ``POMCP(...,
process_group=WORLD)`` with K replicas each.  Rank r's replicas take keys
(seed, r*K .. r*K+K-1); one all-reduce of the [K][A][2] merge buffer per
get_action (gloo here: the box has one GPU; the bench uses nccl = RCCL), then
the device merge.  Both ranks must play the same actions, and those must equal
the CPU restatement over the 2K oracle replicas (oracle/root_parallel.py) bit
for bit."""
import math
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

K, SIMS, STEPS, ENV_SEED = 4, 64, 4, 321
CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, seed=17, state_belief_only=True)


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpu_util import product_config, product_model
    from oracle.episode import run_episode
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    model = product_model("Driving-v1")
    config = product_config(CFG, SIMS * K)
    config.root_parallel = K
    planner = POMCP(model, "0", config, RandomSearchPolicy(model, "0"),
                    process_group=dist.group.WORLD)
    planner.reset()
    recs = []

    def step(obs):
        a = planner.step(obs)
        if not planner.root.is_absorbing:
            recs.append((int(a), [float(x) for x in planner.root.child_visits],
                         [float(x).hex() for x in planner.root.child_totals]))
        return a

    run_episode(step, ENV_SEED, max_steps=STEPS)
    planner.close()
    out[rank] = recs
    dist.barrier()
    dist.destroy_process_group()


def _oracle():
    """2K oracle replicas; the merge sums each replica index over the ranks
    first (the all-reduce), then the K indices in k_merge_roots' order."""
    from oracle.episode import run_episode
    from oracle.root_parallel import merge_roots
    from oracle.run import make_oracle
    reps = [make_oracle(CFG, SIMS, tree=t) for t in range(2 * K)]
    recs, last = [], [None]

    def step(obs):
        if all(p.on_abs[p.root] for p in reps):
            return last[0]
        for p in reps:
            p.stats = {"searched": True}
            p.update(last[0], obs)
        if all(p.on_abs[p.root] for p in reps):
            last[0] = 0
            return 0
        for p in reps:
            p.get_action()
        z = [0] * 5
        vis = [[a + b for a, b in zip(reps[k].stats.get("child_visits", z),
                                      reps[K + k].stats.get("child_visits", z))] for k in range(K)]
        tot = [[a + b for a, b in zip(reps[k].stats.get("child_totals", z),
                                      reps[K + k].stats.get("child_totals", z))] for k in range(K)]
        a, sv, st = merge_roots(vis, tot, CFG["action_selection"])
        recs.append((a, [float(x) for x in sv], [float(x).hex() for x in st]))
        last[0] = a
        return a

    run_episode(step, ENV_SEED, max_steps=STEPS)
    return recs


def test_root_parallel_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True,
                           start_method="spawn")
        res = dict(out)
    assert res[0] == res[1]
    assert len(res[0]) >= 2
    assert res[0] == _oracle()
