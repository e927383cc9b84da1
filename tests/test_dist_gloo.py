"""Root-parallel exchange on world_size 2 (gloo, CPU): each rank's per-root
(visits, total value) come from the oracle with that rank's search key
(seed ^ rank << 32, as bench.py / pomcp_rekey do on the GPU); the all-reduce
+ merged argmax of posggym_baselines_amd.planning.parallel must equal a CPU
merge of the same oracle runs."""
import math
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.run import oracle_first_step

CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, seed=0, state_belief_only=True)
B, S, A = 3, 48, 5


def rank_stats(rank):
    m = np.zeros((B, A, 2))
    for b in range(B):
        rec, p = oracle_first_step(CFG, S, b, 1000 + b, rekey=CFG["seed"] ^ (rank << 32))
        m[b, :, 0] = p.stats["child_visits"]
        m[b, :, 1] = p.stats["child_totals"]
    return m


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from posggym_baselines_amd.planning.parallel import root_parallel_merge
    merge = torch.tensor(rank_stats(rank).reshape(-1))
    actions = root_parallel_merge(merge, A, world)
    out[rank] = (actions.tolist(), merge.tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_root_parallel_merge_world2():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    total = rank_stats(0) + rank_stats(1)
    vis, tot = total[..., 0], total[..., 1]
    with np.errstate(invalid="ignore", divide="ignore"):
        val = np.where(vis > 0, tot / np.maximum(vis, 1), -np.inf)
    expected = np.argmax(val, axis=-1).tolist()
    assert res[0][0] == res[1][0] == expected
    assert np.allclose(res[0][1], total.reshape(-1))
    # ranks really searched differently (independent keys)
    assert not np.array_equal(rank_stats(0), rank_stats(1))
