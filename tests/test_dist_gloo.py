"""Root-parallel exchange on world_size 2 (gloo, CPU): each rank's per-root
(visits, total value) come from the oracle with that rank's search key
(seed ^ rank << 32, as bench.py / pomcp_rekey do on the GPU); the all-reduce
+ merged argmax of posggym_baselines_amd.planning.parallel must equal a CPU
merge of the same oracle runs."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.root_parallel import merge_roots
from oracle.run import oracle_first_step

CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, seed=0, state_belief_only=True)
B, S, A = 3, 48, 5


def rank_stats(rank, sel="ucb"):
    m = np.zeros((B, A, 2))
    for b in range(B):
        rec, p = oracle_first_step(dict(CFG, action_selection=sel), S, b, 1000 + b,
                                   rekey=CFG["seed"] ^ (rank << 32))
        m[b, :, 0] = p.stats["child_visits"]
        m[b, :, 1] = p.stats["child_totals"]
    return m


def _worker(rank, world, port, sel, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from posggym_baselines_amd.planning.parallel import root_parallel_merge
    merge = torch.tensor(rank_stats(rank, sel).reshape(-1))
    actions = root_parallel_merge(merge, A, world, sel)
    out[rank] = (actions.tolist(), merge.tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sel", ["ucb", "pucb"])
def test_root_parallel_merge_world2(sel):
    """The merged rule follows the planner's final selection: summed visits
    for PUCB (mcts.py:565-581), summed total / visits otherwise (583-600); it
    equals the device merge's CPU restatement (oracle/root_parallel.py)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, port, sel, out), nprocs=2, join=True)
        res = dict(out)
    r0, r1 = rank_stats(0, sel), rank_stats(1, sel)
    total = r0 + r1
    expected = [merge_roots([total[b, :, 0]], [total[b, :, 1]], sel)[0] for b in range(B)]
    assert res[0][0] == res[1][0] == expected
    assert np.array_equal(np.array(res[0][1]), total.reshape(-1))
    # ranks really searched differently (independent keys)
    assert not np.array_equal(r0, r1)


def test_merge_rule_ties_and_unvisited():
    from posggym_baselines_amd.planning.parallel import root_parallel_merge
    m = torch.tensor([[[0, 0.0], [3, 3.0], [3, 3.0], [1, 5.0], [0, 0.0]],
                      [[0, 0.0]] * 5], dtype=torch.float64)
    assert root_parallel_merge(m.clone().reshape(-1), 5, 1, "pucb").tolist() == [1, 0]
    assert root_parallel_merge(m.clone().reshape(-1), 5, 1, "ucb").tolist() == [3, 0]
    for sel, exp in (("pucb", 1), ("ucb", 3)):
        assert merge_roots([m[0, :, 0].tolist()], [m[0, :, 1].tolist()], sel)[0] == exp
        assert merge_roots([m[1, :, 0].tolist()], [m[1, :, 1].tolist()], sel)[0] == 0
