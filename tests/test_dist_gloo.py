"""Root-parallel exchange across ranks on the CPU (gloo), world_size 2 and 4.

Rank r holds the exchange records (include/pomcp.h POMCP_XREC) of its K
replicas j = r*K + k -- the oracle planner under tree key j, as
``POMCP(..., process_group=...)`` keys them.  The product exchange
(``parallel.gather_records``, an all-gather) must leave every rank the same
rank-major [world][K][R] buffer, so that the fixed-order merge
(``pomcp_merge_roots``; ``oracle/root_parallel.py``) of the world x K replicas is
identical on every rank and equal to one process merging all of them -- which
an all-reduce of FP64 totals could not guarantee beyond two ranks.  Failure
agreement (``parallel.raise_together``): a failing rank makes every rank raise,
in ``update`` and in ``get_action``, instead of leaving its peers waiting in a
collective.
"""
import math
import os
import socket
from types import SimpleNamespace

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
S, A = 48, 5
R = 2 * A + 6


def replica_record(j, sel):
    """Exchange record of replica j: the oracle's first search under tree key j."""
    _, p = oracle_first_step(dict(CFG, action_selection=sel), S, j, 1000)
    st = p.stats
    rec = np.zeros(R)
    rec[0:2 * A:2] = st["child_visits"]
    rec[1:2 * A:2] = st["child_totals"]
    rec[2 * A:] = [st["num_sims"], st["root_visits"], st["search_depth"], 0,
                   st["min_value"], st["max_value"]]
    return rec


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _gather_worker(rank, world, port, K, recs, out):
    _init(rank, world, port)
    from posggym_baselines_amd.planning.parallel import gather_records
    local = torch.tensor(np.concatenate(recs[rank * K:(rank + 1) * K]))
    buf = torch.zeros(world * K * R, dtype=torch.float64)
    gather_records(local, buf)
    g = buf.numpy().reshape(world * K, R)
    a, sv, st = merge_roots(g[:, 0:2 * A:2].tolist(), g[:, 1:2 * A:2].tolist(), out["sel"])
    out[rank] = (buf.numpy().view(np.uint64).tolist(), a, sv, [x.hex() for x in st])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,K,sel", [(2, 3, "ucb"), (4, 2, "ucb"), (4, 2, "pucb")])
def test_allgather_exchange_is_rank_order_and_merge_is_identical(world, K, sel):
    recs = [replica_record(j, sel) for j in range(world * K)]
    with mp.Manager() as mgr:
        out = mgr.dict()
        out["sel"] = sel
        mp.spawn(_gather_worker, args=(world, _port(), K, recs, out), nprocs=world, join=True)
        res = {r: out[r] for r in range(world)}
    expected = np.concatenate(recs).view(np.uint64).tolist()
    a, sv, st = merge_roots([r[0:2 * A:2].tolist() for r in recs],
                            [r[1:2 * A:2].tolist() for r in recs], sel)
    for r in range(world):
        assert res[r][0] == expected              # every rank: the same rank-major buffer
        assert res[r][1:] == (a, sv, [x.hex() for x in st])
    # the replicas really searched differently (independent keys)
    assert len({tuple(r[1:2 * A:2]) for r in recs}) > 1


class _FakeEngine:
    """Enough of PomcpEngine for the drop-in's update / get_action host logic."""

    def __init__(self, fail_update=False, fail_search=False):
        self.fail_update, self.fail_search = fail_update, fail_search
        self.wall_clock_sims = None
        self.type_based = False

    def root_stats(self):   # (the search's work counters: none here)
        return []

    def update(self, actions, keys):
        if self.fail_update:
            raise RuntimeError("update failed: POMCP_E_ARENA")
        return np.zeros(1, dtype=bool)

    def search(self, n, fetch=True, final=True):
        if self.fail_search:
            raise RuntimeError("search failed: POMCP_E_HIP")


def _planner(rank, fail_update, fail_search):
    from posggym_baselines_amd.planning.pomcp import POMCP, RootView
    p = POMCP.__new__(POMCP)
    p._world, p._rank, p._pg, p._K = 2, rank, None, 1
    p._num_sims, p._per_replica = 8, 4
    p.config = SimpleNamespace(device=0, search_time_limit=0.1)
    p.root = RootView(t=1)
    p._emodel = SimpleNamespace(obs_key=lambda o: 0)
    p._engine = _FakeEngine(fail_update, fail_search)
    p.step_statistics = {}
    p.action_space = list(range(A))
    p._last_action = 0
    return p


def _failure_worker(rank, world, port, what, out):
    _init(rank, world, port)
    from posggym_baselines_amd.planning.parallel import PeerFailure
    p = _planner(rank, what == "update" and rank == 1, what == "search" and rank == 1)
    try:
        if what == "update":
            p.update(0, None)
        else:
            p.get_action()
        out[rank] = "ok"
    except PeerFailure:
        out[rank] = "peer"
    except RuntimeError as e:
        out[rank] = "own:" + str(e)
    dist.barrier()   # both ranks got here: nobody is stuck in a collective
    dist.destroy_process_group()


@pytest.mark.parametrize("what", ["update", "search"])
def test_failure_on_one_rank_raises_on_every_rank(what):
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_failure_worker, args=(2, _port(), what, out), nprocs=2, join=True)
        res = dict(out)
    assert res[0] == "peer"
    assert res[1].startswith("own:")


def _small_worker(rank, world, port, out):
    _init(rank, world, port)
    from posggym_baselines_amd.planning.parallel import allgather_small, raise_together
    out[rank] = allgather_small([rank, 10.0 * rank + 0.5]).tolist()
    rows = raise_together(None, [rank + 1])
    out[("rows", rank)] = rows.tolist()
    dist.barrier()
    dist.destroy_process_group()


def test_allgather_small_rows_in_rank_order():
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_small_worker, args=(3, _port(), out), nprocs=3, join=True)
        res = dict(out)
    for r in range(3):
        assert res[r] == [[0.0, 0.5], [1.0, 10.5], [2.0, 20.5]]
        assert res[("rows", r)] == [[0.0, 1.0], [0.0, 2.0], [0.0, 3.0]]


def test_merge_rule_ties_and_unvisited():
    vis = [[0, 3, 3, 1, 0]]
    tot = [[0.0, 3.0, 3.0, 5.0, 0.0]]
    assert merge_roots(vis, tot, "pucb")[0] == 1
    assert merge_roots(vis, tot, "ucb")[0] == 3
    assert merge_roots([[0] * 5], [[0.0] * 5], "pucb")[0] == 0
    assert merge_roots([[0] * 5], [[0.0] * 5], "ucb")[0] == 0
