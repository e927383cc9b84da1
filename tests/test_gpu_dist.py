"""Root-parallel POMCP across ranks on real hardware (BASELINE config 4's code
path): 2 and 4 processes on one GPU, ``POMCP(...,
process_group=WORLD)`` with K replicas each.  Rank r's replicas take keys
(seed, r*K .. r*K+K-1) and search ceil(num_sims / (world K)) simulations each;
one all-gather of the [K][R] exchange records per get_action (gloo here: the
box has one GPU; the bench uses nccl = RCCL), then the device merge of the
world x K replicas in replica order.  Every rank must play the same actions,
and those must equal the CPU merge of the world x K oracle replicas
(oracle/root_parallel.py) bit for bit -- for 4 ranks as for 2.  A replica
arena overflow on one rank must raise on every rank (no rank left waiting in
a collective)."""
import math
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

K, SIMS, STEPS, ENV_SEED = 4, 64, 4, 321
CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, seed=17, state_belief_only=True)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpu_util import product_config, product_model
    from oracle.episode import run_episode
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    model = product_model("Driving-v1")
    config = product_config(CFG, SIMS * K * world)
    config.root_parallel = K
    planner = POMCP(model, "0", config, RandomSearchPolicy(model, "0"),
                    process_group=dist.group.WORLD)
    planner.reset()
    recs = []

    def step(obs):
        a = planner.step(obs)
        if not planner.root.is_absorbing:
            st = planner.step_statistics
            recs.append((int(a), [float(x) for x in planner.root.child_visits],
                         [float(x).hex() for x in planner.root.child_totals],
                         int(st["num_sims"]), int(planner.root.visits),
                         float(st["min_value"]).hex(), float(st["max_value"]).hex()))
        return a

    run_episode(step, ENV_SEED, max_steps=STEPS)
    planner.close()
    out[rank] = recs
    dist.barrier()
    dist.destroy_process_group()


def _oracle(world):
    """world x K oracle replicas (keys 0 .. world K - 1, rank-major), merged in
    replica order as k_merge_roots does after the all-gather."""
    from oracle.episode import fhex, run_episode
    from oracle.root_parallel import OracleRootParallel
    from oracle.run import make_oracle
    reps = [make_oracle(CFG, SIMS, tree=t) for t in range(world * K)]
    orc = OracleRootParallel(reps, CFG["action_selection"])
    recs = []

    def step(obs):
        was_abs = orc.absorbing()
        a = orc.step(obs)
        if not was_abs and orc.merged is not None:
            _, sv, st = orc.merged
            live = [p for p in reps if "child_visits" in p.stats]
            recs.append((a, [float(x) for x in sv], [float(x).hex() for x in st],
                         SIMS * world * K,
                         sum(p.stats["root_visits"] for p in live),
                         fhex(min(p.stats["min_value"] for p in live)),
                         fhex(max(p.stats["max_value"] for p in live))))
        return a

    run_episode(step, ENV_SEED, max_steps=STEPS)
    return recs


@pytest.mark.parametrize("world", [2, 4])
def test_root_parallel_ranks_one_gpu(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_worker, args=(world, _port(), out), nprocs=world, join=True,
                           start_method="spawn")
        res = dict(out)
    for r in range(1, world):
        assert res[r] == res[0]
    assert len(res[0]) >= 2
    exp = _oracle(world)
    assert [r[:3] for r in res[0]] == [e[:3] for e in exp]    # actions, merged visits / totals
    assert res[0] == exp                                     # + step statistics over all ranks


def _arena_worker(rank, world, port, out):
    """Rank 1's engine gets a 2-block arena: its search overflows (POMCP_E_ARENA)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpu_util import product_config, product_model
    from oracle.episode import run_episode
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    from posggym_baselines_amd.planning import engine as E
    if rank == 1:
        plan = E.plan_capacities

        def tiny(*a, **kw):
            caps = plan(*a, **kw)
            caps.max_blocks = 2
            return caps
        E.plan_capacities = tiny
    model = product_model("Driving-v1")
    config = product_config(CFG, SIMS * K * world)
    config.root_parallel = K
    planner = POMCP(model, "0", config, RandomSearchPolicy(model, "0"),
                    process_group=dist.group.WORLD)
    planner.reset()
    try:
        run_episode(planner.step, ENV_SEED, max_steps=STEPS)
        out[rank] = "ok"
    except Exception as e:  # noqa: BLE001
        out[rank] = type(e).__name__ + ": " + str(e)[:200]
    dist.barrier()   # reached by both ranks: neither is stuck in a collective
    planner.close()
    dist.destroy_process_group()


def test_arena_error_on_one_rank_raises_on_every_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_arena_worker, args=(2, _port(), out), nprocs=2, join=True,
                           start_method="spawn")
        res = dict(out)
    assert res[0] != "ok" and res[1] != "ok", res
    assert "ARENA" in res[0] and "ARENA" in res[1], res
