"""Root parallelisation on one GPU (BASELINE config 2 as one
planner): K replica trees of ONE planner, merged on the device.

* every replica is the exact oracle planner with RNG key (seed, k), fed the
  merged action and the real observation (oracle/root_parallel.py);
* the device merge (pomcp_merge_roots) equals the CPU restatement bit for bit;
* the merge buffer (the operand of the cross-GPU all-gather) equals the root
  statistics it is built from, and the merge over a gathered buffer of any
  rank count follows the replica order.
"""
import math

import numpy as np
import pytest

from gpu_util import product_config, product_model

pytestmark = pytest.mark.gpu

CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, seed=11, state_belief_only=True)


def _replica_record(st, A):
    from oracle.episode import fhex
    return (int(st.num_sims), int(st.root_visits), [int(x) for x in st.child_visits[:A]],
            [fhex(x) for x in st.child_values[:A]], [fhex(x) for x in st.child_totals[:A]],
            fhex(st.min_value), fhex(st.max_value), int(st.search_depth))


def _oracle_replica_record(p):
    from oracle.episode import fhex
    s = p.stats
    return (int(s["num_sims"]), int(s["root_visits"]), list(s["child_visits"]),
            [fhex(x) for x in s["child_values"]], [fhex(x) for x in s["child_totals"]],
            fhex(s["min_value"]), fhex(s["max_value"]), int(s["search_depth"]))


@pytest.mark.parametrize("env,sel,K,sims,ego", [("Driving-v1", "ucb", 8, 128, "0"),
                                                 ("Driving-v1", "pucb", 70, 700, "0"),
                                                 ("PursuitEvasion-v1", "uniform", 12, 240, "1")])
def test_root_parallel_planner_matches_oracle_replicas(env, sel, K, sims, ego):
    from oracle.episode import fhex, run_episode
    from oracle.root_parallel import OracleRootParallel, per_replica_sims
    from oracle.run import make_oracle
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    cfg = dict(CFG, action_selection=sel)
    model = product_model(env)
    A = model.action_spaces[ego].n
    config = product_config(cfg, sims)
    config.root_parallel = K
    planner = POMCP(model, ego, config, RandomSearchPolicy(model, ego))
    planner.reset()
    per = per_replica_sims(sims, K)
    orc = OracleRootParallel([make_oracle(cfg, per, ego=ego, tree=k, env=env) for k in range(K)],
                             sel)
    steps = []

    def step(obs):
        searched = not planner.root.is_absorbing
        a = planner.step(obs)
        b = orc.step(obs)
        assert a == b, (len(steps), a, b)
        if searched and orc.merged is not None:
            eng = planner._engine
            st = eng.root_stats()
            for k in range(K):
                if orc.planners[k].on_abs[orc.planners[k].root]:
                    assert st[k].root_absorbing
                    continue
                assert _replica_record(st[k], A) == _oracle_replica_record(orc.planners[k]), \
                    (len(steps), k)
            _, sv, stt = orc.merged
            assert list(planner.root.child_visits) == [int(v) for v in sv]
            assert [fhex(x) for x in planner.root.child_totals] == [fhex(x) for x in stt]
            assert planner.step_statistics["num_sims"] == per * K
        steps.append(a)
        return a

    run_episode(step, 4242, ego=ego, max_steps=6, env=env)
    assert len(steps) >= 2
    planner.close()


def _records(bp, A):
    """The merge buffer as [trees][xrec(A)] and the root stats it must equal."""
    import torch
    from posggym_baselines_amd.planning.parallel import merge_buffer_tensor
    B = bp.num_trees
    st = bp.engine.root_stats()   # synchronises the engine's stream first
    buf = merge_buffer_tensor(bp.engine, torch.device("cuda:0")).cpu().numpy().reshape(B, -1)
    return buf, st


@pytest.mark.parametrize("sel", ["ucb", "pucb"])
def test_device_merge_equals_cpu_merge_and_merge_buffer_equals_root_stats(sel):
    from oracle.root_parallel import merge_roots
    from posggym_baselines_amd.planning import BatchedPOMCP
    model = product_model("Driving-v1")
    B, S, group = 4160, 64, 1040      # 4 planners x 1040 replicas (uneven 64-lane chunks)
    bp = BatchedPOMCP(model, "0", product_config(dict(CFG, action_selection=sel), S), B, S)
    bp.init_synthetic(77)
    bp.search(fetch=False)
    A = 5
    buf, st = _records(bp, A)
    assert buf.shape == (B, 2 * A + 6)
    vis = np.array([list(s.child_visits[:A]) for s in st], dtype=np.float64)
    tot = np.array([list(s.child_totals[:A]) for s in st], dtype=np.float64)
    assert np.array_equal(buf[:, 0:2 * A:2], vis)
    assert np.array_equal(buf[:, 1:2 * A:2].view(np.uint64), tot.view(np.uint64))
    stats = np.array([[s.num_sims, s.root_visits, s.search_depth, s.error, s.min_value,
                       s.max_value] for s in st], dtype=np.float64)
    assert np.array_equal(buf[:, 2 * A:].view(np.uint64), stats.view(np.uint64))
    merged = bp.engine.merge_roots(group)
    for g in range(B // group):
        sl = slice(g * group, (g + 1) * group)
        a, sv, stt = merge_roots(vis[sl].tolist(), tot[sl].tolist(), sel)
        m = merged[g]
        assert m.action == a
        assert list(m.visits[:A]) == sv
        assert [x.hex() for x in m.totals[:A]] == [x.hex() for x in stt]
        assert m.num_trees == group
        assert m.num_sims == sum(s.num_sims for s in st[sl])
        assert m.root_visits == sum(s.root_visits for s in st[sl])
        assert m.search_depth == max(s.search_depth for s in st[sl])
        assert m.min_value == min(s.min_value for s in st[sl])
        assert m.max_value == max(s.max_value for s in st[sl])
    bp.close()


@pytest.mark.parametrize("world,group", [(3, 5), (8, 1), (5, 40)])
def test_device_merge_over_gathered_ranks(world, group):
    """pomcp_merge_roots(world > 1) on a gather buffer: rank r's records are the
    batch's records rolled by r * group trees (as if rank r had searched those
    roots), so planner g's replica j = r * group + k is tree (g group + k + r
    group) mod B.  The device merge of the world x group replicas equals the
    CPU merge in replica order, bit for bit (the order the all-gather fixes for
    every rank count)."""
    import torch
    from oracle.root_parallel import merge_roots
    from posggym_baselines_amd.planning import BatchedPOMCP
    from posggym_baselines_amd.planning.parallel import gather_buffer_tensor
    model = product_model("Driving-v1")
    A, S = 5, 48
    B = group * 8
    bp = BatchedPOMCP(model, "0", product_config(CFG, S), B, S)
    bp.init_synthetic(501)
    bp.search(fetch=False)
    buf, st = _records(bp, A)
    gath = gather_buffer_tensor(bp.engine, world, torch.device("cuda:0"))
    rows = np.concatenate([np.roll(buf, -r * group, axis=0) for r in range(world)])
    gath.copy_(torch.from_numpy(rows.reshape(-1)).to("cuda:0"))
    torch.cuda.synchronize()
    merged = bp.engine.merge_roots(group, world=world)
    for g in range(B // group):
        idx = [(g * group + k + r * group) % B for r in range(world) for k in range(group)]
        a, sv, stt = merge_roots(buf[idx, 0:2 * A:2].tolist(), buf[idx, 1:2 * A:2].tolist(), "ucb")
        m = merged[g]
        assert m.num_trees == world * group
        assert m.action == a
        assert list(m.visits[:A]) == sv
        assert [x.hex() for x in m.totals[:A]] == [x.hex() for x in stt]
        assert m.num_sims == sum(int(buf[i, 2 * A]) for i in idx)
        assert m.min_value == min(buf[i, 2 * A + 4] for i in idx)
    bp.close()


def test_single_root_65536_sims_over_replicas():
    """Config 2's 65,536 simulations for ONE root spread over 1,024 replicas
    (64 each): one launch; the merged visits account for every simulation."""
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    from oracle.episode import run_episode
    model = product_model("Driving-v1")
    config = product_config(CFG, 65536)
    config.root_parallel = 1024
    planner = POMCP(model, "0", config, RandomSearchPolicy(model, "0"))
    planner.reset()
    acts = []

    def step(obs):
        a = planner.step(obs)
        if not planner.root.is_absorbing:
            assert planner.step_statistics["num_sims"] == 65536
            if not acts:   # the first root: no visits from earlier searches
                assert sum(planner.root.child_visits) == 65536
                assert planner.root.visits == 65536
        acts.append(a)
        return a

    run_episode(step, 99, max_steps=3)
    assert all(0 <= a < 5 for a in acts)
    planner.close()


def test_root_parallel_wall_clock_episode():
    """num_sims=None with K = 16 replicas: the time-limited chunk loop drives
    all replicas together (each chunk within every replica's arena headroom),
    the device merge picks each action, a multi-step episode runs without an
    arena error or early stop and every step searches all replicas."""
    from oracle.episode import run_episode
    from posggym_baselines_amd.planning import MCTSConfig, POMCP, RandomSearchPolicy
    model = product_model("Driving-v1")
    cfg = MCTSConfig(**dict(CFG, search_time_limit=0.25))
    cfg.root_parallel = 16
    planner = POMCP(model, "0", cfg, RandomSearchPolicy(model, "0"))
    planner.reset()
    steps = []

    def step(obs):
        a = planner.step(obs)
        if not planner.root.is_absorbing:
            st = planner.step_statistics
            assert not st.get("arena_full")
            assert 0.2 <= st["search_time"] < 1.5
            steps.append((int(a), int(st["num_sims"])))
        return a

    trace = run_episode(step, 77, max_steps=12)
    planner.close()
    assert trace["len"] >= 3 and len(steps) >= 2
    assert all(0 <= a < 5 and n >= 16 * 16 and n % 16 == 0 for a, n in steps), steps


def test_allgather_root_c_abi_single_rank():
    """pomcp_allgather_root (the C-ABI exchange of SURVEY §8(b)) over a one-rank
    RCCL communicator made with the process's librccl (ncclCommInitAll; the
    library resolves ncclAllGather in the copy already loaded): the gather
    buffer of one rank equals the merge buffer, and the merge over it equals
    the local merge."""
    import ctypes as C
    import torch
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning import BatchedPOMCP
    from posggym_baselines_amd.planning.parallel import gather_buffer_tensor, merge_buffer_tensor
    model = product_model("Driving-v1")
    bp = BatchedPOMCP(model, "0", product_config(CFG, 64), 16, 64)
    bp.init_synthetic(1000)
    bp.search()
    bp.engine.root_stats()   # synchronises the engine
    dev = torch.device("cuda:0")
    local = merge_buffer_tensor(bp.engine, dev).cpu().clone()
    key = lambda ms: [(m.action, list(m.visits), [float(x).hex() for x in m.totals], m.num_sims,
                       m.root_visits, m.search_depth) for m in ms]
    m0 = key(bp.engine.merge_roots(4))
    rccl = C.CDLL("librccl.so.1")
    comm = C.c_void_p()
    devs = (C.c_int * 1)(0)
    assert rccl.ncclCommInitAll(C.byref(comm), 1, devs) == 0
    try:
        assert N.load().pomcp_allgather_root(bp.engine._ctx, comm, 1) == 0
        bp.engine.root_stats()
        gathered = gather_buffer_tensor(bp.engine, 1, dev).cpu()
        assert torch.equal(gathered.view(torch.int64), local.view(torch.int64))
        assert key(bp.engine.merge_roots(4, world=1)) == m0
    finally:
        rccl.ncclCommDestroy(comm)
        bp.close()
