"""GPU parity of the I-NTMCP engine (BASELINE config 5) through the C ABI:
every step record of the reference goldens (level-1 root statistics, root
particles with the other agent's histories, every level-0 node those histories
name: visits, children, particles) must match bit for bit."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))

from golden_util import (INTMCP0_CASES, INTMCP2_CASES, INTMCP3_CASES, INTMCP45_CASES,
                         INTMCP_CASES, INTMCP_SP_CASES, cfg_kwargs, load, search_probs)
from gpu_util import gpu_intmcp_episode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", INTMCP_CASES + INTMCP0_CASES + INTMCP2_CASES + INTMCP3_CASES
                         + INTMCP45_CASES + INTMCP_SP_CASES)
def test_gpu_intmcp_matches_reference_goldens(case):
    """Nesting level 1 (intmcp_*) and 0 (intmcp0_*: the planner's own tree,
    the other agent acting by the planner's random choice), 2 to 5
    (intmcp2_* ... intmcp5_*: three to six trees); *_sp_*: fixed-distribution
    search policies per level and agent."""
    data = load(case)
    for ep in data["episodes"]:
        kw = cfg_kwargs(ep["config"])
        trace, records = gpu_intmcp_episode(kw, data["num_sims"], ep["env_seed"],
                                            ego=data["ego"], max_steps=data["max_steps"],
                                            env=data["env"],
                                            nesting_level=data.get("nesting_level", 1),
                                            search_probs=search_probs(data))
        assert len(records) == len(ep["records"]), case
        for t, (got, exp) in enumerate(zip(records, ep["records"])):
            assert got == exp, f"{case} env_seed {ep['env_seed']} step {t}"
        assert trace == ep["trace"]


TEST_CFG = dict(discount=0.95, search_time_limit=0.1, c=2 ** 0.5, truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, seed=3, state_belief_only=False)


def _check_all_pairs(name, got):
    """Every pair's records against the oracle's digest (tests/golden/
    make_oracle_digests.py); a mismatching pair is rerun on the oracle so the
    failure shows the first differing step."""
    from golden_util import load
    from make_oracle_digests import CASES, oracle_pair, record_digest
    fx = load("oracle_digests")[name]
    assert len(got) == len(fx["digests"]) == CASES[name]["pairs"]
    bad = [b for b, recs in enumerate(got) if record_digest(recs) != fx["digests"][b]]
    if bad:
        b = bad[0]
        exp = oracle_pair(CASES[name], b)
        for t, (g, e) in enumerate(zip(got[b], exp)):
            assert g == e, f"{name}: {len(bad)} pairs differ; pair {b} step {t}"
        assert len(got[b]) == len(exp), f"{name}: pair {b} step count"
        raise AssertionError(f"{name}: {len(bad)} pairs differ (first {b}): digest only")


def _run_case(name, softmax_slack=None, exact=None):
    from gpu_util import batched_intmcp_episodes
    from make_oracle_digests import CASES, case_cfg
    c = CASES[name]
    seeds = [c["seed0"] + b for b in range(c["pairs"])]
    return batched_intmcp_episodes(case_cfg(c), c["sims"], seeds, c["steps"], env=c["env"],
                                   ego=c["ego"], softmax_slack=softmax_slack, exact=exact)


@pytest.mark.parametrize("name", ["im_drv_ucb_48", "im_pe_uniform_48"])
def test_batched_pairs_match_oracle(name):
    """Planner pairs in one engine, lockstep episodes (4 steps, 48 simulations
    per level): EVERY pair b equals the oracle planner with tree key b.  1,100
    Driving pairs (the update runs a lane per pair) and 150 PursuitEvasion pairs
    (a wave per pair, shared log scans)."""
    _check_all_pairs(name, _run_case(name))


@pytest.mark.parametrize("name", ["im_drv_ucb_256", "im_pe_ucb_256"])
def test_bench_workload_pairs_match_oracle(name):
    """The bench's 256 simulations per level (bench.py --planner intmcp,
    TEST_CFG of the bench), 3 lockstep steps of 130 pairs: every pair equals
    the oracle planner with its tree key (every step record, incl. the
    level-0 nodes the root's histories name)."""
    _check_all_pairs(name, _run_case(name))


def test_softmax_exact_fallback_fires_and_is_exact():
    """The other agent's softmax (intmcp.py:763-791) takes its choice from
    bounded FP32 weights and falls back to the exact FP64 path near a
    cumulative weight.  With the product's bound the fallback
    fires on a small fraction of draws; with the bound widened 3000x it takes
    most draws.  Both runs of the bench workload's 130 Driving pairs are
    bit-exact against the oracle, and both count exact-path draws."""
    n1, n3000 = [], []
    _check_all_pairs("im_drv_ucb_256", _run_case("im_drv_ucb_256", softmax_slack=1.0, exact=n1))
    _check_all_pairs("im_drv_ucb_256", _run_case("im_drv_ucb_256", softmax_slack=3000.0,
                                                 exact=n3000))
    assert n1[0] > 0 and n3000[0] > 10 * n1[0], (n1, n3000)


@pytest.mark.parametrize("case", INTMCP_CASES)
def test_gpu_intmcp_goldens_exact_softmax_path(case):
    """The reference goldens with the fast softmax bound widened 3000x (the
    exact FP64 path decides most draws): still bit-exact, and the exact path
    ran."""
    data = load(case)
    exact = []
    for ep in data["episodes"]:
        kw = cfg_kwargs(ep["config"])
        trace, records = gpu_intmcp_episode(kw, data["num_sims"], ep["env_seed"],
                                            ego=data["ego"], max_steps=data["max_steps"],
                                            env=data["env"], softmax_slack=3000.0, exact=exact)
        assert records == ep["records"], case
        assert trace == ep["trace"]
    assert sum(exact) > 0, case


def test_batched_many_pairs_properties():
    """4096 pairs, one step: every pair searched 2 x num_sims simulations, its
    level-1 root visits equal num_sims, and the root's children visits sum to it."""
    import numpy as np
    from gpu_util import product_config, product_model
    from posggym_baselines_amd.planning import BatchedINTMCP
    model = product_model("Driving-v1")
    B, S = 4096, 256
    bp = BatchedINTMCP(model, "0", product_config(TEST_CFG, S), B, S)
    bp.init_synthetic(1000)
    actions = bp.search()
    st = bp.engine.root_stats()
    assert np.all((actions >= 0) & (actions < 5))
    for s in st:
        assert s.error == 0
        if s.root_absorbing:
            continue
        assert s.num_sims == 2 * S
        assert s.root_visits == S
        assert sum(s.child_visits[i] for i in range(s.num_children)) == S
    bp.close()


def test_device_softmax_exp_equals_math_exp():
    """The softmax exp of the other agent's action draw (intmcp.py:782-790) runs
    on the device as host_exp (csrc/host_exp.h): it must equal this host's
    math.exp bit for bit on every v / sqrt(N) the softmax can see (all of them
    for N <= 4096, a sample up to N = 65,536) plus random and special
    arguments, > 9 M in all.  math.exp is evaluated here, on the GPU box's host."""
    import ctypes as C
    import numpy as np
    from posggym_baselines_amd import _native as N
    from test_host_exp import _py_exp, _same, softmax_arguments, special_arguments
    rng = np.random.default_rng(1)
    x = np.concatenate([softmax_arguments(rng), special_arguments(rng)])
    assert len(x) > 9_000_000
    out = np.zeros_like(x)
    P = C.POINTER(C.c_double)
    assert N.load().pomcp_debug_exp(x.ctypes.data_as(P), len(x), out.ctypes.data_as(P)) == 0
    ref = _py_exp(x)
    bad = np.nonzero(~_same(out, ref))[0]
    assert len(bad) == 0, [(x[i].hex(), out[i].hex(), ref[i].hex()) for i in bad[:5]]


def _wall_clock_episode(time_limit, env_seed, max_steps, nesting_level=1):
    from gpu_util import product_model
    from oracle.episode import run_episode
    from posggym_baselines_amd.planning import INTMCP, MCTSConfig
    model = product_model("Driving-v1")
    cfg = MCTSConfig(**dict(TEST_CFG, search_time_limit=time_limit))   # num_sims=None
    planner = INTMCP.initialize(model, "0", cfg, nesting_level, None)
    planner.reset()
    steps = []

    def step(obs):
        a = planner.step(obs)
        if not planner.root.is_absorbing:
            st = planner._engine.root_stats()[0]
            steps.append(dict(planner.step_statistics, visits=planner.root.visits,
                              child_visits=sum(c[1] for c in planner.root.children),
                              n_log=(int(st.n_log[0]), int(st.n_log[1])),
                              n_nodes=(int(st.n_nodes[0]), int(st.n_nodes[1]))))
        return a

    trace = run_episode(step, env_seed, max_steps=max_steps)
    planner.close()
    return trace, steps, planner._engine.wall_clock_sims


def test_wall_clock_episode_half_second():
    """The reference's default mode (num_sims=None, intmcp.py:383-397: the time
    limit split over the levels) over a whole Driving-v1 episode at
    search_time_limit=0.5: arenas sized from the time limit, every chunk within
    the headroom, no POMCP_E_ARENA and no early stop."""
    trace, steps, ceiling = _wall_clock_episode(0.5, 41, 50)
    assert trace["len"] >= 3 and len(steps) >= 2
    for st in steps:
        assert not st.get("arena_full")
        assert 0.45 <= st["search_time"] < 2.0
        assert 64 < st["num_sims"] <= 2 * ceiling
        assert 0 < st["child_visits"] <= st["visits"]
    print("I-NTMCP wall-clock sims per step:", [st["num_sims"] for st in steps])


def test_wall_clock_nesting2_episode():
    """Nesting level 2 in the reference's default mode: the time limit split
    over three levels, chunks per level (intmcp_search_level) within the
    headroom of all three trees (intmcp_get_tree_counts), no arena failure."""
    trace, steps, ceiling = _wall_clock_episode(0.6, 43, 8, nesting_level=2)
    assert len(steps) >= 2
    for st in steps:
        assert not st.get("arena_full")
        assert 0.5 <= st["search_time"] < 2.5
        assert 3 <= st["num_sims"] <= 3 * ceiling
        assert 0 < st["child_visits"] <= st["visits"]
    print("I-NTMCP nesting-2 wall-clock sims per step:", [st["num_sims"] for st in steps])


def test_wall_clock_nesting3_episode():
    """Nesting level 3 in the reference's default mode: the time limit split
    over four levels, within the headroom of all four trees, no arena failure."""
    trace, steps, ceiling = _wall_clock_episode(0.8, 47, 6, nesting_level=3)
    assert len(steps) >= 2
    for st in steps:
        assert not st.get("arena_full")
        assert 0.7 <= st["search_time"] < 3.0
        assert 4 <= st["num_sims"] <= 4 * ceiling
        assert 0 < st["child_visits"] <= st["visits"]
    print("I-NTMCP nesting-3 wall-clock sims per step:", [st["num_sims"] for st in steps])


def test_wall_clock_small_arena_stops_early(monkeypatch):
    """A 64 K-node arena (the floor) cannot hold a 1 s episode: the chunk loop
    stops at the headroom (step_statistics["arena_full"]) instead of failing,
    the update's reinvigoration still fits, and every step returns an action."""
    from posggym_baselines_amd.planning import intmcp as M
    monkeypatch.setattr(M, "INTMCP_WALL_CLOCK_HBM_BUDGET", 1)
    trace, steps, _ = _wall_clock_episode(1.0, 41, 12)
    assert len(steps) >= 2   # (the episode's length depends on the actions chosen)
    assert any(st.get("arena_full") for st in steps)
    assert all(st["child_visits"] <= st["visits"] for st in steps)


def test_wall_clock_old_beliefs_cleared(monkeypatch):
    """intmcp.py:326-330: at every update the particles of nodes more than two
    steps behind are dropped, so the particle logs hold about three searches'
    records (a search's records sit at depths t+1..t+3 and are dropped five
    steps later), not the episode's.  With a node / log arena of ~3 M entries
    (a 2 GiB budget) a 1 s episode appending ~150-300 k records per tree per
    step never stops early, and the log stays bounded while the trees grow."""
    from posggym_baselines_amd.planning import intmcp as M
    monkeypatch.setattr(M, "INTMCP_WALL_CLOCK_HBM_BUDGET", 2 << 30)
    trace, steps, ceiling = _wall_clock_episode(1.0, 41, 12)
    assert len(steps) >= 6, len(steps)
    for st in steps:
        assert not st.get("arena_full"), [(x["n_log"], x["num_sims"]) for x in steps]
    appended = sum(x["num_sims"] for x in steps) * 3   # <= 3 records per simulation (depth 2)
    peak = max(max(x["n_log"]) for x in steps)
    assert peak < appended // 2, (peak, appended)
    print("I-NTMCP 1 s episode, n_log per step:", [x["n_log"] for x in steps])


def test_search_split_over_launches_equals_one_launch():
    """The wall-clock loop's chunked launches (search_levels, several per level,
    then the final selection alone) are bit-identical to one launch of the same
    totals, and so is the next step (update + search) after them: the RNG
    words k_im_search computes ahead and does not consume are not counted as
    drawn (ImPair::la_pend)."""
    import numpy as np
    from gpu_util import intmcp_state_record, product_config, product_model
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning import BatchedINTMCP
    model = product_model("Driving-v1")
    B, S = 130, 96
    one = BatchedINTMCP(model, "0", product_config(TEST_CFG, S), B, S, searches=2)
    split = BatchedINTMCP(model, "0", product_config(TEST_CFG, S), B, S, searches=2)
    keys = one.init_synthetic(1000)
    split.init_synthetic(1000)
    for step in range(2):
        a1 = one.search()
        e = split.engine
        e.search_levels(40, 0, N.INTMCP_BEGIN)
        e.search_levels(S - 40, 0, 0)
        e.search_levels(0, 7, 0)
        e.search_levels(0, S - 7, 0)
        e.search_levels(0, 0, N.INTMCP_FINAL)
        a2 = np.array([s.action for s in e.root_stats()], dtype=a1.dtype)
        assert np.array_equal(a1, a2), step
        for b in (0, 1, 63, 64, 129):
            r1 = intmcp_state_record(one.engine, b, True, int(a1[b]))
            r2 = intmcp_state_record(e, b, True, int(a2[b]))
            assert r1 == r2, (step, b)
        acts = np.asarray(a1, dtype=np.int32)
        one.engine.update(acts, keys)
        e.update(acts, keys)
    one.close()
    split.close()


@pytest.mark.parametrize("env,ego", [("Driving-v1", "0"), ("PursuitEvasion-v1", "1")])
def test_gpu_intmcp_nesting0_batched_pairs_match_oracle(env, ego):
    """Nesting level 0, many planners in one launch: every planner's records
    against the oracle (oracle/intmcp.py, pinned at nesting 0 by the
    intmcp0_* goldens) with that planner's tree key."""
    from gpu_util import batched_intmcp_episodes
    from oracle.run import oracle_intmcp_episode
    B, sims, steps = 6, 40, 8
    seeds = [300 + b for b in range(B)]
    got = batched_intmcp_episodes(TEST_CFG, sims, seeds, steps, env=env, ego=ego,
                                  nesting_level=0)
    for b in range(B):
        _, exp = oracle_intmcp_episode(TEST_CFG, sims, seeds[b], ego=ego, tree=b,
                                       max_steps=steps, env=env, nesting_level=0)
        assert len(got[b]) == len(exp), b
        for t, (g, e) in enumerate(zip(got[b], exp)):
            assert g == e, f"{env} pair {b} step {t}"


@pytest.mark.parametrize("nesting", [1, 2])
def test_gpu_intmcp_step_limit_cutoffs_match_oracle(nesting):
    """A planner step limit well below the depth limit (step_limit=6, epsilon
    0.05: depth_limit 59): the descent stops at obs_node.t + depth >
    step_limit (intmcp.py:450-453), at a depth that shrinks every step -- the
    level at which k_im_search loads only the child's node (no statistics
    heads, no next history view) is then decided by the step limit.  5 pairs
    x 6 steps against the oracle."""
    from gpu_util import batched_intmcp_episodes
    from oracle.run import oracle_intmcp_episode
    cfg = dict(TEST_CFG, step_limit=6, epsilon=0.05)
    B, sims, steps = 5, 24, 6
    seeds = [700 + b for b in range(B)]
    got = batched_intmcp_episodes(cfg, sims, seeds, steps, nesting_level=nesting)
    for b in range(B):
        _, exp = oracle_intmcp_episode(cfg, sims, seeds[b], tree=b, max_steps=steps,
                                       nesting_level=nesting)
        assert len(got[b]) == len(exp), b
        for t, (g, e) in enumerate(zip(got[b], exp)):
            assert g == e, f"nesting {nesting} pair {b} step {t}"


def test_intmcp_nesting0_rejects_level1_simulations():
    import ctypes as C
    from gpu_util import product_config, product_model
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning import INTMCP
    planner = INTMCP.initialize(product_model("Driving-v1"), "0", product_config(TEST_CFG, 16),
                                0, None)
    assert planner.other_agent_policies == {}
    rc = N.load().intmcp_search_levels(planner._engine._ctx, 4, 4, N.INTMCP_BEGIN, None)
    assert rc == N.POMCP_E_INVALID
    planner.close()


@pytest.mark.parametrize("env,ego", [("Driving-v1", "0"), ("PursuitEvasion-v1", "1")])
def test_gpu_intmcp_nesting2_batched_pairs_match_oracle(env, ego):
    """Nesting level 2 (three trees per pair), many planners in one launch:
    every planner's records against the oracle (oracle/intmcp.py, pinned at
    nesting 2 by the intmcp2_* goldens) with that planner's tree key."""
    from gpu_util import batched_intmcp_episodes
    from oracle.run import oracle_intmcp_episode
    B, sims, steps = 5, 24, 6
    seeds = [400 + b for b in range(B)]
    got = batched_intmcp_episodes(TEST_CFG, sims, seeds, steps, env=env, ego=ego,
                                  nesting_level=2)
    for b in range(B):
        _, exp = oracle_intmcp_episode(TEST_CFG, sims, seeds[b], ego=ego, tree=b,
                                       max_steps=steps, env=env, nesting_level=2)
        assert len(got[b]) == len(exp), b
        for t, (g, e) in enumerate(zip(got[b], exp)):
            assert g == e, f"{env} pair {b} step {t}"


@pytest.mark.parametrize("env,ego", [("Driving-v1", "1"), ("PursuitEvasion-v1", "0")])
def test_gpu_intmcp_nesting3_batched_pairs_match_oracle(env, ego):
    """Nesting level 3 (four trees per pair, two middle belief tables), many
    planners in one launch: every planner's records against the oracle
    (pinned at nesting 3 by the intmcp3_* goldens) with that planner's tree key."""
    from gpu_util import batched_intmcp_episodes
    from oracle.run import oracle_intmcp_episode
    B, sims, steps = 4, 20, 5
    seeds = [450 + b for b in range(B)]
    got = batched_intmcp_episodes(TEST_CFG, sims, seeds, steps, env=env, ego=ego,
                                  nesting_level=3)
    for b in range(B):
        _, exp = oracle_intmcp_episode(TEST_CFG, sims, seeds[b], ego=ego, tree=b,
                                       max_steps=steps, env=env, nesting_level=3)
        assert len(got[b]) == len(exp), b
        for t, (g, e) in enumerate(zip(got[b], exp)):
            assert g == e, f"{env} pair {b} step {t}"


@pytest.mark.parametrize("nesting,env,ego", [(4, "Driving-v1", "0"), (4, "PursuitEvasion-v1", "1"),
                                              (5, "Driving-v1", "1")])
def test_gpu_intmcp_deep_nesting_batched_pairs_match_oracle(nesting, env, ego):
    """Nesting levels 4 and 5 (five / six trees per pair, three / four middle
    belief tables; level 5's level-4 middle planner on the streams past the
    action streams), several planners in one launch: every planner's records
    against the oracle (pinned at these levels by the intmcp4_* / intmcp5_*
    goldens) with that planner's tree key."""
    from gpu_util import batched_intmcp_episodes
    from oracle.run import oracle_intmcp_episode
    B, sims, steps = 3, 10, 4
    seeds = [480 + 10 * nesting + b for b in range(B)]
    got = batched_intmcp_episodes(TEST_CFG, sims, seeds, steps, env=env, ego=ego,
                                  nesting_level=nesting)
    for b in range(B):
        _, exp = oracle_intmcp_episode(TEST_CFG, sims, seeds[b], ego=ego, tree=b,
                                       max_steps=steps, env=env, nesting_level=nesting)
        assert len(got[b]) == len(exp), b
        for t, (g, e) in enumerate(zip(got[b], exp)):
            assert g == e, f"{env} nesting {nesting} pair {b} step {t}"


def test_intmcp_nesting_beyond_the_build_is_refused():
    """INTMCP.initialize accepts any nesting level (intmcp.py:949-994); the GPU
    engine builds 0 .. MAX_NESTING and refuses a deeper one before touching the
    GPU (NotImplementedError), never silently planning a shallower chain."""
    from gpu_util import product_config, product_model
    from posggym_baselines_amd.planning import INTMCP
    from posggym_baselines_amd.planning.intmcp import MAX_NESTING
    model = product_model("Driving-v1")
    with pytest.raises(NotImplementedError):
        INTMCP.initialize(model, "0", product_config(TEST_CFG, 8), MAX_NESTING + 1, None)


def test_intmcp_nesting3_search_level_chunks_equal_one_search():
    """Nesting level 3: chunks per level (intmcp_search_level) equal one launch
    of all four levels, record for record (every tree, both middle tables)."""
    import numpy as np
    from gpu_util import intmcp_state_record, product_config, product_model
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning.intmcp import BatchedINTMCP
    model = product_model("Driving-v1")
    cfg = product_config(TEST_CFG, 20)
    one = BatchedINTMCP(model, "0", cfg, 3, 20, searches=3, nesting_level=3)
    split = BatchedINTMCP(model, "0", cfg, 3, 20, searches=3, nesting_level=3)
    keys = one.init_synthetic(600)
    split.init_synthetic(600)
    for step in range(2):
        a1 = one.search()
        e = split.engine
        e.search_level(0, 9, N.INTMCP_BEGIN)
        e.search_level(0, 11, 0)
        e.search_level(1, 20, 0)
        e.search_level(2, 20, 0)
        e.search_level(3, 5, 0)
        a2 = e.search_level(3, 15, N.INTMCP_FINAL, fetch=True)
        assert np.array_equal(a1, a2), step
        for b in range(3):
            assert e.root_stats()[b].num_sims == 80
            r1 = intmcp_state_record(one.engine, b, True, int(a1[b]))
            r2 = intmcp_state_record(e, b, True, int(a2[b]))
            assert r1 == r2 and "nested3_digest" in r1, (step, b)
        acts = np.asarray(a1, dtype=np.int32)
        one.engine.update(acts, keys)
        e.update(acts, keys)
    with pytest.raises(Exception):
        e.mid_support(0, 3)   # the level-0 tree is not a middle tree
    one.close()
    split.close()


def test_intmcp_nesting2_search_level_chunks_equal_one_search():
    """Nesting level 2: get_action as chunks per level (intmcp_search_level, the
    wall-clock loop's launches) is bit-identical to one launch of all three
    levels."""
    import numpy as np
    from gpu_util import intmcp_state_record, product_config, product_model
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning.intmcp import BatchedINTMCP
    model = product_model("Driving-v1")
    cfg = product_config(TEST_CFG, 30)
    one = BatchedINTMCP(model, "0", cfg, 4, 30, searches=3, nesting_level=2)
    split = BatchedINTMCP(model, "0", cfg, 4, 30, searches=3, nesting_level=2)
    keys = one.init_synthetic(500)
    split.init_synthetic(500)
    for step in range(2):
        a1 = one.search()
        e = split.engine
        e.search_level(0, 7, N.INTMCP_BEGIN)
        e.search_level(0, 23, 0)
        e.search_level(1, 30, 0)
        e.search_level(2, 11, 0)
        a2 = e.search_level(2, 19, N.INTMCP_FINAL, fetch=True)
        assert np.array_equal(a1, a2), step
        for b in range(4):
            assert e.root_stats()[b].num_sims == 90
            r1 = intmcp_state_record(one.engine, b, True, int(a1[b]))
            r2 = intmcp_state_record(e, b, True, int(a2[b]))
            assert r1 == r2, (step, b)
        acts = np.asarray(a1, dtype=np.int32)
        one.engine.update(acts, keys)
        e.update(acts, keys)
    one.close()
    split.close()
