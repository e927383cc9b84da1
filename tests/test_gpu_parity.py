"""GPU parity: the HIP engine through the C ABI against the reference goldens
and the oracle (bit-exact: actions, visit counts, FP64 values, particles)."""
import math

import numpy as np
import pytest

from golden_util import EPISODE_CASES, IPOMCP_CASES, case_env, case_max_steps, cfg_kwargs, load
from gpu_util import gpu_episode, product_config, stats_record
from oracle.episode import run_episode
from oracle.run import make_oracle, oracle_record

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["lane", "lane_eager", "wave", "wave_tree", "wave_plain"])
def search_kernel(request, monkeypatch):
    """Every parity test runs on every search kernel: k_search (a tree per lane,
    tree in HBM) with cut-off children deferred to the re-root ("lane") and
    looked up during the search ("lane_eager", pomcp_set_defer_cutoff) -- both
    forced through POMCP_DEFER_CUTOFF, so they hold for every planner whatever
    its own choice (the default: deferred) -- and
    k_search_lds (a wave per tree, tree in LDS) -- with its step-tree producer
    waves as the engine picks them ("wave"), forced on for any depth limit
    ("wave_tree") and off ("wave_plain"); they must give the same bits as the
    reference / oracle."""
    kind, _, mode = request.param.partition("_")
    monkeypatch.setenv("POMCP_SEARCH_KERNEL", kind)
    if kind == "lane":   # the override wins over the planners' own choice
        monkeypatch.setenv("POMCP_DEFER_CUTOFF", "0" if mode == "eager" else "1")
    elif mode:
        monkeypatch.setenv("POMCP_STEP_TREE", "1" if mode == "tree" else "0")
    return kind

SQRT2 = math.sqrt(2)
TEST_CFG = dict(discount=0.95, search_time_limit=0.1, c=SQRT2, truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, seed=0, state_belief_only=True)


def test_device_fp64_is_correctly_rounded():
    import ctypes as C
    from posggym_baselines_amd import _native as N
    rng = np.random.default_rng(0)
    n = 1 << 16
    a = np.concatenate([rng.random(n // 2) * 10, np.exp(rng.normal(0, 20, n // 2))])
    b = np.concatenate([rng.random(n // 2) + 1e-3, np.exp(rng.normal(0, 20, n // 2))])
    out = np.zeros(4 * n)
    P = C.POINTER(C.c_double)
    assert N.load().pomcp_debug_fp_selftest(a.ctypes.data_as(P), b.ctypes.data_as(P), n,
                                            out.ctypes.data_as(P)) == 0
    out = out.reshape(n, 4)
    assert np.array_equal(out[:, 0], np.sqrt(a))
    assert np.array_equal(out[:, 1], a / b)
    assert np.array_equal(out[:, 2], a + 0.95 * b)
    assert np.array_equal(out[:, 3], (a - b) / (a + b))


def test_fast_ucb_reciprocals_error_bound():
    """k_search's fast UCB scores use rcp_nr(range) and rsq_nr(n) (hardware
    estimates + one Newton step); their exact fallback (a 1e-12 relative
    margin) needs each far more accurate than that.  Checked
    here against correctly rounded 1/x and 1/sqrt(x) on every visit count up
    to 2^20 and on random positive doubles: relative error <= 1e-14 (measured
    ~5e-15)."""
    import ctypes as C
    from posggym_baselines_amd import _native as N
    rng = np.random.default_rng(1)
    x = np.concatenate([np.arange(1, 1 << 20, dtype=np.float64),
                        np.exp(rng.uniform(-30, 30, 1 << 18)), rng.uniform(1e-3, 4.0, 1 << 18)])
    out = np.zeros(2 * len(x))
    P = C.POINTER(C.c_double)
    assert N.load().pomcp_debug_fast_recip(x.ctypes.data_as(P), len(x), out.ctypes.data_as(P)) == 0
    out = out.reshape(-1, 2)

    assert (np.abs(out[:, 0] - 1.0 / x) * x).max() <= 1e-14
    assert (np.abs(out[:, 1] - 1.0 / np.sqrt(x)) * np.sqrt(x)).max() <= 1e-14


@pytest.mark.parametrize("case", EPISODE_CASES)
def test_gpu_matches_reference_goldens(case):
    data = load(case)
    for ep in data["episodes"]:
        kw = cfg_kwargs(ep["config"])
        trace, records = gpu_episode(kw, data["num_sims"], ep["env_seed"], ego=data["ego"],
                                     max_steps=case_max_steps(case, data), env=case_env(data))
        assert len(records) == len(ep["records"])
        for t, (got, exp) in enumerate(zip(records, ep["records"])):
            assert got == exp, f"{case} step {t}"
        assert trace == ep["trace"]


@pytest.mark.parametrize("case", IPOMCP_CASES)
def test_gpu_ipomcp_matches_reference_goldens(case):
    """The IPOMCP drop-in (random other agents) against the real reference
    IPOMCP run with state_belief_only=False (ipomcp.py:11-38)."""
    data = load(case)
    for ep in data["episodes"]:
        kw = cfg_kwargs(ep["config"])
        assert kw["state_belief_only"] is False
        trace, records = gpu_episode(kw, data["num_sims"], ep["env_seed"], ego=data["ego"],
                                     max_steps=case_max_steps(case, data), env=case_env(data),
                                     planner_cls="IPOMCP")
        assert records == ep["records"]
        assert trace == ep["trace"]


def _oracle_first_step(cfg, num_sims, tree, env_seed, rekey=None, env="Driving-v1"):
    p = make_oracle(cfg, num_sims, tree=tree, env=env)
    recs = []

    def step(obs):
        p.update(None, obs)
        if rekey is not None:
            p.s.rekey(rekey)
        a = p.get_action()
        p.stats["searched"] = True
        recs.append(oracle_record(p, True, a))
        return a

    run_episode(step, env_seed, max_steps=1, env=env)
    return recs[0]


def _batched_vs_oracle(cfg, num_trees, num_sims, check_trees, rekey=None, env="Driving-v1",
                       select_margin=None):
    from gpu_util import product_model
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning import BatchedPOMCP
    model = product_model(env)
    A = model.action_spaces["0"].n
    bp = BatchedPOMCP(model, "0", product_config(cfg, num_sims), num_trees, num_sims)
    if select_margin is not None:
        assert N.load().pomcp_debug_set_select_margin(bp.engine._ctx, float(select_margin)) == 0
    bp.init_synthetic(1000)
    if rekey is not None:
        bp.engine.rekey(rekey)
    actions = bp.search()
    stats = bp.engine.root_stats()
    for b in check_trees:
        exp = _oracle_first_step(cfg, num_sims, b, 1000 + b, rekey=rekey, env=env)
        got = stats_record(stats[b], A, True, actions[b], bp.engine.root_belief(b))
        assert got == exp, f"tree {b}"
    bp.close()
    return stats


@pytest.mark.parametrize("islots", [1, 2])
def test_overflow_map_bit_exact(islots):
    """The overflow map of obs children (beyond an action node's inline slots:
    k_search's ovf_child, k_reroot_child's lookup, k_compact's rebuild).  The
    models here rarely give an action node more than 6 obs children (none in
    4,096-simulation searches from 2,125-particle roots on either model), so
    the engine uses only `islots` inline slots (pomcp_debug_set_inline_slots)
    and the rest go to the map: 40 planners over 5 real steps with re-roots,
    bit-exact against the oracle, the map probed every search."""
    from gpu_util import batched_episodes
    from oracle.run import oracle_episode
    S, K = 128, 5
    seeds, exp = [], []
    s = 4400
    while len(seeds) < 40:
        trace, recs = oracle_episode(TEST_CFG, S, s, tree=len(seeds), max_steps=K)
        if trace["len"] >= K and all(r["searched"] for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    probes = []
    got = batched_episodes(TEST_CFG, S, seeds, K, inline_slots=islots, probes=probes)
    for b in range(len(seeds)):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"
    assert all(n > 0 for n in probes), probes


def test_batched_synthetic_roots_ucb():
    _batched_vs_oracle(TEST_CFG, 37, 256, range(37))


def test_batched_synthetic_roots_pucb_deep():
    cfg = dict(TEST_CFG, action_selection="pucb", discount=0.99, epsilon=0.01, seed=3)
    _batched_vs_oracle(cfg, 9, 128, range(9))


def test_root_parallel_rekey():
    seed = TEST_CFG["seed"]
    _batched_vs_oracle(TEST_CFG, 6, 200, range(6), rekey=seed ^ (3 << 32))


def test_rekey_survives_restore():
    """bench.py's root-parallel ranks: snapshot, rekey, then restore + search
    every step.  The restore must keep the rank's key (it used to copy the
    snapshot's seed back), so two keys give different statistics, each equal to
    the oracle under its own key."""
    from posggym_baselines_amd.planning import BatchedPOMCP
    from gpu_util import product_model
    model = product_model("Driving-v1")
    S, B = 200, 4
    key = lambda st: [(s.action, tuple(s.child_visits[:5]), tuple(s.child_values[:5])) for s in st]
    runs = []
    for r in (0, 1):
        seed = TEST_CFG["seed"] ^ (r << 32)
        bp = BatchedPOMCP(model, "0", product_config(TEST_CFG, S), B, S)
        bp.init_synthetic(1000)
        bp.engine.rekey(seed)
        bp.restore()
        bp.search()
        first = key(bp.engine.root_stats())
        bp.restore()
        actions = bp.search()
        stats = bp.engine.root_stats()
        assert key(stats) == first
        for b in range(B):
            exp = _oracle_first_step(TEST_CFG, S, b, 1000 + b, rekey=seed)
            assert stats_record(stats[b], 5, True, actions[b], bp.engine.root_belief(b)) == exp
        runs.append(first)
        bp.close()
    assert runs[0] != runs[1]


def test_full_size_65536_sims():
    """BASELINE config 2 size: 65,536 simulations from one root, bit-exact."""
    stats = _batched_vs_oracle(TEST_CFG, 2, 65536, [0])
    # size-independent properties on the other tree
    st = stats[1]
    assert st.num_sims == 65536 and st.root_visits == 65536
    assert sum(st.child_visits[:5]) == 65536


def test_many_trees_properties():
    """Large batch: invariants that hold for every tree (visit conservation,
    Welford totals, action = argmax value)."""
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import BatchedPOMCP
    model = DrivingModel()
    B, S = 2048, 512
    bp = BatchedPOMCP(model, "0", product_config(TEST_CFG, S), B, S)
    bp.init_synthetic(5000)
    actions = bp.search()
    stats = bp.engine.root_stats()
    for b in range(B):
        st = stats[b]
        v = np.array(st.child_visits[:5])
        assert st.error == 0 and st.num_sims == S and st.root_visits == S and v.sum() == S
        vals = np.array(st.child_values[:5])
        tot = np.array(st.child_totals[:5])
        assert np.allclose(vals[v > 0], tot[v > 0] / v[v > 0], rtol=1e-9, atol=1e-12)
        assert vals[actions[b]] == vals.max()
    # determinism: restore + search reproduces every tree bit for bit
    first = [(s.action, tuple(s.child_visits), tuple(s.child_values)) for s in stats]
    bp.restore()
    bp.search()
    again = [(s.action, tuple(s.child_visits), tuple(s.child_values))
             for s in bp.engine.root_stats()]
    assert first == again
    bp.close()


def test_batched_episodes_reroot_across_waves():
    """70 planners (two search waves sharing particle logs) over 6 real steps:
    re-root + log extraction + reinvigoration per tree equal the oracle."""
    from gpu_util import batched_episodes
    from oracle.run import oracle_episode
    S, K = 96, 6
    seeds, exp = [], []
    s = 3000
    while len(seeds) < 70:   # planners whose episodes last >= K steps
        trace, recs = oracle_episode(TEST_CFG, S, s, tree=len(seeds), max_steps=K)
        if trace["len"] >= K and all(r["searched"] for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    got = batched_episodes(TEST_CFG, S, seeds, K)
    for b in range(len(seeds)):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"


def test_step_limit_cutoffs_in_batched_episodes():
    """A planner step limit below the depth limit (MCTSConfig.step_limit=5,
    depth_limit 90): the cut-offs come from t + 1 > step_limit (mcts.py:315),
    deferred or looked up, at a depth that shrinks every step; 12 planners x 5
    real steps (the reference asserts root.t <= step_limit, mcts.py:114) equal
    the oracle, re-roots included."""
    from gpu_util import batched_episodes
    from oracle.run import oracle_episode
    cfg = dict(TEST_CFG, step_limit=5, epsilon=0.01)
    S, K = 128, 5
    seeds, exp = [], []
    s = 5200
    while len(seeds) < 12:
        trace, recs = oracle_episode(cfg, S, s, tree=len(seeds), max_steps=K)
        if trace["len"] >= K and all(r["searched"] for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    got = batched_episodes(cfg, S, seeds, K)
    for b in range(len(seeds)):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"


def test_batched_pursuit_evasion_roots():
    """BASELINE config 3 (PursuitEvasion-v1): batched synthetic roots, evader
    ego, bit-exact against the oracle (ucb and pucb)."""
    _batched_vs_oracle(TEST_CFG, 40, 256, range(40), env="PursuitEvasion-v1")
    cfg = dict(TEST_CFG, action_selection="pucb", seed=5)
    _batched_vs_oracle(cfg, 8, 200, range(8), env="PursuitEvasion-v1")


def test_pursuit_evasion_full_size_65536_sims():
    """BASELINE config 3 size: 65,536 simulations from one PursuitEvasion-v1 root."""
    stats = _batched_vs_oracle(TEST_CFG, 2, 65536, [0], env="PursuitEvasion-v1")
    st = stats[1]
    assert st.num_sims == 65536 and st.root_visits == 65536
    assert sum(st.child_visits[:4]) == 65536


@pytest.mark.parametrize("env", ["Driving-v1", "PursuitEvasion-v1"])
def test_full_size_reroot_episodes(search_kernel, env):
    """The re-root at the benchmarked size (BASELINE configs 2 / 3, bench.py's
    update()-inclusive step): 3-step episodes at 65,536 simulations per search
    -- the initial update, then two re-roots of a 65,536-simulation tree --
    for two planners in one engine, against the REAL reference planner's
    records at that size (tests/golden/make_fullsize_reroot.py runs the
    reference and the oracle and checks they agree): actions, root statistics
    (FP64 bits) and the re-rooted belief (size and insertion-order digest)
    every step.  A re-root here keeps ~10^4 particles, thousands of deferred
    cut-off records per tree (several k_compact_log materialisation chunks of
    1,024) and overflow-free inline slots; Driving plans as agent "0",
    PursuitEvasion as agent "1" (the pursuer)."""
    import os
    from gpu_util import batched_episodes
    data = load("fullsize_reroot")
    cases = [c for c in data["cases"] if c["env"] == env]
    S, K = data["num_sims"], data["steps"]
    assert S == 65536 and K >= 3 and [c["tree"] for c in cases] == list(range(len(cases)))
    # the kept subtree of every re-root holds more cut-off records than one
    # materialisation chunk of k_compact_log (T = 1,024 threads)
    assert all(min(c["kept_cutoff_records"]) > 1024 for c in cases), \
        [c["kept_cutoff_records"] for c in cases]
    assert all(min(r["belief_size"] for r in c["records"][1:]) > 1000 for c in cases)
    counters = []
    got = batched_episodes(cfg_kwargs(data["config"]), S, [c["env_seed"] for c in cases], K,
                           env=env, ego=cases[0]["ego"], counters=counters)
    for b, c in enumerate(cases):
        for t in range(K):
            assert got[b][t] == c["records"][t], f"{env} tree {b} step {t}"
    if search_kernel == "lane" and os.environ.get("POMCP_DEFER_CUTOFF") == "1":
        # every search deferred > 1,000 cut-off records per tree
        assert all(d > 1000 * len(cases) for _, d, _ in counters), counters


@pytest.mark.parametrize("case", ["c1_ucb", "pe_evader_ucb"])
def test_episode_harness_replays_reference_episodes(case):
    """run_planning_episodes (exp_utils.py:468-552 / test_pomcp.py:16-33) with the
    POMCP drop-in replays the reference planner's golden episodes step for step:
    actions of both agents, rewards, length and return (bit-exact)."""
    from gpu_util import product_model
    from oracle.episode import fhex
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    from posggym_baselines_amd.planning.episodes import run_planning_episodes
    data = load(case)
    env = case_env(data)
    ego = data["ego"]
    for ep in data["episodes"]:
        steps = ep["trace"]["steps"]
        for until in ("all_done", "agent_done"):
            model = product_model(env)
            planner = POMCP(model, ego, product_config(cfg_kwargs(ep["config"]), data["num_sims"]),
                            RandomSearchPolicy(model, ego))
            seen = []
            rows = run_planning_episodes(
                planner, product_model(env), 1, ego, env_seeds=[ep["env_seed"]], until=until,
                on_step=lambda t, obs, acts, ts: seen.append(
                    ([acts[i] for i in sorted(acts)], fhex(ts.rewards[ego]),
                     bool(ts.terminations[ego]))))
            planner.close()
            n = len(steps)
            if until == "agent_done":   # exp_utils.py:522: stop when the planning agent is done
                n = next((t + 1 for t, s in enumerate(seen) if s[2]), len(seen))
            assert rows[0]["len"] == n == len(seen)
            for t in range(n):
                assert seen[t][0] == steps[t]["actions"], (case, until, t)
                assert seen[t][1] == steps[t]["reward"], (case, until, t)
            if until == "all_done":
                assert fhex(rows[0]["return"]) == ep["trace"]["return"]
            assert set(rows[0]) >= {"num", "len", "return", "discounted_return", "time",
                                    "search_time", "num_sims", "mem_usage"}


def test_search_split_over_launches_equals_one_launch():
    """get_action as several launches (pomcp_search_continue ... pomcp_search(0),
    the wall-clock loop of mcts.py:285) consumes exactly the draws of one launch
    of the total: every tree's statistics and action are bit-identical."""
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import BatchedPOMCP
    model = DrivingModel()
    B, S = 256, 512
    bp = BatchedPOMCP(model, "0", product_config(dict(TEST_CFG, action_selection="pucb"), S), B, S)
    bp.init_synthetic(7000)
    key = lambda st: [(s.action, tuple(s.child_visits), tuple(s.child_values),
                       tuple(s.child_totals), s.root_visits, s.min_value, s.max_value)
                      for s in st]
    bp.search()
    one = key(bp.engine.root_stats())
    bp.restore()
    for n in (16, 112, 384):
        bp.engine.search(n, final=False)
        assert all(s.action == -1 for s in bp.engine.root_stats())
    bp.engine.search(0)
    assert key(bp.engine.root_stats()) == one
    bp.close()


def test_wall_clock_search_mode():
    """num_sims=None: the reference's time-limited loop (mcts.py:285) as chunked
    launches; one final action choice, sims / depth reported over all chunks."""
    from gpu_util import product_model
    from posggym_baselines_amd.planning import POMCP, MCTSConfig, RandomSearchPolicy
    model = product_model("Driving-v1")
    cfg = MCTSConfig(num_sims=None, **dict(TEST_CFG, search_time_limit=0.05))
    planner = POMCP(model, "0", cfg, RandomSearchPolicy(model, "0"))
    planner.reset()
    obs = model.sample_initial_obs(model.sample_initial_state())
    a = planner.step(obs["0"])
    st = planner.step_statistics
    assert 0 <= a < 5 and st["num_sims"] >= 16 and st["search_depth"] >= 1
    assert planner.root.visits == st["num_sims"] == sum(planner.root.child_visits)
    planner.close()


@pytest.mark.parametrize("scan", ["stream", "stream_global_cmap", "legacy"])
def test_subtree_compaction_forced_small_arena(scan, monkeypatch):
    """Arenas sized for ~2 searches carry 8-step episodes: every update compacts
    the tree to the new root's subtree (k_compact / k_compact_log: blocks moved,
    overflow map rebuilt, particle log filtered and relabelled) and every tree
    stays bit-exact with the oracle, whose tree is never compacted.  In each
    re-root scan: the streaming one (k_log_filter + the materialising pass), the
    same with the filter classifying from the global block maps (the path of
    logs whose maps do not fit the packed table), and the one-workgroup-per-log
    k_compact_log (POMCP_LOG_SCAN=legacy)."""
    if scan == "legacy":
        monkeypatch.setenv("POMCP_LOG_SCAN", "legacy")
    if scan == "stream_global_cmap":
        monkeypatch.setenv("POMCP_LF_PACKED_CMAP", "off")
    from posggym_baselines_amd.planning.engine import plan_capacities
    from posggym_baselines_amd.planning import MCTSConfig
    from gpu_util import batched_episodes
    S, steps, B = 64, 8, 70
    cfg = MCTSConfig(num_sims=S, **TEST_CFG)
    caps = plan_capacities(cfg, 50, S, 2, num_actions=5, overflow_slots=64)
    # one search plus the kept subtree (the new root and its expanded children,
    # at most its visits): no room for 8 searches without compaction
    caps.max_blocks = S + S // 2 + 16
    levels = cfg.depth_limit + 1
    caps.max_particles = 2 * S * levels + 2 * (cfg.num_particles + cfg.extra_particles) + 64
    caps.log_table_size = S * (steps + 1) + 2   # math.log(N): root visits accumulate
    from oracle.run import oracle_episode
    usage, seeds, exp = [], [], []
    s = 7000
    while len(seeds) < B:   # planners whose episodes last >= steps (searched every step)
        trace, recs = oracle_episode(TEST_CFG, S, s, tree=len(seeds), max_steps=steps)
        if trace["len"] >= steps and all(r["searched"] and r["num_sims"] for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    got = batched_episodes(TEST_CFG, S, seeds, steps, capacities=caps, usage=usage)
    for b in range(B):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"
    before = [u for k, u in usage if k == "before_update"][1:]
    after = [u for k, u in usage if k == "after_update"][1:]
    assert all(a[0] < bb[0] and a[1] < bb[1] for a, bb in zip(after, before)), (before, after)
    assert sum(bb[1] for bb in before) > 2 * caps.max_particles   # several logs' worth in all


def test_wall_clock_episode_one_second():
    """The reference's default mode (num_sims=None, mcts.py:285) over a full
    Driving-v1 episode at search_time_limit=1.0 (exp_utils.py:27 budgets): the
    arenas are sized from the time limit, compacted at every update, and the
    chunk loop never overflows them."""
    from oracle.episode import run_episode
    from posggym_baselines_amd.planning import MCTSConfig, POMCP, RandomSearchPolicy
    from gpu_util import product_model
    model = product_model("Driving-v1")
    cfg = MCTSConfig(**dict(TEST_CFG, search_time_limit=1.0))
    planner = POMCP(model, "0", cfg, RandomSearchPolicy(model, "0"))
    planner.reset()
    sims = []

    def step(obs):
        a = planner.step(obs)
        if not planner.root.is_absorbing:
            st = planner.step_statistics
            assert not st.get("arena_full"), len(sims)
            assert 0.9 <= st["search_time"] < 3.0
            sims.append(st["num_sims"])
        return a

    trace = run_episode(step, 31, max_steps=50)
    assert trace["len"] >= 3 and min(sims) > 1000
    planner.close()


@pytest.mark.parametrize("time_limit", [1.0, 20.0])
def test_reinvigoration_many_particles(time_limit):
    """The rejection reinvigoration (mcts.py:651-700, belief.py:145-194) at the
    reference's particle counts for 1 s and 20 s budgets (100 + 7 and 2000 + 125
    particles, config.py:47-48): k_update runs 64 tries per pass (one per lane,
    ballot-ranked accepts / rejects); beliefs equal the oracle's, insertion order
    included (belief digests), over 3 real steps."""
    from gpu_util import batched_episodes
    from oracle.run import oracle_episode
    cfg = dict(TEST_CFG, search_time_limit=time_limit)
    S, K, B = 32, 3, 5
    seeds, exp = [], []
    s = 9100
    while len(seeds) < B:   # (a root that turned absorbing is not reinvigorated: skip)
        trace, recs = oracle_episode(cfg, S, s, tree=len(seeds), max_steps=K)
        if trace["len"] >= K and all(r["searched"] and r.get("num_sims") for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    got = batched_episodes(cfg, S, seeds, K)
    for b in range(B):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"
        assert got[b][-1]["belief_size"] >= 100


def test_search_from_host_belief():
    """pomcp_set_root_belief: a fresh planner searches from caller-supplied
    particles (another planner's b0 particles, insertion order kept) and then
    re-roots as usual; both steps equal the oracle holding the same belief."""
    from oracle.envs import make_model
    from oracle.rng import Streams
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    from gpu_util import product_model
    donor = make_oracle(TEST_CFG, 8, tree=9)
    run_episode(lambda obs: (donor.update(None, obs), 0)[1], 55, max_steps=1)
    parts = list(donor.belief[donor.root])
    rows = [(t,) + tuple(donor.model.pack_words(st)) for st, t in parts]
    S = 300
    model = product_model("Driving-v1")
    planner = POMCP(model, "0", product_config(TEST_CFG, S), RandomSearchPolicy(model, "0"))
    planner.reset()
    planner.set_root_belief(rows)
    p = make_oracle(TEST_CFG, S, tree=0)
    node = p._new_obs_node(rows[0][0], 0)
    p.belief[node] = list(parts)
    p.root = node

    def both_records(a, b):
        p.stats["searched"] = True
        p.stats["belief"] = list(p.belief[p.root])
        st = planner._engine.root_stats()[0]
        return (stats_record(st, 5, True, a, planner.root_belief()), oracle_record(p, True, b))

    a = planner.get_action()
    p.stats = {}
    b = p.get_action()
    got, exp = both_records(a, b)
    assert got == exp
    # one real step on: an observation from the belief's first particle
    env = make_model("Driving-v1", Streams(77, 0x40000000))
    obs = env.step(parts[0][0], {"0": a, "1": 0}).observations["0"]
    planner.update(a, obs)
    p.stats = {}
    p.update(b, obs)
    a2, b2 = planner.get_action(), p.get_action()
    got, exp = both_records(a2, b2)
    assert got == exp
    planner.close()


def test_search_kernel_override_is_used(search_kernel):
    from gpu_util import product_model
    from posggym_baselines_amd.planning import BatchedPOMCP
    bp = BatchedPOMCP(product_model("Driving-v1"), "0", product_config(TEST_CFG, 16), 3, 16)
    assert bp.engine.search_kernel() == search_kernel
    bp.close()


def test_deep_tree_beyond_the_lds_pool():
    """gamma 0.99 / epsilon 0.01 (depth_limit 459): a 1,500-simulation search
    expands ~one block per simulation, far past the wave kernel's LDS pool
    (224 blocks for A = 5): the blocks beyond it are read and written in HBM.
    Bit-exact against the oracle either way; a second step re-roots into the
    big tree (compaction moves blocks across the LDS / HBM boundary)."""
    from gpu_util import batched_episodes
    from oracle.run import oracle_episode
    cfg = dict(TEST_CFG, discount=0.99, epsilon=0.01, seed=21)
    S, K = 1500, 2
    seeds, exp = [], []
    s = 610
    while len(seeds) < 2:
        trace, recs = oracle_episode(cfg, S, s, tree=len(seeds), max_steps=K)
        if trace["len"] >= K and all(r["searched"] for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    usage = []
    got = batched_episodes(cfg, S, seeds, K, usage=usage)
    for b in range(len(seeds)):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"
    assert max(u[0] for k, u in usage) > 300   # blocks in use: beyond the LDS pool


def test_late_step_tree_handoff_falls_back():
    """k_search_lds with its step-tree producers (wave_tree): when a hand-off is
    late the search wave stops the producers and computes the rest of the
    launch itself -- never an error.  With the wait bounded at one poll, most
    searches fall back at once; 12 planners over 3 real steps stay bit-exact
    against the oracle."""
    from gpu_util import batched_episodes
    from oracle.run import oracle_episode
    S, K = 256, 3
    seeds, exp = [], []
    s = 700
    while len(seeds) < 12:
        trace, recs = oracle_episode(TEST_CFG, S, s, tree=len(seeds), max_steps=K)
        if trace["len"] >= K and all(r["searched"] and r["num_sims"] > 0 for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    got = batched_episodes(TEST_CFG, S, seeds, K, spin_limit=1)
    for b in range(len(seeds)):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"


def _pe_oracle_episodes(cfg, S, K, B, s0):
    from oracle.run import oracle_episode
    seeds, exp = [], []
    s = s0
    while len(seeds) < B:   # planners whose episodes last >= K steps, searched every step
        trace, recs = oracle_episode(cfg, S, s, tree=len(seeds), max_steps=K,
                                     env="PursuitEvasion-v1")
        if trace["len"] >= K and all(r["searched"] and r.get("num_sims") for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    return seeds, exp


@pytest.mark.parametrize("islots", [6, 2])
def test_pursuit_evasion_batched_reroot(search_kernel, islots):
    """PursuitEvasion-v1 planners over 5 real steps in one engine: re-root,
    extraction, reinvigoration and subtree compaction after every search.  In
    the "lane" mode the cut-off children are deferred and materialised by
    k_compact_log from the records (Env::obs_key / Env::done_of of
    PursuitEvasion), in "lane_eager" they are looked up during the search;
    with 2 inline slots most children go through the overflow map (deferred
    ones inserted by the re-root).  Bit-exact against the oracle every step."""
    import os
    from gpu_util import batched_episodes
    cfg = dict(TEST_CFG, seed=11)
    S, K, B = 160, 5, 40
    seeds, exp = _pe_oracle_episodes(cfg, S, K, B, 8800)
    counters = []
    got = batched_episodes(cfg, S, seeds, K, env="PursuitEvasion-v1", inline_slots=islots,
                           counters=counters)
    for b in range(B):
        assert got[b] == exp[b], f"tree {b} (env seed {seeds[b]})"
    deferred = sum(c[1] for c in counters)
    cut = sum(c[2] for c in counters)
    if search_kernel == "lane":
        if os.environ.get("POMCP_DEFER_CUTOFF") == "1":
            assert deferred > 0 and deferred == cut, counters
        else:
            assert deferred == 0 and cut > 0, counters


def test_exact_selection_fallback_fires_and_is_exact(search_kernel):
    """k_search's fast UCB / PUCB selection falls back to the exact FP64 scores
    near a tie (DESIGN.md §4 "Fast selection").  With the margin widened to
    1e-4 (pomcp_debug_set_select_margin) that path decides a large share of the
    selections; the reference goldens (UCB, PUCB, deep, PursuitEvasion), a
    65,536-simulation search and re-rooting batched planners stay bit-exact and
    the lane kernel counts the exact-path selections (n_exact_selects).  The
    wave kernel always scores exactly (its count is 0)."""
    from gpu_util import batched_episodes
    from oracle.run import oracle_episode
    lane = search_kernel == "lane"
    for case in ("c1_ucb", "c1_pucb", "deep_ucb", "pe_evader_ucb", "pe_pursuer_pucb"):
        data = load(case)
        ep = data["episodes"][0]
        exact = []
        trace, records = gpu_episode(cfg_kwargs(ep["config"]), data["num_sims"], ep["env_seed"],
                                     ego=data["ego"], max_steps=case_max_steps(case, data),
                                     env=case_env(data), select_margin=1e-4, exact=exact)
        assert records == ep["records"], case
        assert trace == ep["trace"], case
        assert (sum(exact) > 0) == lane, (case, exact)
    stats = _batched_vs_oracle(TEST_CFG, 2, 65536, [0], select_margin=1e-4)
    sel = sum(int(st.n_exact_selects) for st in stats)
    assert (sel > 1000) == lane, sel
    cfg = dict(TEST_CFG, action_selection="pucb", seed=4)
    S, K = 128, 4
    seeds, exp = [], []
    s = 5100
    while len(seeds) < 24:
        trace, recs = oracle_episode(cfg, S, s, tree=len(seeds), max_steps=K)
        if trace["len"] >= K and all(r["searched"] for r in recs):
            seeds.append(s)
            exp.append(recs)
        s += 1
    counters = []
    got = batched_episodes(cfg, S, seeds, K, select_margin=1e-4, counters=counters)
    assert got == exp
    assert (sum(c[0] for c in counters) > 0) == lane, counters


def test_select_margin_below_the_error_bound_is_rejected():
    from gpu_util import product_model
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning import BatchedPOMCP
    bp = BatchedPOMCP(product_model("Driving-v1"), "0", product_config(TEST_CFG, 16), 3, 16)
    lib = N.load()
    assert lib.pomcp_debug_set_select_margin(bp.engine._ctx, 1e-13) == N.POMCP_E_INVALID
    assert lib.pomcp_debug_set_select_margin(bp.engine._ctx, float("nan")) == N.POMCP_E_INVALID
    assert lib.pomcp_debug_set_select_margin(bp.engine._ctx, 1e-12) == 0
    bp.close()


def test_mode_change_with_pending_deferred_records_is_refused(search_kernel):
    """Deferred cut-off records take their absorbing flag from the last record at
    the re-root; an eager arrival in between could be overwritten (mcts.py:370's
    last arrival must win).  So while a lane search's deferred records are
    pending, switching deferral or the kernel is refused (POMCP_E_STATE); an
    update / restore / reset clears them."""
    import numpy as np
    from gpu_util import product_model
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning import BatchedPOMCP
    if search_kernel != "lane":
        pytest.skip("lane kernel")
    bp = BatchedPOMCP(product_model("Driving-v1"), "0", product_config(TEST_CFG, 64), 4, 64,
                      searches=3, reroot=True, defer_cutoff=True)
    bp.engine._defer_forced = False
    bp.init_synthetic(1000)
    lib, ctx = N.load(), bp.engine._ctx
    assert lib.pomcp_set_defer_cutoff(ctx, 1) == 0
    acts = bp.search()
    assert sum(int(s.n_deferred) for s in bp.engine.root_stats()) > 0
    assert lib.pomcp_set_defer_cutoff(ctx, 0) == N.POMCP_E_STATE
    assert lib.pomcp_set_search_kernel(ctx, N.SEARCH_WAVE) == N.POMCP_E_STATE
    assert lib.pomcp_set_defer_cutoff(ctx, 1) == 0            # no change: allowed
    assert lib.pomcp_set_search_kernel(ctx, N.SEARCH_LANE) == 0
    bp.engine.update(acts, bp.engine.synthetic_step(1000, acts))
    assert lib.pomcp_set_defer_cutoff(ctx, 0) == 0
    bp.search()
    assert sum(int(s.n_deferred) for s in bp.engine.root_stats()) == 0
    assert lib.pomcp_set_defer_cutoff(ctx, 1) == 0   # eager records: nothing pending
    bp.close()


def test_step_statistics_hbm_bytes_and_rate(search_kernel):
    """the drop-in keeps the reference's step_statistics keys
    (mcts.py:140-153) and adds hbm_bytes (the search's algorithmic bytes from
    the kernel's counters, engine.search_bytes -- bench.py's roofline
    numerator) and sims_per_s."""
    from gpu_util import product_model
    from posggym_baselines_amd.planning import POMCP, RandomSearchPolicy
    from posggym_baselines_amd.planning.engine import b_level, search_bytes
    model = product_model("Driving-v1")
    S = 512
    planner = POMCP(model, "0", product_config(TEST_CFG, S), RandomSearchPolicy(model, "0"))
    planner.reset()
    obs = model.sample_initial_obs(model.sample_initial_state())
    planner.step(obs["0"])
    st = planner.step_statistics
    assert {"search_time", "update_time", "reinvigoration_time", "evaluation_time",
            "policy_calls", "inference_time", "search_depth", "num_sims", "mem_usage",
            "min_value", "max_value"} <= set(st)
    rs = planner._engine.root_stats()
    assert st["hbm_bytes"] == search_bytes(rs, 5) > 0
    assert st["hbm_bytes"] >= 16 * S + (b_level(5) - 28) * int(rs[0].n_levels)
    assert st["sims_per_s"] == pytest.approx(S / st["search_time"])
    planner.close()
