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


def _batched_vs_oracle(cfg, num_trees, num_sims, check_trees, rekey=None, env="Driving-v1"):
    from gpu_util import product_model
    from posggym_baselines_amd.planning import BatchedPOMCP
    model = product_model(env)
    A = model.action_spaces["0"].n
    bp = BatchedPOMCP(model, "0", product_config(cfg, num_sims), num_trees, num_sims)
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
