"""GPU parity of the I-NTMCP engine (BASELINE config 5) through the C ABI:
every step record of the reference goldens (level-1 root statistics, root
particles with the other agent's histories, every level-0 node those histories
name: visits, children, particles) must match bit for bit."""
import pytest

from golden_util import INTMCP_CASES, cfg_kwargs, load
from gpu_util import gpu_intmcp_episode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", INTMCP_CASES)
def test_gpu_intmcp_matches_reference_goldens(case):
    data = load(case)
    for ep in data["episodes"]:
        kw = cfg_kwargs(ep["config"])
        trace, records = gpu_intmcp_episode(kw, data["num_sims"], ep["env_seed"],
                                            ego=data["ego"], max_steps=data["max_steps"],
                                            env=data["env"])
        assert len(records) == len(ep["records"]), case
        for t, (got, exp) in enumerate(zip(records, ep["records"])):
            assert got == exp, f"{case} env_seed {ep['env_seed']} step {t}"
        assert trace == ep["trace"]


TEST_CFG = dict(discount=0.95, search_time_limit=0.1, c=2 ** 0.5, truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, seed=3, state_belief_only=False)


@pytest.mark.parametrize("env,ego,sel", [("Driving-v1", "0", "ucb"),
                                         ("PursuitEvasion-v1", "1", "uniform")])
def test_batched_pairs_match_oracle(env, ego, sel):
    """150 planner pairs (3 launch blocks) in one engine, lockstep episodes:
    pair b equals the oracle planner with tree key b."""
    from gpu_util import batched_intmcp_episodes
    from oracle.run import oracle_intmcp_episode
    cfg = dict(TEST_CFG, action_selection=sel)
    seeds = [500 + b for b in range(150)]
    steps, sims = 4, 48
    got = batched_intmcp_episodes(cfg, sims, seeds, steps, env=env, ego=ego)
    for b in (0, 1, 63, 64, 100, 127, 128, 149):
        _, exp = oracle_intmcp_episode(cfg, sims, seeds[b], ego=ego, tree=b, max_steps=steps,
                                       env=env)
        assert got[b] == exp, f"pair {b}"


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
