"""Oracle pinning: the CPU restatement against the reference's golden vectors."""
import pytest

from golden_util import (EPISODE_CASES, IPOMCP_CASES, case_env, case_max_steps, cfg_kwargs, load,
                         search_probs)
from oracle.pomcp import OracleConfig
from oracle.rng import PHILOX_ROUNDS, Streams, StreamRandom, philox4x32, philox4x32_10
from oracle.run import oracle_episode


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32 7 rounds (the build's streams since
    # round 6, csrc/philox.h) ...
    assert PHILOX_ROUNDS == 7
    assert philox4x32(0, 0, 0, 0, 0, 0) == (0x5F6FB709, 0x0D893F64, 0x4F121F81, 0x4F730A48)
    assert philox4x32(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344,
                      0xA4093822, 0x299F31D0) == (0x4DFCCABA, 0x190A87F0, 0xC47362BA, 0xB6B5242A)
    # ... and for philox4x32_10 (the same round function run 10 rounds)
    assert philox4x32_10(0, 0, 0, 0, 0, 0) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    m = 0xFFFFFFFF
    assert philox4x32_10(m, m, m, m, m, m) == (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)
    assert philox4x32_10(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344,
                         0xA4093822, 0x299F31D0) == (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)


def test_stream_layout():
    s = Streams(5, 3)
    words = [s.u32(1) for _ in range(6)]
    b0 = philox4x32(0, 0, 1, 0, 5, 3)
    b1 = philox4x32(1, 0, 1, 0, 5, 3)
    assert words == list(b0) + list(b1[:2])
    assert s.counters() == {1: 6}
    # randint is a multiply-shift of one word
    s2 = Streams(5, 3)
    assert [s2.randint(1, 7) for _ in range(6)] == [(w * 7) >> 32 for w in words]


def test_stream_random_choices_matches_cpython_arithmetic():
    """random.choices: cum_weights via accumulate, bisect(cum, random()*total, 0, n-1)."""
    import bisect
    import itertools

    w = [0.2] * 5
    cum = list(itertools.accumulate(w))
    sr = StreamRandom(Streams(1, 2), 1)
    ref = Streams(1, 2)
    for _ in range(200):
        got = sr.choices(list(range(5)), weights=w, k=1)[0]
        exp = bisect.bisect(cum, ref.random(1) * (cum[-1] + 0.0), 0, 4)
        assert got == exp


def test_config_kats():
    for row in load("config_kats"):
        kw = dict(discount=row["discount"], search_time_limit=row["search_time_limit"], c=1.0,
                  epsilon=row["epsilon"], extra_particles_prop=row["extra_particles_prop"])
        if "raises" in row:
            with pytest.raises(ZeroDivisionError):
                OracleConfig(num_sims=1, **kw)
            continue
        c = OracleConfig(num_sims=1, **kw)
        assert (c.num_particles, c.extra_particles, c.depth_limit) == (
            row["num_particles"], row["extra_particles"], row["depth_limit"])


@pytest.mark.parametrize("case", EPISODE_CASES + IPOMCP_CASES)
def test_oracle_matches_reference_goldens(case):
    data = load(case)
    for ep in data["episodes"]:
        # IPOMCP cases: the reference ran with histories in the particles; the
        # POMCP restatement (state beliefs) must give the same records
        kw = dict(cfg_kwargs(ep["config"]), state_belief_only=True)
        trace, records = oracle_episode(kw, data["num_sims"], ep["env_seed"], ego=data["ego"],
                                        max_steps=case_max_steps(case, data),
                                        env=case_env(data))
        assert trace == ep["trace"]
        assert len(records) == len(ep["records"])
        for t, (got, exp) in enumerate(zip(records, ep["records"])):
            assert got == exp, f"{case} step {t}"


@pytest.mark.parametrize("case", ["intmcp_ucb", "intmcp_ego1", "intmcp_uniform", "intmcp_deep",
                                  "intmcp_pe", "intmcp0_ucb", "intmcp0_ego1_uniform",
                                  "intmcp0_deep", "intmcp0_pe", "intmcp_sp_ucb",
                                  "intmcp0_sp_ego1", "intmcp_sp_pe", "intmcp2_ucb",
                                  "intmcp2_ego1_uniform", "intmcp2_pe", "intmcp2_sp_ucb",
                                  "intmcp3_ucb", "intmcp3_pe", "intmcp4_ucb", "intmcp4_pe",
                                  "intmcp5_ucb"])
def test_intmcp_oracle_matches_reference_goldens(case):
    """I-NTMCP nesting 1 (BASELINE config 5) and nesting 0: the oracle
    restatement against the real reference planner's records (root children,
    beliefs with the other agent's histories, the level-0 nodes of every history
    in the belief; at nesting 0 the single tree and its belief)."""
    from oracle.run import oracle_intmcp_episode
    data = load(case)
    for ep in data["episodes"]:
        trace, records = oracle_intmcp_episode(ep["config"], data["num_sims"], ep["env_seed"],
                                               ego=data["ego"], max_steps=data["max_steps"],
                                               env=case_env(data),
                                               nesting_level=data.get("nesting_level", 1),
                                               search_probs=search_probs(data))
        assert trace == ep["trace"]
        for t, (got, exp) in enumerate(zip(records, ep["records"])):
            assert got == exp, f"{case} step {t}"
        assert len(records) == len(ep["records"])


def test_intmcp_depleted_branch_unreachable_for_valid_configs():
    """intmcp.py:421-431 reinvigorates a depleted belief at search time (root
    below extra_particles, or an empty level-0 node).  With the reference's own
    BeliefRejectionSampler (belief.py:85 asserts sample_limit_factor >= 1, and
    use_rejected_samples=True fills up with rejected samples) every update leaves
    the level-1 root with num_particles + extra_particles >= extra_particles and
    every non-absorbing level-0 support node with ceil(p * target) >= 1
    particles, and an absorbing node always holds the particle of the visit
    that marked it -- so the branch cannot fire (the GPU engine
    reports POMCP_E_UNSUPPORTED if it ever did).  Checked here on the extreme
    valid settings (every particle an extra one, the minimum try budget)."""
    import math
    import oracle.intmcp as OI
    from oracle.run import oracle_intmcp_episode
    hits = []
    orig = OI._Planner._nested_sim

    def spy(self, n, search_level, top_level):
        size = len(self.tree.belief[n])
        if size == 0 or (top_level and size < self.cfg.extra_particles):
            hits.append((self.level, size))
        return orig(self, n, search_level, top_level)

    OI._Planner._nested_sim = spy
    try:
        cfg = dict(discount=0.95, search_time_limit=0.2, c=math.sqrt(2), truncated=False,
                   action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                   step_limit=None, epsilon=0.92, seed=2, state_belief_only=False,
                   extra_particles_prop=1.0, reinvigoration_sample_limit_factor=1.0)
        oracle_intmcp_episode(cfg, 16, 2, ego="0", max_steps=50)
        oracle_intmcp_episode(dict(cfg, action_selection="uniform", seed=5), 16, 5, ego="1",
                              max_steps=40, env="PursuitEvasion-v1")
    finally:
        OI._Planner._nested_sim = orig
    assert hits == []


@pytest.mark.parametrize("name", ["im_drv_ucb_48", "im_pe_uniform_48", "im_drv_ucb_256",
                                  "im_pe_ucb_256"])
def test_oracle_digests_fixture(name):
    """tests/golden/oracle_digests.json (the GPU suite compares every batched
    I-NTMCP pair against it): a sample of its per-pair digests recomputed from
    the oracle here."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_oracle_digests import CASES, oracle_pair, record_digest
    fx = load("oracle_digests")[name]
    assert {k: v for k, v in fx.items() if k != "digests"} == CASES[name]
    n = CASES[name]["pairs"]
    for b in sorted({0, 1, 63, 64, n // 2, n - 1}):
        assert record_digest(oracle_pair(CASES[name], b)) == fx["digests"][b], f"pair {b}"
