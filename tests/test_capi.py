"""C-ABI boundary checks that need no GPU: the shared object loads, exports
every symbol include/*.h declares, and the ctypes structs match the C layout."""
import ctypes
import os
import re
import subprocess

import pytest

from posggym_baselines_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("pomcp.h", "pomcp_debug.h",
                                                                  "intmcp.h")]


def declared_functions():
    names = []
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:int|void|int32_t|const char\s*\*)\s+((?:pomcp|intmcp)_\w+)\s*\(", src, re.M)
    return names


def test_library_exports_every_declared_symbol():
    lib = N.load()
    names = declared_functions()
    assert len(names) >= 19
    for n in names:
        assert hasattr(lib, n), n
    bound = {s[0] for s in N.SIGNATURES + N.DEBUG_SIGNATURES + N.INTMCP_SIGNATURES}
    assert set(names) == bound
    assert lib.pomcp_abi_version() == N.POMCP_ABI_VERSION


def test_struct_layout_matches_header(tmp_path):
    probe = tmp_path / "probe.c"
    fields = {
        "pomcp_config": [f[0] for f in N.PomcpConfig._fields_],
        "pomcp_root_stats": [f[0] for f in N.PomcpRootStats._fields_],
        "pomcp_grid": [f[0] for f in N.PomcpGrid._fields_],
        "pomcp_pe_grid": [f[0] for f in N.PomcpPeGrid._fields_],
        "pomcp_merged_root": [f[0] for f in N.PomcpMergedRoot._fields_],
        "pomcp_type_policies": [f[0] for f in N.PomcpTypePolicies._fields_],
        "intmcp_config": [f[0] for f in N.IntmcpConfig._fields_],
        "intmcp_root_stats": [f[0] for f in N.IntmcpRootStats._fields_],
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "intmcp.h"', "int main(void){"]
    for st, fs in fields.items():
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    probe.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(probe), "-o",
                    str(exe)], check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.run(
        [str(exe)], check=True, capture_output=True, text=True).stdout.split("\n") if line)
    for st, cls in (("pomcp_config", N.PomcpConfig), ("pomcp_root_stats", N.PomcpRootStats),
                    ("pomcp_grid", N.PomcpGrid), ("pomcp_pe_grid", N.PomcpPeGrid),
                    ("pomcp_merged_root", N.PomcpMergedRoot),
                    ("pomcp_type_policies", N.PomcpTypePolicies),
                    ("intmcp_config", N.IntmcpConfig), ("intmcp_root_stats", N.IntmcpRootStats)):
        assert int(out[st]) == ctypes.sizeof(cls), st
        for f in fields[st]:
            assert int(out[f"{st}.{f}"]) == getattr(cls, f).offset, f"{st}.{f}"


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import POMCP, MCTSConfig, RandomSearchPolicy
    m = DrivingModel()
    cfg = MCTSConfig(discount=0.95, search_time_limit=0.1, c=1.4, truncated=False,
                     action_selection="ucb", epsilon=0.92, seed=0, state_belief_only=True,
                     num_sims=16)
    with pytest.raises(N.PomcpError):
        POMCP(m, "0", cfg, RandomSearchPolicy(m, "0"))


def test_engine_rejects_unsupported_search_policy():
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import POMCP, MCTSConfig, SearchPolicy

    class Other(SearchPolicy):
        def get_initial_state(self): return {}
        def get_next_state(self, a, o, s): return {}
        def sample_action(self, s): return 0
        def get_pi(self, s): return {}
        def get_value(self, s): return 0.0

    m = DrivingModel()
    cfg = MCTSConfig(discount=0.95, search_time_limit=0.1, c=1.4, truncated=False, seed=0)
    with pytest.raises(NotImplementedError):
        POMCP(m, "0", cfg, Other(m, "0", "x"))


def test_ipomcp_validates_other_agent_policies():
    """IPOMCP / MCTS (ipomcp.py:11-38, mcts.py:22-91): every other agent needs a
    policy; random and fixed-distribution policies run in-kernel, others raise
    (checked before any GPU use)."""
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import (IPOMCP, MCTS, MCTSConfig, OtherAgentPolicy,
                                                RandomSearchPolicy)

    class Scripted(OtherAgentPolicy):
        def sample_initial_state(self): return {}
        def get_next_state(self, a, o, s): return {}
        def sample_action(self, s): return 0
        def get_pi(self, s): return {0: 1.0}

    m = DrivingModel()
    cfg = MCTSConfig(discount=0.95, search_time_limit=0.1, c=1.4, truncated=False, seed=0,
                     state_belief_only=False, num_sims=16)
    for cls in (IPOMCP, MCTS):
        with pytest.raises(AssertionError):
            cls(m, "0", cfg, {}, RandomSearchPolicy(m, "0"))
        with pytest.raises(NotImplementedError):
            cls(m, "0", cfg, {"1": Scripted(m, "1")}, RandomSearchPolicy(m, "0"))


def test_episode_results_header_matches_reference(tmp_path):
    """episode_results.csv columns of run_planning_exp (exp_utils.py:325-331)."""
    from posggym_baselines_amd.planning.episodes import EPISODE_RESULT_HEADS, EpisodeResultsWriter
    assert EPISODE_RESULT_HEADS == [
        "num", "len", "return", "discounted_return", "time", "search_time", "update_time",
        "reinvigoration_time", "evaluation_time", "policy_calls", "inference_time",
        "search_depth", "num_sims", "mem_usage", "min_value", "max_value"]
    w = EpisodeResultsWriter(str(tmp_path / "episode_results.csv"))
    w({k: 1 for k in EPISODE_RESULT_HEADS})
    lines = open(tmp_path / "episode_results.csv").read().splitlines()
    assert lines[0].split(",") == EPISODE_RESULT_HEADS and len(lines) == 2


def test_host_philox_words_match_the_oracle():
    """pomcp_philox_words (the episode loop's random agents) == oracle/rng.py."""
    import ctypes
    from oracle.rng import Streams
    out = (ctypes.c_uint32 * 8)()
    assert N.load().pomcp_philox_words(7, 0x40000000, 41, 0, 8, out) == 0
    s = Streams(7, 0x40000000)
    assert list(out) == [s.u32(41) for _ in range(8)]


def test_episode_loop_replays_golden_trajectories_on_cpu():
    """run_planning_episodes with a planner that replays the reference planner's
    recorded actions: the host environment (same driving.h / pursuit_evasion.h
    through the C ABI) and the random other agents reproduce the golden
    trajectories exactly (other agent's actions, rewards, length, return)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import load
    from oracle.episode import fhex
    from posggym_baselines_amd.envs import DrivingModel, PursuitEvasionModel
    from posggym_baselines_amd.planning.episodes import run_planning_episodes

    class Replay:
        class config:
            discount = 0.95

        def __init__(self, actions):
            self.actions, self.t = actions, 0

            class _T:
                def get_episode(self_inner):
                    return {}
            self.stat_tracker = _T()

        def reset(self):
            self.t = 0

        def step(self, obs):
            a = self.actions[self.t]
            self.t += 1
            return a

    for case, Model in (("c1_ucb", DrivingModel), ("c1_pucb", DrivingModel),
                        ("pe_evader_ucb", PursuitEvasionModel)):
        data = load(case)
        ego = int(data["ego"])
        for ep in data["episodes"]:
            steps = ep["trace"]["steps"]
            seen = []
            rows = run_planning_episodes(
                Replay([s["actions"][ego] for s in steps]), Model(), 1, data["ego"],
                env_seeds=[ep["env_seed"]], until="all_done",
                on_step=lambda t, o, acts, ts: seen.append(
                    ([acts[i] for i in sorted(acts)], fhex(ts.rewards[data["ego"]]))))
            assert [s[0] for s in seen] == [s["actions"] for s in steps], case
            assert [s[1] for s in seen] == [s["reward"] for s in steps], case
            assert rows[0]["len"] == ep["trace"]["len"]
            assert fhex(rows[0]["return"]) == ep["trace"]["return"]
