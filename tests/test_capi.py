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
    policy; only RandomOtherAgentPolicy runs in-kernel (checked before any GPU use)."""
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
