"""host_exp (csrc/host_exp.h), the exp of I-NTMCP's other-agent softmax
(intmcp.py:782-790), equals Python's math.exp bit for bit.

This is the host build of the same function the GPU kernel runs; the GPU side
is checked against math.exp in tests/test_gpu_intmcp.py.  Arguments: every
v / sqrt(N) the softmax can see for N <= 4096 (all v <= N), a sample of it up
to N = 65,536, random arguments over the whole finite range, and the special
cases (0, subnormals, |x| >= 512, overflow / underflow, inf, nan)."""
import ctypes as C
import math
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def softmax_arguments(rng, full_n=4096, sampled_n=65536, per_n=48):
    xs = []
    for n in range(1, full_n + 1):
        xs.append(np.arange(n + 1, dtype=np.float64) / math.sqrt(n))
    for n in rng.integers(full_n, sampled_n + 1, 20000):
        v = rng.integers(0, n + 1, per_n)
        xs.append(v.astype(np.float64) / math.sqrt(float(n)))
    return np.concatenate(xs)


def special_arguments(rng):
    edge = [0.0, -0.0, 5e-324, -5e-324, 2.0**-54, -2.0**-54, 2.0**-53, 2.0**-1022,
            511.999, 512.0, -512.0, 700.0, 709.78, 709.79, -700.0, -745.0, -745.2, -1000.0,
            1023.9, 1024.0, -1024.0, 1e300, -1e300, math.inf, -math.inf]
    wide = rng.uniform(-745.0, 709.0, 200000)
    tiny = rng.uniform(-1, 1, 20000) * 2.0 ** rng.integers(-70, -40, 20000)
    return np.concatenate([np.array(edge), wide, tiny])


def _py_exp(x):
    out = np.empty_like(x)
    for i, v in enumerate(x.tolist()):
        try:
            out[i] = math.exp(v)
        except OverflowError:
            out[i] = math.inf
    return out


def _same(a, b):
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


def test_host_exp_equals_math_exp():
    from posggym_baselines_amd import _native as N
    lib = N.load()
    rng = np.random.default_rng(0)
    x = np.concatenate([softmax_arguments(rng), special_arguments(rng)])
    out = np.zeros_like(x)
    P = C.POINTER(C.c_double)
    assert lib.pomcp_debug_host_exp(x.ctypes.data_as(P), len(x), out.ctypes.data_as(P)) == 0
    ref = _py_exp(x)
    bad = np.nonzero(~_same(out, ref))[0]
    assert len(x) > 9_000_000
    assert len(bad) == 0, [(x[i].hex(), out[i].hex(), ref[i].hex()) for i in bad[:5]]
    # nan propagates
    nan = np.array([math.nan])
    assert lib.pomcp_debug_host_exp(nan.ctypes.data_as(P), 1, out.ctypes.data_as(P)) == 0
    assert math.isnan(out[0])


def test_exp_table_is_the_hosts():
    """The generated table (from its definition) equals the host libm's."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_exp_table.py"),
                        "--check-only"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_host_log_table_equals_math_log():
    """The planner's log(N) table (engine.log_table, mcts.py:534's
    math.log(N)) comes from pomcp_host_log_table, the C library's log: equal to
    Python's math.log bit for bit on every N < 2^21, on a sample up to 2^31,
    and across an offset start."""
    from posggym_baselines_amd import _native as N
    lib = N.load()
    P = C.POINTER(C.c_double)
    n = 1 << 21
    out = np.zeros(n)
    assert lib.pomcp_host_log_table(0, n, out.ctypes.data_as(P)) == 0
    ref = np.array([0.0] + [math.log(i) for i in range(1, n)])
    assert np.array_equal(out.view(np.uint64), ref.view(np.uint64))
    rng = np.random.default_rng(3)
    for first in rng.integers(1, 2**31 - 4096, 64):
        seg = np.zeros(4096)
        assert lib.pomcp_host_log_table(int(first), 4096, seg.ctypes.data_as(P)) == 0
        exp = np.array([math.log(int(first) + k) for k in range(4096)])
        assert np.array_equal(seg.view(np.uint64), exp.view(np.uint64))
