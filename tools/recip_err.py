"""Max relative error of the fast reciprocals (rcp_nr, rsq_nr) of the loaded
library, on every visit count up to 2^20 and random positive doubles (the
same inputs as tests/test_gpu_parity.py::test_fast_ucb_reciprocals_error_bound).
GPU box diagnostics: POMCP_LIB_PATH selects an A/B build."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd")]
from posggym_baselines_amd import _native as N  # noqa: E402

rng = np.random.default_rng(1)
x = np.concatenate([np.arange(1, 1 << 20, dtype=np.float64),
                    np.exp(rng.uniform(-30, 30, 1 << 18)), rng.uniform(1e-3, 4.0, 1 << 18)])
out = np.zeros(2 * len(x))
P = C.POINTER(C.c_double)
assert N.load().pomcp_debug_fast_recip(x.ctypes.data_as(P), len(x), out.ctypes.data_as(P)) == 0
out = out.reshape(-1, 2)
r1 = np.abs(out[:, 0] - 1.0 / x) * x
r2 = np.abs(out[:, 1] - 1.0 / np.sqrt(x)) * np.sqrt(x)
print(f"{os.path.basename(os.environ.get('POMCP_LIB_PATH') or 'in-tree')}: rcp max rel {r1.max():.3e}, "
      f"rsq max rel {r2.max():.3e}")
