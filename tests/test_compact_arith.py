"""Integer identities the re-root kernels rely on (CPU, no GPU).

k_compact_log (csrc/pomcp_kernels.hip) divides action-node indices by the
action count with a multiply: x / A == (x * ceil(2^32 / A)) >> 32 for every
x below the node-id bound 2^26 (pomcp_create refuses larger arenas) and every
action count the search kernels accept (2..5, pomcp_capi.hip).  Checked here
over the whole range.
"""
import numpy as np

ID_BOUND = 1 << 26   # kIdBits (pomcp_device.h)


def test_divide_by_action_count_with_a_multiply_is_exact():
    for a in range(1, 6):
        m = np.uint64(((1 << 32) + a - 1) // a)
        for s in range(0, ID_BOUND, 1 << 24):
            x = np.arange(s, s + (1 << 24), dtype=np.uint64)
            q = (x * m) >> np.uint64(32)
            assert np.array_equal(q, x // np.uint64(a)), a
