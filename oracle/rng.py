"""Counter-based RNG streams (Philox4x32-7) shared by oracle, harness and HIP.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

The reference draws from four unrelated generator families:
the planner's ``random.Random(seed)`` (``mcts.py:51``, ``belief.py:55``), the
global ``random`` module (``mcts.py:496,532,555,571,581,590,600``), the
gymnasium ``Discrete.sample()`` of each agent's action space
(``search_policy.py:177``, ``other_policy.py:151``) and the model's own RNG.
The build gives each family one *stream*: draw ``j`` of stream ``s`` under key
``(seed, tree)`` is word ``j & 3`` of ``philox4x32(ctr=(j>>2 lo, j>>2 hi, s,
seed_hi), key=(seed_lo, tree))`` with ``PHILOX_ROUNDS`` = 7 rounds (rounds 1-5
of the build used 10; ``csrc/philox.h`` gives the statistical argument).  A uniform int in ``[0, n)`` is
``(u32 * n) >> 32`` and a uniform float is ``u32 * 2**-32``.  The HIP kernels
(``csrc/philox.h``) implement exactly this function.
"""

MASK32 = 0xFFFFFFFF
_M0, _M1 = 0xD2511F53, 0xCD9E8D57
_W0, _W1 = 0x9E3779B9, 0xBB67AE85

# Stream ids.  Keep in sync with csrc/philox.h.
S_BELIEF = 0        # planner random.Random(seed): belief.sample(), rejection sampling
S_SELECT = 1        # global `random` module: UCB/PUCB N==0 draws, final tie-breaks
S_MODEL = 2         # generative model RNG (initial state sampling, exec-order shuffle)
S_MIXTURE = 4       # other_policy.py `random`: OtherAgentMixturePolicy.sample_initial_state
S_ACT_BASE = 8      # Discrete(n).sample() of agent i's action space: stream 8 + i
S_ENV_MODEL = 32    # harness: the "real" environment's model RNG
S_ENV_POLICY_BASE = 40  # harness: true (non-planning) agent i's random policy: 40 + i
# The step streams of a simulation: the model's and both agents' action streams.
# Each simulation of a search (a depth-0 ``_simulate`` call, mcts.py:286-288)
# starts them at a Philox block boundary: their counters are rounded up to a
# multiple of 4 (``Streams.align_sim``), so a simulation's first four draws of
# each come from ONE block -- the HIP search computes one block per stream per
# simulation instead of one per draw (DESIGN.md §4 "Simulation-aligned
# streams").  Draws outside simulations (update, reinvigoration) are unaligned.
SIM_STREAMS = (S_MODEL, S_ACT_BASE, S_ACT_BASE + 1)


PHILOX_ROUNDS = 7


def philox4x32(c0, c1, c2, c3, k0, k1, rounds=PHILOX_ROUNDS):
    """Random123 Philox4x32 with ``rounds`` rounds (pure Python ints)."""
    for _ in range(rounds):
        p0 = _M0 * c0
        p1 = _M1 * c2
        c0, c1, c2, c3 = (
            ((p1 >> 32) ^ c1 ^ k0) & MASK32,
            p1 & MASK32,
            ((p0 >> 32) ^ c3 ^ k1) & MASK32,
            p0 & MASK32,
        )
        k0 = (k0 + _W0) & MASK32
        k1 = (k1 + _W1) & MASK32
    return c0, c1, c2, c3


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Random123's default; the known answers of the round function)."""
    return philox4x32(c0, c1, c2, c3, k0, k1, rounds=10)


class Streams:
    """Per-(seed, tree) family of independent counters."""

    __slots__ = ("seed", "tree", "_k0", "_k1", "_c3", "ctr", "_blk")

    def __init__(self, seed: int, tree: int = 0):
        self.ctr = {}
        self._blk = {}
        self.rekey(seed, tree)

    def rekey(self, seed: int, tree=None):
        """Change the key, keep every stream's counter (root-parallel offsets)."""
        if tree is None:
            tree = self.tree
        self.seed = int(seed)
        self.tree = int(tree)
        self._k0 = self.seed & MASK32
        self._k1 = self.tree & MASK32
        self._c3 = (self.seed >> 32) & MASK32
        self._blk = {}

    def u32(self, stream: int) -> int:
        j = self.ctr.get(stream, 0)
        self.ctr[stream] = j + 1
        b = j >> 2
        cached = self._blk.get(stream)
        if cached is None or cached[0] != b:
            words = philox4x32(b & MASK32, (b >> 32) & MASK32, stream, self._c3,
                                  self._k0, self._k1)
            cached = (b, words)
            self._blk[stream] = cached
        return cached[1][j & 3]

    def align_sim(self):
        """Start of a simulation: the step streams' counters to the next
        multiple of 4 (``SIM_STREAMS``)."""
        for s in SIM_STREAMS:
            j = self.ctr.get(s, 0)
            if j & 3:
                self.ctr[s] = (j + 3) & ~3

    def randint(self, stream: int, n: int) -> int:
        """Uniform int in [0, n) (no rejection)."""
        return (self.u32(stream) * n) >> 32

    def random(self, stream: int) -> float:
        return self.u32(stream) * (1.0 / 4294967296.0)

    def counters(self):
        return dict(self.ctr)


class StreamRandom:
    """`random.Random`-shaped view of one stream (for injection into the reference)."""

    def __init__(self, streams: Streams, stream: int):
        self._s = streams
        self._id = stream

    def random(self):
        return self._s.random(self._id)

    def choice(self, seq):
        if len(seq) == 0:
            raise IndexError("Cannot choose from an empty sequence")
        return seq[self._s.randint(self._id, len(seq))]

    def choices(self, population, weights=None, *, cum_weights=None, k=1):
        """Same arithmetic as CPython's ``random.choices`` with our ``random()``."""
        n = len(population)
        if cum_weights is None:
            if weights is None:
                return [population[self._s.randint(self._id, n)] for _ in range(k)]
            cum_weights = []
            acc = 0.0
            first = True
            for w in weights:
                acc = w if first else acc + w
                first = False
                cum_weights.append(acc)
        total = cum_weights[-1] + 0.0
        hi = n - 1
        out = []
        for _ in range(k):
            x = self.random() * total
            # bisect_right(cum_weights, x, 0, hi)
            lo, h = 0, hi
            while lo < h:
                mid = (lo + h) // 2
                if x < cum_weights[mid]:
                    h = mid
                else:
                    lo = mid + 1
            out.append(population[lo])
        return out

    def shuffle(self, x):
        for i in reversed(range(1, len(x))):
            j = self._s.randint(self._id, i + 1)
            x[i], x[j] = x[j], x[i]
