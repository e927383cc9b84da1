"""Python handle on one ``pomcp_ctx`` (a batch of independent search trees on
one GPU).  Builds the C config from a model + ``MCTSConfig``, sizes the
per-tree HBM arenas, and exposes update / search / statistics as numpy.
"""
import ctypes as C
import math
import os
from dataclasses import dataclass

import numpy as np

from posggym_baselines_amd import _native as N

INT32_MAX = 2**31 - 1


@dataclass
class Capacities:
    max_blocks: int           # expanded obs nodes (each A x 128 B action nodes)
    max_particles: int        # particle log records (16 B)
    max_belief: int           # root belief region (16 B records): the root belief and the
                              # next one, one from each end (pomcp_device.h bel_at)
    overflow_slots: int       # obs children beyond 6 per action node (32 B)
    log_table_size: int
    discount_pow_size: int

    def bytes_per_tree(self, num_actions: int, type_based: bool = False,
                       reroot: bool = False) -> int:
        """HBM of one tree (pomcp_create): (A + 1 [+ 1]) x 128 B per block, 32 B
        overflow entries, 12 [16] B particle records, the 16 B root belief region;
        with ``reroot`` also the re-root's scratch (allocated on the first update
        that re-roots: the block map / parents, the overflow rebuild, the scan's
        per-tree record, its share of the look-back records -- 528 B per 16,384
        log records of its search wave, an upper bound -- and of its wave's
        packed block map, 24,840 B)."""
        tm = 1 if type_based else 0
        b = (self.max_blocks * (num_actions + 1 + tm) * 128 + self.overflow_slots * 32
             + self.max_particles * (12 + 4 * tm) + self.max_belief * 16)
        if reroot:
            b += (8 * self.max_blocks + 36 * self.overflow_slots + 16
                  + -(-64 * self.max_particles // 16384) * 528 // 64 + 528 + 389)
        return b


def _next_pow2(n: int) -> int:
    return 1 << max(4, (int(n) - 1).bit_length())


ID_LIMIT = (1 << 26) - 1   # obs node ids share a log word with the lane (pomcp_device.h)
# ids per block and action: 6 inline child slots + 1 deferred-record id (pomcp_device.h)
IDS_PER_ACTION = 7


def plan_capacities(config, step_limit: int, num_sims: int, searches: int = 1,
                    reroot: bool = True, max_blocks: int = None, overflow_slots: int = None,
                    num_actions: int = 5):
    """Worst-case arena sizes for ``searches`` searches of ``num_sims`` each.

    Every simulation expands at most one leaf (mcts.py:318-328) and appends one
    particle per tree level stepped (mcts.py:371), at most
    min(depth_limit, step_limit) + 1 levels.  Pass smaller ``max_blocks`` /
    ``overflow_slots`` to trade worst-case guarantees for memory: overflow is
    detected and reported (POMCP_E_ARENA), never silent.
    """
    levels = min(config.depth_limit, step_limit) + 1
    n_target = config.num_particles + config.extra_particles
    total = num_sims * searches
    ovf = _next_pow2(max(64, total // 8)) if overflow_slots is None else overflow_slots
    ovf = min(ovf, 1 << 24)
    if max_blocks is None:
        # one expansion per simulation at most, within the obs node id space
        nb = min(total + 2 * searches + 16, (ID_LIMIT - 1 - ovf) // (num_actions * IDS_PER_ACTION))
    else:
        nb = max_blocks
    np_ = total * min(levels, 64) + searches * 2 * n_target + 64
    # the root belief region holds the root belief and the next (a re-root's
    # extraction + reinvigoration), each at most a log's worth of particles
    nr = 2 * (np_ + 2 * n_target + 64) if reroot else 2 * (4 * n_target + 64)
    return Capacities(
        max_blocks=nb, max_particles=np_, max_belief=nr, overflow_slots=ovf,
        log_table_size=total + 2, discount_pow_size=min(levels, 4096) + 2)


# Wall-clock mode (num_sims=None, the reference's default, mcts.py:285) sizes
# the arenas from the time limit: an upper bound on one tree's simulation rate
# (a lone tree on the wave-per-tree kernel: 130-330 k simulations/s on MI355X
# depending on how deep its simulations go; ~3x margin) times
# search_time_limit per search, within the 2^26 obs-node id space (about 1.1 M
# simulations per search for A = 5: a longer budget ends its search there,
# step_statistics "arena_full").  The arena holds one
# search plus the subtree kept by the re-root (subtree compaction at update,
# pomcp_kernels.hip k_compact), and get_action stops launching chunks before
# a chunk could overflow it (POMCP.get_action), so a time-limited episode never
# fails with POMCP_E_ARENA.  HBM budget for all trees of one engine:
# Algorithmic HBM bytes of a search (DESIGN.md §4 "Algorithmic
# bytes"), from the kernel's own per-tree counters: per simulation its root
# particle (16); per tree level stepped the node (8) + A action statistics
# (12 each) + child lookup (16) + child visit / absorbing flag (8 + 4) +
# particle record (16) + backup of {visits, value, total} (40); per leaf
# expansion 20 A + 4; per obs node created 28.  Charged only for what the
# kernel does: no lookup at a deferred level (no probe), no child write at a
# cut-off level (mcts.py:315).  Type-based searches add the node's
# action_probs (16 A per level, 8 A per expansion).  bench.py's roofline
# numerator and step_statistics["hbm_bytes"] both come from here.
B_SIM, B_NEW_NODE, B_LOOKUP, B_CHILD_WRITE = 16, 28, 16, 12


def b_level(A: int) -> int:
    return 8 + 12 * A + 84


def b_expand(A: int) -> int:
    return 20 * A + 4


def search_bytes(stats, A: int, type_based: bool = False) -> int:
    """Algorithmic bytes of the last search of the trees in `stats`
    (pomcp_root_stats records)."""
    tot = 0
    for s in stats:
        tot += (B_SIM * s.num_sims + b_level(A) * s.n_levels - B_LOOKUP * s.n_deferred
                - B_CHILD_WRITE * s.n_cutoff + b_expand(A) * s.n_expansions
                + B_NEW_NODE * s.n_new_nodes)
        if type_based:
            tot += 16 * A * s.n_levels + 8 * A * s.n_expansions
    return int(tot)


WALL_CLOCK_SIMS_PER_S = 1_000_000
WALL_CLOCK_HBM_BUDGET = 64 << 30


def plan_wallclock_capacities(config, step_limit: int, num_trees: int = 1, num_actions: int = 5):
    """Capacities of a wall-clock (num_sims=None) engine; returns (capacities,
    per-search simulation bound)."""
    levels = min(config.depth_limit, step_limit) + 1
    # block + particle records, worst case; batches of up to 256 trees run on the
    # wave-per-tree kernel, whose per-tree scratch log holds one more 12 B record
    # per level (k_search_lds, allocated on its first search)
    per_sim = num_actions * 128 + 16 * min(levels, 64)
    if num_trees <= 256:
        per_sim += 12 * min(levels, 64)
    sims = math.ceil(config.search_time_limit * WALL_CLOCK_SIMS_PER_S)
    sims = min(sims, WALL_CLOCK_HBM_BUDGET // (2 * per_sim * max(1, num_trees)))
    ovf = 1 << 16
    nb_id = (ID_LIMIT - 1 - ovf) // (num_actions * IDS_PER_ACTION)
    sims = max(256, min(sims, nb_id // 2 - 64))
    caps = plan_capacities(config, step_limit, sims, 2, num_actions=num_actions,
                           overflow_slots=ovf)
    # log(N) of a node's visit count: a node at depth d of a search was visited
    # by at most one search's simulations in each of the d searches before it
    # became the root (depth <= min(depth_limit, step_limit) + 1)
    caps.log_table_size = (min(levels, 64) + 1) * sims + 2
    return caps, sims


_LOG_TABLE = np.zeros(1, dtype=np.float64)


def log_table(n: int) -> np.ndarray:
    """[0.0, log(1), .., log(n-1)] with the host's math.log (the reference's
    UCB term, mcts.py:534), bit for bit; one cached table per process, grown on
    demand (wall-clock arenas ask for tens of millions of entries).  Computed
    by pomcp_host_log_table: the C library's log, which math.log calls for a
    float (tests/test_host_exp.py pins the two equal)."""
    global _LOG_TABLE
    if len(_LOG_TABLE) < n:
        m = len(_LOG_TABLE)
        ext = np.empty(n - m, dtype=np.float64)
        rc = N.load().pomcp_host_log_table(m, n - m, ext.ctypes.data_as(C.POINTER(C.c_double)))
        if rc != N.POMCP_OK:
            raise N.PomcpError(rc, "pomcp_host_log_table failed")
        _LOG_TABLE = np.concatenate([_LOG_TABLE, ext])
    return _LOG_TABLE[:n]


class PomcpEngine:
    SELECTION = {"pucb": N.SEL_PUCB, "ucb": N.SEL_UCB, "uniform": N.SEL_UNIFORM}

    def __init__(self, model, agent_id, config, num_trees=1, capacities=None, num_sims=None,
                 searches=None, device=None, stream=None, tree_key_base=0, seed=None,
                 wall_clock=False, type_policies=None):
        lib = N.load()
        from posggym_baselines_amd.envs import engine_model
        model = engine_model(model)   # posggym-style models by spec.id + kwargs
        if config.truncated and not config.use_rollout_if_no_value:
            raise NotImplementedError("truncated search needs a value function (none on GPU)")
        self.model = model
        self.config = config
        self.num_trees = int(num_trees)
        self.ego = model.possible_agents.index(agent_id)
        self.A = model.action_spaces[agent_id].n
        if config.step_limit is not None:
            step_limit = int(config.step_limit)
        elif getattr(model, "spec", None) is not None and model.spec.max_episode_steps:
            step_limit = int(model.spec.max_episode_steps)
        else:
            step_limit = INT32_MAX
        self.step_limit = step_limit
        self.wall_clock_sims = None
        if capacities is None and wall_clock:
            capacities, self.wall_clock_sims = plan_wallclock_capacities(
                config, step_limit, self.num_trees, model.action_spaces[agent_id].n)
        if capacities is None:
            sims = num_sims if num_sims is not None else (config.num_sims or 4096)
            budget = searches if searches is not None else (
                (step_limit if step_limit < INT32_MAX else 100) + 1)
            capacities = plan_capacities(config, step_limit, sims, budget,
                                         num_actions=self.A)
        self.capacities = capacities
        c = N.PomcpConfig()
        c.abi_version = N.POMCP_ABI_VERSION
        c.num_agents = len(model.possible_agents)
        c.ego_agent = self.ego
        c.num_actions = self.A
        c.action_selection = self.SELECTION[config.action_selection]
        c.depth_limit = min(config.depth_limit, INT32_MAX)
        c.step_limit = step_limit
        c.num_particles = config.num_particles
        c.extra_particles = config.extra_particles
        kb = config.known_bounds
        c.has_known_bounds = 1 if kb else 0
        if kb:
            c.known_min, c.known_max = float(kb[0]), float(kb[1])
        c.num_trees = self.num_trees
        c.discount = config.discount
        c.c = config.c
        c.pucb_exploration_fraction = config.pucb_exploration_fraction
        c.reinvigoration_sample_limit_factor = config.reinvigoration_sample_limit_factor
        s = config.seed if seed is None else seed
        if s is None:
            s = int(np.random.SeedSequence().entropy) & (2**63 - 1)
        c.seed = int(s) & (2**64 - 1)
        c.tree_key_base = int(tree_key_base)
        c.max_blocks = capacities.max_blocks
        c.max_particles = capacities.max_particles
        c.max_belief = capacities.max_belief
        c.overflow_slots = capacities.overflow_slots
        # FP64 tables from Python's own math.log and float ** int (bit-exact with
        # mcts.py:534 and mcts.py:421)
        self._logtab = log_table(capacities.log_table_size)
        self._dpow = np.array([config.discount ** k for k in range(capacities.discount_pow_size)],
                              dtype=np.float64)
        c.log_table = self._logtab.ctypes.data_as(C.POINTER(C.c_double))
        c.log_table_size = len(self._logtab)
        c.discount_pow = self._dpow.ctypes.data_as(C.POINTER(C.c_double))
        c.discount_pow_size = len(self._dpow)
        model.configure_engine(c)
        c.type_based = 1 if type_policies is not None else 0
        self.type_based = type_policies is not None
        self._cfg = c
        dev = config.device if device is None else device
        ctx = C.c_void_p()
        rc = lib.pomcp_create(C.byref(c), int(dev), stream, C.byref(ctx))
        if rc != N.POMCP_OK:
            raise N.PomcpError(rc, "pomcp_create failed (no GPU, bad config or out of memory)")
        self._ctx = ctx
        self._lib = lib
        self._stats = (N.PomcpRootStats * self.num_trees)()
        if type_policies is not None:
            self._check(lib.pomcp_set_type_policies(ctx, C.byref(type_policies)),
                        "set_type_policies")
        # search kernel override (tests / benchmarks): POMCP_SEARCH_KERNEL=lane|wave.
        # A type-based (POTMMCP) context has only the lane kernel: the process-wide
        # override does not apply to it (an explicit set_search_kernel still raises)
        kind = os.environ.get("POMCP_SEARCH_KERNEL", "auto")
        if kind != "auto" and not (self.type_based and kind == "wave"):
            self.set_search_kernel(kind)
        # deferral override (tests): POMCP_DEFER_CUTOFF=0|1
        if os.environ.get("POMCP_DEFER_CUTOFF") in ("0", "1"):
            self.set_defer_cutoff(os.environ["POMCP_DEFER_CUTOFF"] == "1")
            self._defer_forced = True

    # ------------------------------------------------------------------
    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.pomcp_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        N.check(rc, self._ctx, what)

    def reset(self):
        self._check(self._lib.pomcp_reset(self._ctx), "reset")

    def root_prior(self, tree=0):
        """Type-based: the root's ObsNode.action_probs (num_actions doubles)."""
        out = (C.c_double * self.A)()
        self._check(self._lib.pomcp_get_root_prior(self._ctx, int(tree), out), "get_root_prior")
        return list(out)

    def root_policies(self, tree=0):
        """Type-based: the other-agent policy index of every root particle."""
        n = C.c_int32()
        self._check(self._lib.pomcp_get_root_policies(self._ctx, int(tree), None, 0, C.byref(n)),
                    "get_root_policies")
        out = np.zeros(max(n.value, 1), dtype=np.int32)
        self._check(self._lib.pomcp_get_root_policies(
            self._ctx, int(tree), out.ctypes.data_as(C.POINTER(C.c_int32)), n.value, C.byref(n)),
            "get_root_policies")
        return out[:n.value]

    def update(self, actions, obs_keys):
        B = self.num_trees
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(actions, dtype=np.int32), (B,)))
        o = np.ascontiguousarray(np.broadcast_to(np.asarray(obs_keys, dtype=np.uint64), (B,)))
        absorbing = np.zeros(B, dtype=np.int32)
        self._check(self._lib.pomcp_update(
            self._ctx, a.ctypes.data_as(C.POINTER(C.c_int32)),
            o.ctypes.data_as(C.POINTER(C.c_uint64)),
            absorbing.ctypes.data_as(C.POINTER(C.c_int32))), "update")
        return absorbing.astype(bool)

    def search(self, num_sims, fetch=True, final=True):
        """``num_sims`` simulations per tree; ``final=False`` leaves out the final
        action choice (more launches of the same get_action follow)."""
        if not final:
            self._check(self._lib.pomcp_search_continue(self._ctx, int(num_sims)), "search")
            return None
        if not fetch:
            self._check(self._lib.pomcp_search(self._ctx, int(num_sims), None), "search")
            return None
        out = np.zeros(self.num_trees, dtype=np.int32)
        self._check(self._lib.pomcp_search(self._ctx, int(num_sims),
                                           out.ctypes.data_as(C.POINTER(C.c_int32))), "search")
        return out

    def set_search_kernel(self, kind):
        """"auto" | "lane" (k_search: a tree per lane, HBM) | "wave" (k_search_lds:
        a wave per tree, tree in LDS); same results, different speed."""
        k = {"auto": N.SEARCH_AUTO, "lane": N.SEARCH_LANE, "wave": N.SEARCH_WAVE}[kind]
        self._check(self._lib.pomcp_set_search_kernel(self._ctx, k), "set_search_kernel")

    def set_defer_cutoff(self, on):
        """Defer cut-off children to the re-root (True, the default: the search
        skips their slot lines and the re-root materialises the survivors in
        bulk) or look them up during the search (False); same results
        (``pomcp_set_defer_cutoff``).
        A process-wide POMCP_DEFER_CUTOFF override (tests) wins."""
        if getattr(self, "_defer_forced", False):
            return
        if not hasattr(self._lib, "pomcp_set_defer_cutoff"):
            return   # an explicitly chosen measurement library from older sources (always defers)
        self._check(self._lib.pomcp_set_defer_cutoff(self._ctx, 1 if on else 0), "set_defer_cutoff")

    def search_kernel(self):
        """The kernel the next search uses: "lane" or "wave"."""
        return "wave" if self._lib.pomcp_search_kernel_used(self._ctx) == N.SEARCH_WAVE else "lane"

    def root_stats(self):
        self._check(self._lib.pomcp_get_root_stats(self._ctx, self._stats), "get_root_stats")
        return self._stats

    def root_belief(self, tree=0):
        n = C.c_int32()
        self._check(self._lib.pomcp_get_root_belief(self._ctx, tree, None, 0, C.byref(n)),
                    "get_root_belief")
        buf = np.zeros(3 * max(n.value, 1), dtype=np.uint32)
        self._check(self._lib.pomcp_get_root_belief(
            self._ctx, tree, buf.ctypes.data_as(C.POINTER(C.c_uint32)), n.value, C.byref(n)),
            "get_root_belief")
        return buf[:3 * n.value].reshape(-1, 3)

    def set_root_belief(self, tree, rows):
        """Root belief of a fresh tree from host particles ((t, v0, v1) rows)."""
        a = np.ascontiguousarray(np.asarray(rows, dtype=np.uint32).reshape(-1, 3))
        self._check(self._lib.pomcp_set_root_belief(
            self._ctx, int(tree), a.ctypes.data_as(C.POINTER(C.c_uint32)), len(a)),
            "set_root_belief")

    def rekey(self, seed):
        self._check(self._lib.pomcp_rekey(self._ctx, int(seed) & (2**64 - 1)), "rekey")

    def merge_buffer_ptr(self) -> int:
        p = C.c_void_p()
        self._check(self._lib.pomcp_root_merge_buffer(self._ctx, C.byref(p)), "merge_buffer")
        return p.value

    def headroom(self):
        """Simulations every tree can still run before its block arena or particle
        log could overflow (worst case: one expansion and min(depth, step) + 1
        particle records per simulation)."""
        nb, nl = C.c_int32(), C.c_int32()
        self._check(self._lib.pomcp_arena_usage(self._ctx, C.byref(nb), C.byref(nl)), "arena_usage")
        nb, nl = nb.value, nl.value
        cap = self.capacities
        levels = min(self.config.depth_limit, self.step_limit) + 1
        return max(0, min(cap.max_blocks - nb - 1, (cap.max_particles - nl - 1) // min(levels, 64)))

    def gather_buffer_ptr(self, world: int) -> int:
        """Device pointer of the [world][trees][xrec(A)] gather buffer."""
        p = C.c_void_p()
        self._check(self._lib.pomcp_root_gather_buffer(self._ctx, int(world), C.byref(p)),
                    "gather_buffer")
        return p.value

    def merge_roots(self, group, fetch=True, world=0):
        """Device merge of root-parallel replicas (``pomcp_merge_roots``): trees
        [g * group, (g + 1) * group) are planner g; ``world`` = 0 merges this
        GPU's records, ``world`` >= 1 the gather buffer of that many ranks.
        Returns the ``PomcpMergedRoot`` array (or None with ``fetch=False``);
        raises if any merged replica reported an error."""
        G = self.num_trees // group
        if not fetch:
            self._check(self._lib.pomcp_merge_roots(self._ctx, int(group), int(world), None),
                        "merge_roots")
            return None
        out = (N.PomcpMergedRoot * G)()
        self._check(self._lib.pomcp_merge_roots(self._ctx, int(group), int(world), out),
                    "merge_roots")
        return out

    def synthetic_obs(self, env_seed_base):
        out = np.zeros(self.num_trees, dtype=np.uint64)
        self._check(self._lib.pomcp_synthetic_obs(
            self._ctx, int(env_seed_base), out.ctypes.data_as(C.POINTER(C.c_uint64))),
            "synthetic_obs")
        return out

    def synthetic_step(self, env_seed_base, actions):
        """The synthetic roots' environment answer to ``actions`` (bench): the
        ego's next observation key per tree (``pomcp_synthetic_step``)."""
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(actions, dtype=np.int32),
                                                 (self.num_trees,)))
        out = np.zeros(self.num_trees, dtype=np.uint64)
        self._check(self._lib.pomcp_synthetic_step(
            self._ctx, int(env_seed_base), a.ctypes.data_as(C.POINTER(C.c_int32)),
            out.ctypes.data_as(C.POINTER(C.c_uint64))), "synthetic_step")
        return out

    def snapshot(self):
        self._check(self._lib.pomcp_snapshot(self._ctx), "snapshot")

    def restore(self):
        self._check(self._lib.pomcp_restore(self._ctx), "restore")

    def set_stream(self, stream):
        self._check(self._lib.pomcp_set_stream(self._ctx, stream), "set_stream")
