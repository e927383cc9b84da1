"""I-NTMCP drop-in: the reference's ``INTMCP`` API (``intmcp.py:22-994``) at
nesting levels 0 to 5 with two agents, the planners' trees, beliefs and
generative model on the GPU (``include/intmcp.h``, ``csrc/intmcp.hip``).

Public surface kept from the reference: ``INTMCP.initialize(model,
ego_agent_id, config, nesting_level, search_policies)``, ``step(obs)``,
``reset()``, ``update(action, obs)``, ``get_action()``, ``close()``, and the
attributes ``model``, ``agent_id``, ``config``, ``nesting_level``,
``num_agents``, ``other_agent_policies`` (the level-0 planner, a view of the
same device state), ``search_policies``, ``action_spaces``, ``step_limit``,
``step_statistics``, ``stat_tracker``, ``root``.

``BatchedINTMCP`` runs many independent planner pairs in one launch (BASELINE
config 5: nested trees as a batched launch).

Scope (DESIGN.md "I-NTMCP"): nesting levels 0 to 5, random or
fixed-distribution search policies (``RandomSearchPolicy`` /
``SearchPolicyWrapper(FixedDistributionPolicy)`` per level and agent: they draw
the rollouts and the other agent's action at an unvisited history; the node
priors they give only matter to PUCB), ``ucb`` / ``uniform`` selection (the reference's
``pucb_action_selection`` reads ``self.action_space``, which INTMCP does not
define, ``intmcp.py:645``).  The reinvigoration of a depleted root during the
search (``intmcp.py:426-431``) cannot run under a valid configuration (the
reference asserts ``reinvigoration_sample_limit_factor >= 1``, ``belief.py:85``;
DESIGN.md §10); the kernel reports POMCP_E_UNSUPPORTED should it ever be reached.

Wall-clock mode (``num_sims=None``, the reference's default): the arenas are
sized from ``search_time_limit`` and an HBM budget
(:func:`plan_intmcp_wallclock_capacities`), and ``get_action`` stops launching
chunks before one could overflow them, so a time-limited episode never fails
with POMCP_E_ARENA (``step_statistics["arena_full"]`` records an early stop).
"""
import ctypes as C
import dataclasses
import logging
import math
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np
import psutil

from posggym_baselines_amd.envs import engine_model

from posggym_baselines_amd import _native as N
from posggym_baselines_amd.planning.config import MCTSConfig
from posggym_baselines_amd.planning.engine import log_table
from posggym_baselines_amd.planning.search_policy import RandomSearchPolicy
from posggym_baselines_amd.planning.utils import PlanningStatTracker

INT32_MAX = 2**31 - 1
# a node's device bytes: its 128 B line + six 32 B action records (csrc/intmcp.hip kImBlock)
INTMCP_NODE_BYTES = 320
MAX_TREES = 6                  # include/intmcp.h INTMCP_MAX_TREES: a tree per nesting level
MAX_NESTING = MAX_TREES - 1


@dataclass
class IntmcpCapacities:
    max_nodes: int              # obs nodes per tree (320 B each: node line + action records)
    max_stats: int              # action statistics per tree (allocation counter limit)
    max_log: int                # particle log records per tree (16 B)
    hash_slots: int             # obs-child map slots per tree (16 B)
    max_root_belief: int        # level-1 root particles (16 B, x2) and support entries (16 B, x2)
    max_support_particles: int  # materialised level-0 particles (8 B, x2)
    log_table_size: int
    discount_pow_size: int
    trees: int = 2              # trees per pair: nesting level + 1 from level 2

    def bytes_per_pair(self, num_actions: int = 5) -> int:
        b = (self.trees * (self.max_nodes * INTMCP_NODE_BYTES + self.max_log * 16
                           + self.hash_slots * 16) + 4 * self.max_root_belief * 16
             + 2 * self.max_support_particles * 8 + self.max_root_belief * 8)
        # each middle planner's beliefs (entries, 16 B particles, distribution)
        b += max(0, self.trees - 2) * (2 * self.max_root_belief * 16
                                       + 2 * self.max_support_particles * 16
                                       + self.max_root_belief * 8)
        return b


def _next_pow2(n: int) -> int:
    return 1 << max(4, (int(n) - 1).bit_length())


def plan_intmcp_capacities(config, step_limit: int, num_sims: int, searches: int,
                           num_actions: int, nesting_level: int = 1) -> IntmcpCapacities:
    """Worst-case sizes for ``searches`` steps of ``num_sims`` simulations per level.

    Per step and tree: every simulation steps at most ``L = min(depth_limit,
    step_limit) + 1`` levels (one node + one log record each); a level-1
    simulation also extends the other agent's history in the level-0 tree;
    each reinvigoration attempt (at most ``limit_factor x target`` per belief)
    creates a level-0 node.  A root / level-0 belief gathers records of the
    last ``L`` searches plus its reinvigoration (accepted and rejected).
    """
    L = min(config.depth_limit, step_limit) + 1
    S = num_sims
    target = config.num_particles + config.extra_particles
    lf = config.reinvigoration_sample_limit_factor
    reinv = int(math.ceil(lf * target)) + target
    levels = nesting_level + 1 if nesting_level >= 2 else 2   # (nesting 0 keeps the level-1 sizing)
    mid = levels - 2                                             # middle planners
    per_step = levels * S * L + 2 * reinv + 2 * target + 8
    # each middle planner's reinvigorations extend the histories of the tree below
    per_step += mid * 2 * reinv * 8
    nodes = searches * per_step + 16
    nr = S * L + 4 * target + 64
    nsp = S * L + 2 * nr + 4 * target + 64
    if mid:   # every history's middle belief, and the histories below it
        nr += 8 * target * mid
        nsp = levels * S * L + 8 * nr + 8 * target + 64
    total_sims = levels * S * searches
    return IntmcpCapacities(
        max_nodes=nodes, max_stats=num_actions * nodes, max_log=nodes,
        hash_slots=_next_pow2(2 * nodes), max_root_belief=nr, max_support_particles=nsp,
        log_table_size=total_sims + 2, discount_pow_size=min(L, 4096) + 2,
        trees=levels)


# Wall-clock sizing.  One pair's simulation rate alone on the GPU (one lane,
# chunked launches) is bounded by INTMCP_WALL_CLOCK_SIMS_PER_S per level
# (measured 80-130 k/s per level on MI355X, tests/test_gpu_intmcp.py
# test_wall_clock_episode_half_second; ~2x margin): a search runs at
# most that many simulations per level per second of its share of
# search_time_limit.  The node arena is the smaller of the worst case for that
# rate and the HBM budget; get_action's headroom check keeps a chunk inside it.
INTMCP_WALL_CLOCK_SIMS_PER_S = 250_000
INTMCP_WALL_CLOCK_HBM_BUDGET = 16 << 30
_INTMCP_ID_LIMIT = (1 << 28) - 1


def plan_intmcp_wallclock_capacities(config, step_limit: int, num_actions: int,
                                     nesting_level: int = 1):
    """Capacities of a wall-clock (``num_sims=None``) I-NTMCP engine; returns
    (capacities, per-level simulation ceiling of one search)."""
    per_level = config.search_time_limit / (nesting_level + 1)
    sims = max(64, math.ceil(per_level * INTMCP_WALL_CLOCK_SIMS_PER_S))
    searches = (step_limit if step_limit < INT32_MAX else 100) + 1
    caps = plan_intmcp_capacities(config, step_limit, sims, searches, num_actions, nesting_level)
    # per node and pair: the trees x (320 B node + 16 B log record + <=64 B of
    # hash slots); per-search arrays (root belief, support) keep their worst case
    nt = caps.trees
    per_node = nt * (INTMCP_NODE_BYTES + 16 + 64)
    fixed = caps.bytes_per_pair(num_actions) - caps.max_nodes * nt * INTMCP_NODE_BYTES \
        - caps.max_log * nt * 16 - caps.hash_slots * nt * 16
    nodes = (INTMCP_WALL_CLOCK_HBM_BUDGET - fixed) // per_node
    nodes = max(1 << 16, min(caps.max_nodes, nodes, _INTMCP_ID_LIMIT))
    caps.max_nodes = caps.max_log = nodes
    caps.max_stats = num_actions * nodes
    caps.hash_slots = _next_pow2(2 * nodes)
    return caps, sims


class IntmcpEngine:
    """Python handle on one ``intmcp_ctx`` (``num_pairs`` planner pairs)."""

    SELECTION = {"ucb": N.SEL_UCB, "uniform": N.SEL_UNIFORM}

    def __init__(self, model, agent_id, config, num_pairs=1, capacities=None, num_sims=None,
                 searches=None, device=None, stream=None, tree_key_base=0, seed=None,
                 wall_clock=False, nesting_level=1):
        lib = N.load()
        model = engine_model(model)   # posggym-style models by spec.id + kwargs
        if len(model.possible_agents) != 2:
            raise NotImplementedError("the I-NTMCP engine plans for two agents")
        if config.action_selection not in self.SELECTION:
            raise NotImplementedError(
                "INTMCP pucb_action_selection reads self.action_space, which INTMCP does not "
                "define (intmcp.py:645); use 'ucb' or 'uniform'")
        self.model = model
        self._emodel = engine_model(model)
        self.config = config
        self.num_pairs = int(num_pairs)
        if not 0 <= int(nesting_level) <= MAX_NESTING:
            raise NotImplementedError(f"the GPU I-NTMCP engine runs nesting levels 0 to {MAX_NESTING}")
        self.nesting_level = int(nesting_level)
        self.ego = model.possible_agents.index(agent_id)
        self.A = model.action_spaces[agent_id].n
        other = model.possible_agents[1 - self.ego]
        if model.action_spaces[other].n != self.A:
            raise NotImplementedError("both agents need the same action count")
        if config.step_limit is not None:
            step_limit = int(config.step_limit)
        elif getattr(model, "spec", None) is not None and model.spec.max_episode_steps:
            step_limit = int(model.spec.max_episode_steps)
        else:
            step_limit = INT32_MAX
        self.step_limit = step_limit
        self.wall_clock_sims = None
        if capacities is None and wall_clock:
            capacities, self.wall_clock_sims = plan_intmcp_wallclock_capacities(
                config, step_limit, self.A, self.nesting_level)
        if capacities is None:
            sims = num_sims if num_sims is not None else (config.num_sims or 1024)
            budget = searches if searches is not None else (
                (step_limit if step_limit < INT32_MAX else 100) + 1)
            capacities = plan_intmcp_capacities(config, step_limit, sims, budget, self.A,
                                                self.nesting_level)
        self.capacities = capacities
        ic = N.IntmcpConfig()
        c = ic.base
        c.abi_version = N.POMCP_ABI_VERSION
        c.num_agents = 2
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
        c.num_trees = self.num_pairs
        c.discount = config.discount
        c.c = config.c
        c.pucb_exploration_fraction = config.pucb_exploration_fraction
        c.reinvigoration_sample_limit_factor = config.reinvigoration_sample_limit_factor
        s = config.seed if seed is None else seed
        if s is None:
            s = int(np.random.SeedSequence().entropy) & (2**63 - 1)
        c.seed = int(s) & (2**64 - 1)
        c.tree_key_base = int(tree_key_base)
        self._logtab = log_table(capacities.log_table_size)
        self._dpow = np.array([config.discount ** k for k in range(capacities.discount_pow_size)],
                              dtype=np.float64)
        c.log_table = self._logtab.ctypes.data_as(C.POINTER(C.c_double))
        c.log_table_size = len(self._logtab)
        c.discount_pow = self._dpow.ctypes.data_as(C.POINTER(C.c_double))
        c.discount_pow_size = len(self._dpow)
        model.configure_engine(c)
        ic.state_belief_only = 1 if config.state_belief_only else 0
        ic.nesting_level = self.nesting_level
        ic.max_nodes = capacities.max_nodes
        ic.max_stats = capacities.max_stats
        ic.max_log = capacities.max_log
        ic.hash_slots = capacities.hash_slots
        ic.max_root_belief = capacities.max_root_belief
        ic.max_support_particles = capacities.max_support_particles
        self._cfg = ic
        dev = config.device if device is None else device
        ctx = C.c_void_p()
        rc = lib.intmcp_create(C.byref(ic), int(dev), stream, C.byref(ctx))
        if rc != N.POMCP_OK:
            why = (lib.intmcp_last_error(None) or b"").decode(errors="replace")
            raise N.PomcpError(rc, "intmcp_create failed: "
                               + (why or "no GPU, bad config or out of memory"))
        self._ctx = ctx
        self._lib = lib
        self._stats = (N.IntmcpRootStats * self.num_pairs)()

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.intmcp_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        N.check(rc, self._ctx, what, last_error="intmcp_last_error")

    def reset(self):
        self._check(self._lib.intmcp_reset(self._ctx), "reset")

    def update(self, actions, obs_keys):
        B = self.num_pairs
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(actions, dtype=np.int32), (B,)))
        o = np.ascontiguousarray(np.broadcast_to(np.asarray(obs_keys, dtype=np.uint64), (B,)))
        absorbing = np.zeros(B, dtype=np.int32)
        self._check(self._lib.intmcp_update(
            self._ctx, a.ctypes.data_as(C.POINTER(C.c_int32)),
            o.ctypes.data_as(C.POINTER(C.c_uint64)),
            absorbing.ctypes.data_as(C.POINTER(C.c_int32))), "update")
        return absorbing.astype(bool)

    def search(self, num_sims, fetch=True):
        if not fetch:
            self._check(self._lib.intmcp_search(self._ctx, int(num_sims), None), "search")
            return None
        out = np.zeros(self.num_pairs, dtype=np.int32)
        self._check(self._lib.intmcp_search(self._ctx, int(num_sims),
                                            out.ctypes.data_as(C.POINTER(C.c_int32))), "search")
        return out

    def set_search_policy(self, level, agent_index, probs=None):
        """``search_policies[level][agent]``: None (random) or a fixed action
        distribution (``intmcp_set_search_policy``)."""
        ptr = None
        if probs is not None:
            self._sp_keep = getattr(self, "_sp_keep", [])
            arr = np.ascontiguousarray(np.asarray(probs, dtype=np.float64))
            if arr.shape != (self.A,):
                raise ValueError(f"search policy: {self.A} action probabilities expected")
            self._sp_keep.append(arr)
            ptr = arr.ctypes.data_as(C.POINTER(C.c_double))
        self._check(self._lib.intmcp_set_search_policy(self._ctx, int(level), int(agent_index), ptr),
                    "set_search_policy")

    def search_level(self, level, sims, flags, fetch=False):
        """One chunk of ``sims`` simulations at nesting ``level`` (``intmcp_search_level``)."""
        out = np.zeros(self.num_pairs, dtype=np.int32) if fetch else None
        ptr = out.ctypes.data_as(C.POINTER(C.c_int32)) if fetch else None
        self._check(self._lib.intmcp_search_level(self._ctx, int(level), int(sims), int(flags), ptr),
                    "search_level")
        return out

    def tree_counts(self):
        """[pairs][MAX_TREES][nodes, log records, stats] (``intmcp_get_tree_counts``)."""
        out = np.zeros((self.num_pairs, MAX_TREES, 3), dtype=np.int32)
        self._check(self._lib.intmcp_get_tree_counts(self._ctx, out.ctypes.data_as(C.POINTER(C.c_int32))),
                    "get_tree_counts")
        return out

    def search_levels(self, level0_sims, level1_sims, flags, fetch=False):
        out = np.zeros(self.num_pairs, dtype=np.int32) if fetch else None
        ptr = out.ctypes.data_as(C.POINTER(C.c_int32)) if fetch else None
        self._check(self._lib.intmcp_search_levels(self._ctx, int(level0_sims), int(level1_sims),
                                                   int(flags), ptr), "search_levels")
        return out

    def root_stats(self):
        self._check(self._lib.intmcp_get_root_stats(self._ctx, self._stats), "get_root_stats")
        return self._stats

    def headroom(self, stats=None):
        """Simulations (of either level) that can still run in every pair
        before the next update without overflowing a tree's arenas: each one
        adds at most ``L`` nodes, statistics blocks and log records to each
        tree, and the next update's reinvigoration is kept in reserve.  Uses
        the counters of ``stats`` (``root_stats()``'s last result)."""
        cfg, caps = self.config, self.capacities
        L = min(cfg.depth_limit, self.step_limit) + 1
        target = cfg.num_particles + cfg.extra_particles
        reinv = int(math.ceil(cfg.reinvigoration_sample_limit_factor * target)) + target
        reserve = 2 * reinv + 2 * target + 8        # plan_intmcp_capacities' per-update share
        room = INT32_MAX
        if getattr(self, "nesting_level", 1) >= 2:   # 3+ trees: intmcp_get_tree_counts
            cnt = self.tree_counts()
            for p in range(self.num_pairs):
                for t in range(self.nesting_level + 1):
                    left = min(caps.max_nodes - cnt[p, t, 0], caps.max_log - cnt[p, t, 1],
                               (caps.max_stats - cnt[p, t, 2]) // self.A) - reserve
                    room = min(room, left // L)
            return max(0, int(room))
        st = self._stats if stats is None else stats
        for p in range(self.num_pairs):
            for t in range(2):
                left = min(caps.max_nodes - st[p].n_nodes[t], caps.max_log - st[p].n_log[t],
                           (caps.max_stats - st[p].n_stats[t]) // self.A) - reserve
                room = min(room, left // L)
        return max(0, room)

    def root_belief(self, pair=0):
        """Level-1 root particles as (v0, v1, level-0 node) u32 rows; at
        nesting level 0 the planner's root particles as (v0, v1) rows."""
        if self.nesting_level == 0:
            ent, parts = self.support(pair)
            if len(ent) == 0:
                return parts[:0]
            return parts[int(ent[0]["off"]):int(ent[0]["off"]) + int(ent[0]["size"])]
        n = C.c_int32()
        self._check(self._lib.intmcp_get_root_belief(self._ctx, pair, None, 0, C.byref(n)),
                    "get_root_belief")
        buf = np.zeros(3 * max(n.value, 1), dtype=np.uint32)
        self._check(self._lib.intmcp_get_root_belief(
            self._ctx, pair, buf.ctypes.data_as(C.POINTER(C.c_uint32)), n.value, C.byref(n)),
            "get_root_belief")
        return buf[:3 * n.value].reshape(-1, 3)

    def _records(self, fn, pair, tree, dtype):
        n = C.c_int32()
        self._check(fn(self._ctx, pair, tree, None, 0, C.byref(n)), fn.__name__)
        out = np.zeros(max(n.value, 1), dtype=dtype)
        self._check(fn(self._ctx, pair, tree, out.ctypes.data_as(C.c_void_p), n.value,
                       C.byref(n)), fn.__name__)
        return out[:n.value]

    def nodes(self, pair=0, tree=0):
        """Obs nodes of one tree (0: the planner's level, then one level down per
        tree) as a structured array."""
        return self._records(self._lib.intmcp_get_nodes, pair, tree, N.INTMCP_NODE_DTYPE)

    def stats(self, pair=0, tree=0):
        return self._records(self._lib.intmcp_get_stats, pair, tree, N.INTMCP_STAT_DTYPE)

    def mid_support(self, pair=0, tree=1):
        """Nesting levels 2, 3: middle tree ``tree``'s materialised beliefs:
        (entries, (v0, v1, next tree's node) particles)."""
        ne, npart = C.c_int32(), C.c_int32()
        fn = self._lib.intmcp_get_middle_support
        self._check(fn(self._ctx, pair, tree, None, 0, C.byref(ne), None, 0, C.byref(npart)),
                    "get_middle_support")
        ent = np.zeros(max(ne.value, 1), dtype=N.INTMCP_SUPPORT_DTYPE)
        parts = np.zeros(3 * max(npart.value, 1), dtype=np.uint32)
        self._check(fn(
            self._ctx, pair, tree, ent.ctypes.data_as(C.POINTER(C.c_int32)), ne.value, C.byref(ne),
            parts.ctypes.data_as(C.POINTER(C.c_uint32)), npart.value, C.byref(npart)),
            "get_middle_support")
        return ent[:ne.value], parts[:3 * npart.value].reshape(-1, 3)

    def support(self, pair=0):
        """The materialised level-0 beliefs: (entries, (v0, v1) particles)."""
        ne, npart = C.c_int32(), C.c_int32()
        self._check(self._lib.intmcp_get_support(self._ctx, pair, None, 0, C.byref(ne), None, 0,
                                                 C.byref(npart)), "get_support")
        ent = np.zeros(max(ne.value, 1), dtype=N.INTMCP_SUPPORT_DTYPE)
        parts = np.zeros(2 * max(npart.value, 1), dtype=np.uint32)
        self._check(self._lib.intmcp_get_support(
            self._ctx, pair, ent.ctypes.data_as(C.POINTER(C.c_int32)), ne.value, C.byref(ne),
            parts.ctypes.data_as(C.POINTER(C.c_uint32)), npart.value, C.byref(npart)),
            "get_support")
        return ent[:ne.value], parts[:2 * npart.value].reshape(-1, 2)

    def synthetic_obs(self, env_seed_base):
        out = np.zeros(self.num_pairs, dtype=np.uint64)
        self._check(self._lib.intmcp_synthetic_obs(
            self._ctx, int(env_seed_base), out.ctypes.data_as(C.POINTER(C.c_uint64))),
            "synthetic_obs")
        return out


def node_order(info: int):
    """Registered actions of a node, registration order (``ObsNode.children``)."""
    n = (int(info) >> 5) & 7
    return [(int(info) >> (8 + 3 * i)) & 7 for i in range(n)]


@dataclasses.dataclass
class RootView:
    """Read-only view of the level-1 root node."""

    t: int = 0
    is_absorbing: bool = False
    visits: int = 0
    children: tuple = ()          # (action, visits, value, total), registration order
    belief_size: int = 0


class _NestedPlanner:
    """A lower-level planner (``other_agent_policies[j]``, and its own at
    nesting level 2): a view of the device state shared with the top planner."""

    def __init__(self, parent, agent_id, nesting_level=0):
        self._parent = parent
        self.model = parent.model
        self.agent_id = agent_id
        self.config = parent.config
        self.nesting_level = nesting_level
        below = [i for i in parent.model.possible_agents if i != agent_id][0]
        self.other_agent_policies = ({below: _NestedPlanner(parent, below, nesting_level - 1)}
                                     if nesting_level > 0 else {})
        self.step_statistics = {"reinvigoration_time": 0.0}

    def reset(self):
        pass

    def close(self):
        pass

    def _collect_nested_statistics(self):
        return {"reinvigoration_time": 0.0}

    def __str__(self):
        return "INTMCP"


class INTMCP:
    """Interactive Nested Tree Monte-Carlo Planning, GPU-resident trees.

    Built with :meth:`initialize` (as in the reference).  With ``num_sims``
    set (``MCTSConfig.num_sims`` or the keyword) every ``get_action`` runs
    exactly that many simulations per nesting level; otherwise the
    ``search_time_limit`` is split evenly over the levels (``intmcp.py:383-397``).
    """

    def __init__(self, model, agent_id: str, config: MCTSConfig, nesting_level: int,
                 other_agent_policies=None, search_policies=None, *,
                 num_sims: Optional[int] = None):
        if not 0 <= int(nesting_level) <= MAX_NESTING:
            raise NotImplementedError(f"the GPU I-NTMCP engine runs nesting levels 0 to {MAX_NESTING}")
        from posggym_baselines_amd.planning.ipomcp import search_policy_probs
        assert agent_id in model.possible_agents
        # {level: {agent: policy}} (INTMCP.initialize) or one {agent: policy}
        # dict for every level
        if search_policies is not None and not all(
                isinstance(v, dict) for v in search_policies.values()):
            search_policies = {lv: search_policies for lv in range(nesting_level + 1)}
        self._search_probs = {
            lv: {i: search_policy_probs(model, i, pol) for i, pol in pols.items()}
            for lv, pols in (search_policies or {}).items()}
        self.model = model
        self._emodel = engine_model(model)
        self.agent_id = agent_id
        self.config = config
        self.nesting_level = nesting_level
        self.num_agents = len(model.possible_agents)
        # this planner's own level's policies (intmcp.py:985: search_policies[nesting_level])
        self.search_policies = (search_policies or {}).get(nesting_level) or {
            i: RandomSearchPolicy(model, i) for i in model.possible_agents}
        self.action_spaces = {i: list(range(model.action_spaces[i].n))
                              for i in model.possible_agents}
        other = [i for i in model.possible_agents if i != agent_id][0]
        # intmcp.py:971-981: a level-0 planner models no other agent; a level-2
        # planner's other agent is a level-1 planner modelling this agent at level 0
        self.other_agent_policies = ({other: _NestedPlanner(self, other, nesting_level - 1)}
                                     if nesting_level else {})
        self._num_sims = num_sims if num_sims is not None else config.num_sims
        self._engine = IntmcpEngine(model, agent_id, config, num_pairs=1,
                                    num_sims=self._num_sims,
                                    wall_clock=self._num_sims is None,
                                    nesting_level=nesting_level)
        for lv, probs in self._search_probs.items():
            if lv > nesting_level:
                continue
            for i, pr in probs.items():
                self._engine.set_search_policy(lv, model.possible_agents.index(i), pr)
        self.step_limit = self._engine.step_limit
        self._logger = logging.getLogger()
        self._last_action = None
        self._step_num = 0
        self.root = RootView()
        self._min_value, self._max_value = self._initial_bounds()
        self.step_statistics = {}
        self._reset_step_statistics()
        self.stat_tracker = PlanningStatTracker(self)

    @classmethod
    def initialize(cls, model, ego_agent_id: str, config: MCTSConfig, nesting_level: int,
                   search_policies=None, *, num_sims: Optional[int] = None) -> "INTMCP":
        """``intmcp.py:949-994``; ``search_policies`` is ``{level: {agent: policy}}``
        (None: ``RandomSearchPolicy`` everywhere); a policy is a
        ``RandomSearchPolicy`` or a ``SearchPolicyWrapper(FixedDistributionPolicy)``
        (others raise ``NotImplementedError``)."""
        return cls(model, ego_agent_id, config, nesting_level, None, search_policies,
                   num_sims=num_sims)

    # ---------------------------------------------------------------- step
    def step(self, obs):
        """``intmcp.py:114-136``."""
        assert self.step_limit is None or self.root.t <= self.step_limit
        if self.root.is_absorbing:
            for k in self.step_statistics:
                self.step_statistics[k] = np.nan
            return self._last_action
        self._reset_step_statistics()
        self.update(self._last_action, obs)
        self._last_action = self.get_action()
        self._step_num += 1
        self.step_statistics["mem_usage"] = psutil.Process().memory_info().rss / 1024**2
        self.stat_tracker.step()
        return self._last_action

    def reset(self):
        """``intmcp.py:158-177``."""
        self.stat_tracker.reset_episode()
        self._step_num = 0
        self._engine.reset()
        self.root = RootView()
        self._min_value, self._max_value = self._initial_bounds()
        self._reset_step_statistics()
        self._last_action = None
        for pi in self.other_agent_policies.values():
            pi.reset()

    def _initial_bounds(self):
        kb = self.config.known_bounds
        return (kb[0], kb[1]) if kb else (float("inf"), -float("inf"))

    def _reset_step_statistics(self):
        self.step_statistics = {
            "search_time": 0.0, "update_time": 0.0, "reinvigoration_time": 0.0,
            "evaluation_time": 0.0, "policy_calls": 0, "inference_time": 0.0,
            "search_depth": 0, "num_sims": 0, "mem_usage": 0,
            "min_value": self._min_value, "max_value": self._max_value,
        }

    # -------------------------------------------------------------- update
    def update(self, action, obs):
        """``intmcp.py:198-214``: ``_initial_nested_update`` at t == 0, else
        ``_nested_update`` of both levels."""
        if self.root.is_absorbing:
            return
        start = time.time()
        a = -1 if self.root.t == 0 else int(action)
        key = self._emodel.obs_key(obs)
        absorbing = self._engine.update([a], [key])
        self.root = dataclasses.replace(self.root, t=self.root.t + 1,
                                        is_absorbing=bool(absorbing[0]))
        self.step_statistics["update_time"] = time.time() - start

    # -------------------------------------------------------------- search
    def get_action(self):
        """``intmcp.py:368-408``."""
        if self.root.is_absorbing:
            return self.action_spaces[self.agent_id][0]
        start = time.time()
        if self._num_sims is not None:
            self._engine.search(self._num_sims, fetch=False)
        else:
            # the reference's per-level time split (intmcp.py:383-397) as
            # launches of growing chunks, each within the arena headroom and the
            # per-level ceiling the arenas were sized for; a full arena ends the
            # search early (step_statistics "arena_full"), it does not fail
            per_level = self.config.search_time_limit / (self.nesting_level + 1)
            ceiling = self._engine.wall_clock_sims
            flags = N.INTMCP_BEGIN
            room = self._engine.headroom(self._engine.root_stats())
            for level in range(self.nesting_level + 1):
                t0, chunk, done = time.time(), 16, 0
                while time.time() - t0 < per_level and done < ceiling:
                    n = min(chunk, room, ceiling - done)
                    if n <= 0:
                        self.step_statistics["arena_full"] = True
                        break
                    self._engine.search_level(level, n, flags)
                    flags = 0
                    room = self._engine.headroom(self._engine.root_stats())   # synchronises
                    done += n
                    chunk = min(chunk * 2, 4096)
            self._engine.search_level(0, 0, flags | N.INTMCP_FINAL)
        st = self._engine.root_stats()[0]
        search_time = time.time() - start
        self._min_value, self._max_value = st.min_value, st.max_value
        kids = tuple((int(st.child_action[i]), int(st.child_visits[i]), st.child_values[i],
                      st.child_totals[i]) for i in range(st.num_children))
        self.root = dataclasses.replace(self.root, visits=st.root_visits,
                                        belief_size=st.belief_size, children=kids)
        self.step_statistics.update(
            search_time=search_time, search_depth=st.search_depth, num_sims=int(st.num_sims),
            min_value=st.min_value, max_value=st.max_value)
        return int(st.action)

    def root_belief(self):
        """Root particles: (v0, v1, level-0 node id) rows at nesting level 1,
        (v0, v1) rows at nesting level 0."""
        return self._engine.root_belief(0)

    def close(self):
        for p in self.search_policies.values():
            if hasattr(p, "close"):
                p.close()
        self._engine.close()

    def __str__(self):
        return "INTMCP"


class BatchedINTMCP:
    """``num_pairs`` independent I-NTMCP planner pairs searched by one launch.

    Pair ``b`` uses RNG key ``(seed, tree_key_base + b)``: bit-identical to a
    single ``INTMCP`` (and to the oracle) with that key.
    """

    def __init__(self, model, agent_id, config: MCTSConfig, num_pairs: int, num_sims: int, *,
                 searches: int = 1, capacities=None, stream=None, tree_key_base: int = 0,
                 device: Optional[int] = None, nesting_level: int = 1):
        if capacities is None:
            step_limit = config.step_limit or model.spec.max_episode_steps
            capacities = plan_intmcp_capacities(config, step_limit, num_sims, searches,
                                                model.action_spaces[agent_id].n, nesting_level)
        self.num_pairs = num_pairs
        self.num_sims = num_sims
        self.engine = IntmcpEngine(model, agent_id, config, num_pairs=num_pairs,
                                   capacities=capacities, stream=stream,
                                   tree_key_base=tree_key_base, device=device,
                                   nesting_level=nesting_level)
        self.engine.reset()

    def init_synthetic(self, env_seed_base: int = 1000):
        keys = self.engine.synthetic_obs(env_seed_base)
        self.engine.update(np.full(self.num_pairs, -1, dtype=np.int32), keys)
        return keys

    def search(self, fetch=True):
        return self.engine.search(self.num_sims, fetch=fetch)

    def close(self):
        self.engine.close()
