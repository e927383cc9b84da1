"""POMCP drop-in: the reference's ``POMCP`` API (``pomcp.py:9-35`` on top of
``mcts.py:22-739``) with the search, the tree, the particle beliefs and the
generative model on the GPU.

Public surface kept from the reference: ``POMCP(model, agent_id, config,
search_policy)``, ``step(obs)``, ``reset()``, ``update(action, obs)``,
``get_action()``, ``close()``, and the attributes ``model``, ``agent_id``,
``config``, ``other_agent_policies``, ``search_policy``, ``step_statistics``,
``stat_tracker``, ``root``.

``BatchedPOMCP`` runs many independent planners (one tree each) in one kernel
launch; it is what the bench and batch experiments use.

``MCTSConfig.root_parallel = K > 1`` gives ONE planner K replica trees on the
GPU (root parallelisation): replica k is the exact single-tree planner with
RNG key (seed, k), every replica is updated with the played action and the
real observation, searches ceil(num_sims / K) simulations, and the played
action is the device merge of the replicas' root statistics
(``pomcp_merge_roots``: summed visits for PUCB, summed total / summed visits
otherwise).  K = 1 (default) is the reference's planner, bit-exact.

``POMCP(..., process_group=pg)`` spreads the replicas over the ranks of a
``torch.distributed`` group (one process per GPU, backend "nccl" = RCCL):
rank r's replicas take keys (seed, r*K .. r*K+K-1), ``num_sims`` is split over
all world x K replicas (ceil(num_sims / (world K)) each), and before the
decision one all-gather collects every rank's replica records
(``parallel.exchange_roots``); the device merge sums the world x K replicas in
one fixed order, so every rank plays the same action and reports the same
step statistics (simulations and root visits summed over all replicas,
min / max over them).  A failure on any rank (arena, HIP) is agreed on before
each collective and raised on every rank (``parallel.raise_together``), so no
rank waits forever in a collective its peer never reaches.
"""
import dataclasses
import logging
import math
import time
from typing import Optional

import numpy as np
import psutil

from posggym_baselines_amd.envs import engine_model

from posggym_baselines_amd.planning.config import MCTSConfig
from posggym_baselines_amd.planning.engine import PomcpEngine, search_bytes
from posggym_baselines_amd.planning.other_policy import RandomOtherAgentPolicy
from posggym_baselines_amd.planning.search_policy import RandomSearchPolicy, SearchPolicy
from posggym_baselines_amd.planning.utils import PlanningStatTracker


@dataclasses.dataclass
class RootView:
    """Read-only view of the GPU root node (``ObsNode`` fields the callers use)."""

    t: int = 0
    is_absorbing: bool = False
    visits: int = 0
    child_visits: tuple = ()
    child_values: tuple = ()
    child_totals: tuple = ()
    belief_size: int = 0


class POMCP:
    """Partially Observable Monte-Carlo Planning, GPU-resident tree.

    Other agents are random (``pomcp.py:28-31``).  The search policy is the
    uniform random one (``RandomSearchPolicy``, the reference's POMCP test
    setup, ``tests/planning/test_pomcp.py:36-74``: the plain kernel) or a
    fixed-distribution one (``SearchPolicyWrapper(FixedDistributionPolicy)``:
    node priors and rollouts, planning/ipomcp.py); history-dependent
    (network) search policies raise ``NotImplementedError``.
    """

    def __init__(self, model, agent_id: str, config: MCTSConfig, search_policy: SearchPolicy,
                 *, num_sims: Optional[int] = None, process_group=None):
        from posggym_baselines_amd.planning.ipomcp import base_type_tables
        if not config.state_belief_only:
            # pomcp.py:32-34 calls config.replace(...), which does not exist on the
            # dataclass (AttributeError in the reference); dataclasses.replace is
            # what it means.  Recorded in DESIGN.md.
            config = dataclasses.replace(config, state_belief_only=True)
        others = {i: RandomOtherAgentPolicy(model, i) for i in model.possible_agents if i != agent_id}
        tables = base_type_tables(model, agent_id, config, others, search_policy)
        self.type_policies = tables
        self._init_planner(model, agent_id, config, search_policy, others, num_sims, process_group,
                           type_policies=tables)

    def _init_planner(self, model, agent_id, config, search_policy, other_agent_policies,
                      num_sims, process_group, type_policies=None):
        self.model = model
        self._emodel = engine_model(model)
        self.agent_id = agent_id
        self.config = config
        self.search_policy = search_policy
        self.other_agent_policies = other_agent_policies
        self.num_agents = len(model.possible_agents)
        self.action_space = list(range(model.action_spaces[agent_id].n))
        self._num_sims = num_sims if num_sims is not None else config.num_sims
        self._K = int(config.root_parallel)
        self._pg = process_group
        self._rank, self._world = 0, 1
        if process_group is not None:
            import torch.distributed as dist
            self._rank = dist.get_rank(process_group)
            self._world = dist.get_world_size(process_group)
        replicas = self._K * self._world
        per = math.ceil(self._num_sims / replicas) if self._num_sims is not None else None
        self._per_replica = per
        self._engine = PomcpEngine(model, agent_id, config, num_trees=self._K,
                                   num_sims=per, tree_key_base=self._rank * self._K,
                                   wall_clock=per is None, type_policies=type_policies)
        # cut-off children are deferred to the re-root (the engine's default):
        # with their bulk materialisation in k_compact_log that is the faster
        # mode for an episode planner too (pomcp_set_defer_cutoff; same results,
        # DESIGN.md §4 "Deferred records")
        self.step_limit = self._engine.step_limit
        self._logger = logging.getLogger()
        self._last_action = None
        self._step_num = 0
        self.root = RootView()
        self.step_statistics = {}
        self._reset_step_statistics()
        self.stat_tracker = PlanningStatTracker(self)

    # ---------------------------------------------------------------- step
    def step(self, obs):
        """``mcts.py:97-117``."""
        assert self.root.t <= self.step_limit
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
        """``mcts.py:123-138``."""
        self.stat_tracker.reset_episode()
        self._step_num = 0
        self._engine.reset()
        self.root = RootView()
        self._min_value, self._max_value = self._initial_bounds()
        self._reset_step_statistics()
        self._last_action = None

    def _initial_bounds(self):
        kb = self.config.known_bounds
        return (kb[0], kb[1]) if kb else (float("inf"), -float("inf"))

    def _reset_step_statistics(self):
        if not hasattr(self, "_min_value"):
            self._min_value, self._max_value = self._initial_bounds()
        self.step_statistics = {
            "search_time": 0.0, "update_time": 0.0, "reinvigoration_time": 0.0,
            "evaluation_time": 0.0, "policy_calls": 0, "inference_time": 0.0,
            "search_depth": 0, "num_sims": 0, "mem_usage": 0,
            "min_value": self._min_value, "max_value": self._max_value,
            # the build's additions (SURVEY §5 metrics): the search's algorithmic
            # HBM bytes on this rank (engine.search_bytes) and its simulations/s
            "hbm_bytes": 0, "sims_per_s": 0.0,
        }

    # -------------------------------------------------------------- update
    def update(self, action, obs):
        """``mcts.py:159-263``: initial belief at t == 0, else re-root + reinvigorate."""
        if self.root.is_absorbing:
            return
        start = time.time()
        if self.root.t == 0:
            self._last_action = None
            a = -1
        else:
            a = int(action)
        key = self._emodel.obs_key(obs)
        if self._world == 1:
            absorbing = self._engine.update([a], [key])   # broadcast to every replica
            # a replica whose root is absorbing stops searching and merges as zeros;
            # the planner is absorbing once all of them are (oracle/root_parallel.py)
            done = bool(np.all(absorbing))
        else:
            # every rank must stop calling the collectives together: absorbing
            # only when every replica of every rank is, and a failed update on
            # any rank raises on all of them
            from posggym_baselines_amd.planning.parallel import raise_together
            exc, done = None, False
            try:
                done = bool(np.all(self._engine.update([a], [key])))
            except Exception as e:  # noqa: BLE001 -- re-raised after the agreement
                exc = e
            rows = raise_together(exc, [1.0 if done else 0.0], self._pg, self._device())
            done = bool(np.all(rows[:, 1] > 0))
        self.root = dataclasses.replace(self.root, t=self.root.t + 1, is_absorbing=done)
        self.step_statistics["update_time"] = time.time() - start

    # -------------------------------------------------------------- search
    def get_action(self):
        """``mcts.py:269-306`` (fixed ``num_sims``, or chunks until the time limit)."""
        if self.root.is_absorbing:
            return self.action_space[0]
        start = time.time()
        K, world = self._K, self._world
        exc, depth, n_sims = None, 0, 0
        self._hbm = 0
        try:
            depth, n_sims = self._search(start)
        except Exception as e:  # noqa: BLE001 -- raised on every rank below
            if world == 1:
                raise
            exc = e
        A = len(self.action_space)
        if world > 1:
            from posggym_baselines_amd.planning.parallel import exchange_roots, raise_together
            rows = raise_together(exc, [n_sims, depth], self._pg, self._device())
            n_sims, depth = int(rows[:, 1].sum()), int(rows[:, 2].max())
            exchange_roots(self._engine, self._device(), self._pg)
        if K == 1 and world == 1:
            st = self._engine.root_stats()[0]
            action = int(st.action)
            visits, belief_size = st.root_visits, st.belief_size
            cv, cval, ctot = (tuple(st.child_visits[:A]), tuple(st.child_values[:A]),
                              tuple(st.child_totals[:A]))
        else:
            # the merged decision (raises on every rank if any replica failed)
            st = self._engine.merge_roots(K, world=world if world > 1 else 0)[0]
            action = int(st.action)
            visits, belief_size = st.root_visits, None
            cv = tuple(int(v) for v in st.visits[:A])
            ctot = tuple(st.totals[:A])
            cval = tuple(t / v if v > 0 else 0.0 for t, v in zip(ctot, cv))
        search_time = time.time() - start
        if self._hbm is None:   # this rank's replicas' algorithmic bytes (engine.search_bytes)
            self._hbm = search_bytes(self._engine.root_stats(), A, self._engine.type_based)
        self._min_value, self._max_value = st.min_value, st.max_value
        self.root = dataclasses.replace(
            self.root, visits=visits, belief_size=belief_size, child_visits=cv,
            child_values=cval, child_totals=ctot)
        self.step_statistics.update(
            search_time=search_time, search_depth=max(depth, st.search_depth), num_sims=n_sims,
            min_value=st.min_value, max_value=st.max_value, hbm_bytes=self._hbm,
            sims_per_s=n_sims / search_time if search_time > 0 else 0.0)
        return action

    def _device(self):
        return f"cuda:{self.config.device}"

    def _search(self, start):
        """This rank's simulations of one get_action; returns (search depth
        seen by the chunk loop, simulations run by this rank's replicas)."""
        K, depth = self._K, 0
        A = len(self.action_space)
        tb = self._engine.type_based
        if self._num_sims is not None:
            self._engine.search(self._per_replica, fetch=False)
            self._hbm = None   # counted after the decision (errors surface in the merge first)
            return depth, self._per_replica * K
        # the wall-clock loop (mcts.py:285) as launches of growing chunks; the
        # final action choice is drawn once, after the last one.  A chunk is
        # never larger than the arena headroom (PomcpEngine.headroom) nor than
        # what is left of the per-search bound the arenas were sized for
        # (wall_clock_sims: the log(N) table and the kept subtree assume at most
        # that many simulations per search): when either is reached the search
        # ends early (step_statistics "arena_full"), it does not fail.
        done, chunk = 0, 16
        ceiling = self._engine.wall_clock_sims
        room = self._engine.headroom()
        while time.time() - start < self.config.search_time_limit:
            n = min(chunk, room, ceiling - done)
            if n <= 0:
                self.step_statistics["arena_full"] = True
                break
            self._engine.search(n, final=False)
            room = self._engine.headroom()    # synchronises
            depth = max(depth, self._depth())
            self._hbm += search_bytes(self._engine.root_stats(), A, tb)   # this chunk's
            done += n
            chunk = min(chunk * 2, 4096)
        self._engine.search(0, fetch=False)
        return depth, done * K

    def _depth(self):
        if self._K == 1:
            return self._engine.root_stats()[0].search_depth
        return self._engine.merge_roots(self._K)[0].search_depth

    def set_root_belief(self, rows):
        """Search from a caller-supplied belief: after ``reset()``, the root
        becomes an unexpanded node at time t holding ``rows`` ((t, v0, v1) packed
        particles, insertion order; ``pomcp_set_root_belief``) in every replica,
        in place of the initial update's b0 samples (mcts.py:175-227)."""
        rows = np.asarray(rows, dtype=np.uint32).reshape(-1, 3)
        for k in range(self._K):
            self._engine.set_root_belief(k, rows)
        self.root = RootView(t=int(rows[0, 0]), belief_size=len(rows))

    def root_belief(self, replica: int = 0):
        """Root particles as (t, v0, v1) packed u32 rows (of one replica)."""
        return self._engine.root_belief(replica)

    def close(self):
        self.search_policy.close()
        for p in self.other_agent_policies.values():
            p.close()
        self._engine.close()

    def __str__(self):
        return "POMCP"


class BatchedPOMCP:
    """``num_trees`` independent POMCP planners searched by one launch.

    Tree ``b`` uses RNG key ``(seed, tree_key_base + b)``; each tree is
    bit-identical to a single ``POMCP`` (and to the oracle) with that key.
    """

    def __init__(self, model, agent_id, config: MCTSConfig, num_trees: int, num_sims: int,
                 *, searches: int = 1, reroot: bool = False, capacities=None, stream=None,
                 tree_key_base: int = 0, device: Optional[int] = None, type_policies=None,
                 defer_cutoff: bool = True):
        """defer_cutoff: defer cut-off children to the re-root (the default, the
        faster mode with or without an update after every search) or look them
        up during the search (False); same results (``pomcp_set_defer_cutoff``)."""
        from posggym_baselines_amd.planning.engine import plan_capacities
        if capacities is None:
            step_limit = config.step_limit or model.spec.max_episode_steps
            capacities = plan_capacities(config, step_limit, num_sims, searches, reroot=reroot,
                                         num_actions=model.action_spaces[agent_id].n)
        self.num_trees = num_trees
        self.num_sims = num_sims
        self.engine = PomcpEngine(model, agent_id, config, num_trees=num_trees,
                                  capacities=capacities, stream=stream,
                                  tree_key_base=tree_key_base, device=device,
                                  type_policies=type_policies)
        self.engine.set_defer_cutoff(defer_cutoff)
        self.engine.reset()

    def init_synthetic(self, env_seed_base: int = 1000):
        """Synthetic Driving-v1 roots: per tree an env b0 sample and
        the initial belief update; snapshot so ``restore()`` can re-search them."""
        keys = self.engine.synthetic_obs(env_seed_base)
        self.engine.update(np.full(self.num_trees, -1, dtype=np.int32), keys)
        self.engine.snapshot()
        return keys

    def search(self, fetch=True):
        return self.engine.search(self.num_sims, fetch=fetch)

    def restore(self):
        self.engine.restore()

    def close(self):
        self.engine.close()


def uct_merge(visits: np.ndarray, totals: np.ndarray) -> np.ndarray:
    """Root-parallel decision from summed (visits, total value) per action:
    argmax of mean value, lowest index on ties."""
    with np.errstate(invalid="ignore", divide="ignore"):
        v = np.where(visits > 0, totals / np.maximum(visits, 1), -math.inf)
    return np.argmax(v, axis=-1)
