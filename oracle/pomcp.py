"""POMCP hot path — CPU restatement of the reference (pure Python).

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

Restates ``posggym_baselines.planning.mcts.MCTS`` as used by ``POMCP``
(``pomcp.py:20-35``: random other agents, ``state_belief_only=True``) with a
``RandomSearchPolicy`` (``search_policy.py:158-185``).  The tree is kept in
flat arrays (the layout the HIP kernels use) instead of node objects; the
arithmetic and the order of every random draw follow the reference line by
line (citations inline).  Pinned by ``tests/golden/*.json``, which
``oracle/ref_harness.py`` produced by running the real reference planner.
"""
import math

from oracle.rng import S_BELIEF, S_SELECT, Streams

INF = float("inf")


class OracleConfig:
    """The derived fields of ``MCTSConfig`` (``config.py:8-55``)."""

    def __init__(self, discount, search_time_limit, c, truncated=False,
                 action_selection="pucb", pucb_exploration_fraction=0.5,
                 known_bounds=None, extra_particles_prop=1.0 / 16,
                 reinvigoration_sample_limit_factor=4.0, step_limit=None,
                 epsilon=0.01, seed=None, state_belief_only=True, num_sims=None):
        assert 0.0 <= discount <= 1.0
        assert search_time_limit > 0.0 and c > 0.0
        assert 0.0 < epsilon < 1.0
        self.discount = discount
        self.search_time_limit = search_time_limit
        self.c = c
        self.truncated = truncated
        self.action_selection = action_selection.lower()
        assert self.action_selection in ("pucb", "ucb", "uniform")
        self.pucb_exploration_fraction = pucb_exploration_fraction
        self.known_bounds = known_bounds
        self.extra_particles_prop = extra_particles_prop
        self.reinvigoration_sample_limit_factor = reinvigoration_sample_limit_factor
        self.step_limit = step_limit
        self.epsilon = epsilon
        self.seed = seed
        self.state_belief_only = state_belief_only
        self.num_sims = num_sims
        # config.py:47-55
        self.num_particles = math.ceil(100 * search_time_limit)
        self.extra_particles = math.ceil(self.num_particles * extra_particles_prop)
        if discount == 0.0:
            self.depth_limit = 0
        else:
            self.depth_limit = math.ceil(math.log(epsilon) / math.log(discount))


class OraclePOMCP:
    """One POMCP planner (one tree).  ``streams`` carries every RNG family."""

    def __init__(self, model, agent_id, cfg: OracleConfig, streams: Streams):
        assert cfg.num_sims is not None, "oracle runs fixed simulation counts"
        self.model = model
        self.agent_id = agent_id
        self.ego = model.possible_agents.index(agent_id)
        self.cfg = cfg
        self.s = streams
        self.A = model.action_spaces[agent_id].n
        # mcts.py:53-58
        if cfg.step_limit is not None:
            self.step_limit = cfg.step_limit
        elif getattr(model, "spec", None) is not None:
            self.step_limit = model.spec.max_episode_steps
        else:
            self.step_limit = INF
        self.reset()

    # ------------------------------------------------------------------ tree
    def _new_obs_node(self, t, visits, absorbing=False):
        i = len(self.on_block)
        self.on_block.append(-1)
        self.on_visits.append(visits)
        self.on_t.append(t)
        self.on_abs.append(absorbing)
        self.belief.append([])
        return i

    def _expand(self, node):
        """``ObsNode.add_child`` for every action (``mcts.py:279-281, 320-321``)."""
        b = len(self.an_visits) // self.A
        self.on_block[node] = b
        self.an_visits.extend([0] * self.A)
        self.an_value.extend([0.0] * self.A)
        self.an_total.extend([0.0] * self.A)
        self.an_agg.extend([0] * self.A)
        return b

    def reset(self):
        """``MCTS.reset`` (``mcts.py:123-138``)."""
        self.on_block, self.on_visits, self.on_t, self.on_abs, self.belief = [], [], [], [], []
        self.an_visits, self.an_value, self.an_total, self.an_agg = [], [], [], []
        self.children = {}
        kb = self.cfg.known_bounds
        self.mm_max, self.mm_min = (kb[1], kb[0]) if kb else (-INF, INF)   # utils.py:21-27
        self.root = self._new_obs_node(0, 0)
        self.last_action = None
        self.stats = {}

    # ---------------------------------------------------------------- minmax
    def _mm_update(self, v):                 # utils.py:29-32 (max()/min() keep first arg on ties)
        if v > self.mm_max:
            self.mm_max = v
        if v < self.mm_min:
            self.mm_min = v

    def _normalize(self, v):                 # utils.py:34-39
        if self.mm_max > self.mm_min:
            return (v - self.mm_min) / (self.mm_max - self.mm_min)
        return v

    # ------------------------------------------------------------------ step
    def step(self, obs):
        """``MCTS.step`` (``mcts.py:97-117``)."""
        assert self.on_t[self.root] <= self.step_limit
        if self.on_abs[self.root]:
            self.stats = {"searched": False}
            return self.last_action
        self.stats = {"searched": True}
        self.update(self.last_action, obs)
        self.last_action = self.get_action()
        return self.last_action

    def update(self, action, obs):
        """``MCTS.update`` (``mcts.py:159-173``)."""
        if self.on_abs[self.root]:
            return
        if self.on_t[self.root] == 0:
            self.last_action = None
            self._initial_update(obs)
        else:
            self._update(action, obs)
        self.stats["belief_size"] = len(self.belief[self.root])
        self.stats["belief"] = list(self.belief[self.root])

    def _initial_update(self, obs):
        """``mcts.py:175-227``: rejection/direct sampling of b0."""
        m = self.model
        # mcts.py:176-177: root -> action None -> obs node (init_visits=0)
        node = self._new_obs_node(self.on_t[self.root] + 1, 0)
        try:                                          # mcts.py:179-184 (probe draws)
            m.sample_agent_initial_state(self.agent_id, obs)
            rejection = False
        except NotImplementedError:
            rejection = True
        target = self.cfg.num_particles + self.cfg.extra_particles
        parts = self.belief[node]
        while len(parts) < target:                    # mcts.py:188
            if rejection:
                st = m.sample_initial_state()
                jo = m.sample_initial_obs(st)
                if jo[self.agent_id] != obs:
                    continue
            else:
                st = m.sample_agent_initial_state(self.agent_id, obs)
                jo = m.sample_initial_obs(st)
            parts.append((st, 1))                     # HistoryPolicyState(state, None, None, t=1)
        self.root = node

    def _update(self, action, obs):
        """``mcts.py:229-263``: re-root to child (a, o), then reinvigorate."""
        root = self.root
        b = self.on_block[root]
        if b < 0:                                      # node.py:58-63 AssertionError
            raise AssertionError(f"root has no child node for {action=}")
        an = b * self.A + action
        key = (an, self.model.pack_obs(obs))
        child = self.children.get(key)
        if child is None:                              # mcts.py:240-247
            child = self._new_obs_node(self.on_t[root] + 1, 0, self.on_abs[root])
            self.children[key] = child
        if not self.on_abs[child]:
            self._reinvigorate(child, action, obs, root)
        self.root = child                              # mcts.py:261-263

    def _reinvigorate(self, node, action, obs, parent):
        """``mcts.py:651-700`` + ``belief.py:145-194`` (use_rejected_samples=True)."""
        n = self.cfg.num_particles + self.cfg.extra_particles - len(self.belief[node])
        if n <= 0:
            return
        pb = self.belief[parent]
        limit = self.cfg.reinvigoration_sample_limit_factor * n
        got, tries, rejected, accepted = 0, 0, [], []
        oid = 1 - self.ego
        while got < n and tries < limit:
            tries += 1
            st, t = pb[self.s.randint(S_BELIEF, len(pb))]          # belief.py:55
            ja = self._joint(action)
            ts = self.model.step(st, ja)
            rec = (ts.state, t + 1)
            if ts.observations[self.agent_id] == obs:
                accepted.append(rec)
                got += 1
            else:
                rejected.append(rec)
        if got < n:
            accepted.extend(rejected[: n - got])
        self.belief[node].extend(accepted)
        del oid

    # ---------------------------------------------------------------- search
    def _joint(self, ego_action):
        """``_get_joint_action`` (``mcts.py:602-615``), other agents random."""
        ja = {}
        for i in self.model.possible_agents:
            if i == self.agent_id:
                ja[i] = ego_action
            else:
                ja[i] = self.model.action_spaces[i].sample()     # other_policy.py:151
        return ja

    def get_action(self):
        """``mcts.py:269-306`` with a fixed simulation count."""
        root = self.root
        if self.on_abs[root]:
            self.stats.update(num_sims=0, search_depth=0)
            return 0
        if self.on_block[root] < 0:
            self._expand(root)
        max_depth = 0
        for _ in range(self.cfg.num_sims):
            parts = self.belief[root]
            st, t = parts[self.s.randint(S_BELIEF, len(parts))]   # belief.py:55
            self.s.align_sim()                                     # (rng.py SIM_STREAMS)
            depth = self._simulate(st, t, root)
            self.on_visits[root] += 1                              # mcts.py:288
            max_depth = max(max_depth, depth)
        b = self.on_block[root] * self.A
        self.stats.update(
            num_sims=self.cfg.num_sims, search_depth=max_depth,
            min_value=self.mm_min, max_value=self.mm_max,
            root_visits=self.on_visits[root],
            child_visits=self.an_visits[b:b + self.A],
            child_values=self.an_value[b:b + self.A],
            child_totals=self.an_total[b:b + self.A],
        )
        return self._final_selection(root)

    def _select(self, node):
        sel = self.cfg.action_selection
        visits = self.on_visits[node]
        b = self.on_block[node] * self.A
        A = self.A
        if sel == "ucb":                                 # mcts.py:529-546
            if visits == 0:
                return self.s.randint(S_SELECT, A)
            log_n = math.log(visits)
            best_v, best_a = -INF, 0
            for a in range(A):
                n = self.an_visits[b + a]
                if n == 0:
                    return a
                v = self._normalize(self.an_value[b + a]) + self.cfg.c * math.sqrt(log_n / n)
                if v > best_v:
                    best_v, best_a = v, a
            return best_a
        if sel == "pucb":                                # mcts.py:492-527
            probs = [1.0 / A] * A                        # uniform get_pi, EMA-invariant
            if visits == 0:
                cum, acc = [], 0.0
                for k, w in enumerate(probs):
                    acc = w if k == 0 else acc + w
                    cum.append(acc)
                x = self.s.random(S_SELECT) * (cum[-1] + 0.0)
                lo, hi = 0, A - 1
                while lo < hi:
                    mid = (lo + hi) // 2
                    if x < cum[mid]:
                        hi = mid
                    else:
                        lo = mid + 1
                return lo
            f = self.cfg.pucb_exploration_fraction
            noise = 1 / A
            sqrt_n = math.sqrt(visits)
            best_v, best_a = -INF, 0
            for a in range(A):
                n = self.an_visits[b + a]
                prior = probs[a] * (1 - f) + f * noise
                explore = self.cfg.c * prior * (sqrt_n / (1 + n))
                v = (self._normalize(self.an_value[b + a]) if n > 0 else 0) + explore
                if v > best_v:
                    best_v, best_a = v, a
            return best_a
        # "uniform" -> min_visit_action_selection, mcts.py:548-563
        if visits == 0:
            return self.s.randint(S_SELECT, A)
        min_n, nxt = visits + 1, 0
        for a in range(A):
            if self.an_visits[b + a] < min_n:
                min_n, nxt = self.an_visits[b + a], a
        return nxt

    def _final_selection(self, node):
        A = self.A
        b = self.on_block[node]
        if self.cfg.action_selection == "pucb":           # max_visit, mcts.py:565-581
            if self.on_visits[node] == 0:
                return self.s.randint(S_SELECT, A)
            best, mx = [], 0
            for a in range(A):
                n = self.an_visits[b * A + a]
                if n == mx:
                    best.append(a)
                elif n > mx:
                    mx, best = n, [a]
            return best[self.s.randint(S_SELECT, len(best))]
        if b < 0:                                          # max_value, mcts.py:583-600
            return self.s.randint(S_SELECT, A)
        best, mx = [], -INF
        for a in range(A):
            v = self.an_value[b * A + a]
            if v == mx:
                best.append(a)
            elif v > mx:
                mx, best = v, [a]
        return best[self.s.randint(S_SELECT, len(best))]

    def _simulate(self, st, t, node):
        """Iterative ``_simulate`` (``mcts.py:308-382``); returns the search depth."""
        cfg = self.cfg
        A = self.A
        depth = 0
        path = []                       # (action node, reward, done) per tree level
        leaf_value = 0
        while True:
            if depth > cfg.depth_limit or self.on_t[node] > self.step_limit:   # mcts.py:315
                leaf_value = 0
                break
            if self.on_block[node] < 0:                                         # mcts.py:318-328
                self._expand(node)
                leaf_value = self._rollout(st, t, depth)
                break
            a = self._select(node)                                              # mcts.py:330
            ts = self.model.step(st, self._joint(a))                            # mcts.py:331-333
            r = ts.rewards[self.agent_id]
            done = (ts.terminations[self.agent_id] or ts.truncations[self.agent_id]
                    or ts.all_done)
            an = self.on_block[node] * A + a
            key = (an, self.model.pack_obs(ts.observations[self.agent_id]))
            child = self.children.get(key)
            if child is not None:                                               # mcts.py:358-367
                self.on_visits[child] += 1
            else:                                                               # mcts.py:369
                child = self._new_obs_node(self.on_t[node] + 1, 1)
                self.children[key] = child
            self.on_abs[child] = done                                           # mcts.py:370
            self.belief[child].append((ts.state, t + 1))                        # mcts.py:371
            path.append((an, r, done))
            if done:
                break
            node, st, t = child, ts.state, t + 1
            depth += 1
        # backup, deepest level first (mcts.py:374-381)
        g = leaf_value
        for an, r, done in reversed(path):
            g = r if done else r + cfg.discount * g
            n = self.an_visits[an] + 1                                           # node.py:173-178
            self.an_visits[an] = n
            self.an_total[an] += g
            delta = g - self.an_value[an]
            self.an_value[an] += delta / n
            self.an_agg[an] += delta * (g - self.an_value[an])
            self._mm_update(self.an_value[an])
        return depth

    def _rollout(self, st, t, depth):
        """``mcts.py:405-452`` with the random search policy."""
        cfg = self.cfg
        ego_id = self.agent_id
        ret = 0
        k = 0
        while depth <= cfg.depth_limit and t <= self.step_limit:
            a = self.model.action_spaces[ego_id].sample()          # search_policy.py:177
            ts = self.model.step(st, self._joint(a))
            ret += cfg.discount ** k * ts.rewards[ego_id]          # mcts.py:420-422
            if ts.terminations[ego_id] or ts.truncations[ego_id] or ts.all_done:
                break
            st, t = ts.state, t + 1
            depth += 1
            k += 1
        return ret
