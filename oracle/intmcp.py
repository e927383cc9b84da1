"""I-NTMCP hot path (nesting levels 0-3, two agents) — CPU restatement (pure Python).

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

Restates ``posggym_baselines.planning.intmcp.INTMCP`` as built by
``INTMCP.initialize(model, ego, config, nesting_level=1, search_policies=None)``
(``intmcp.py:949-994``: random search policies at every level) with
``state_belief_only=False`` (``tests/planning/test_intmcp.py:34-71``): the ego's
level-1 tree and the other agent's level-0 tree.  The trees are flat arrays
(the layout the HIP kernels use); the arithmetic and the order of every random
draw follow the reference (citations inline).  Pinned by
``tests/golden/intmcp_*.json``, produced by ``oracle/ref_harness.py`` running
the real reference planner.

Representation (equivalent to the reference's objects, DESIGN.md "I-NTMCP"):
  * obs nodes are keyed by the agent's history: a node's parent edge is
    (parent node, action) and its observation; the root (t = 0) is node 0 and
    the ``None`` action of the initial observation is action index ``A``;
  * a particle of the level-1 tree carries the other agent's history as the
    id of its node in the level-0 tree.  That node is created when the
    particle is (``_tree.child``), but the ``add_child(action)`` registration
    that ``INTMCP.traverse`` (``intmcp.py:797-809``) performs happens only when
    the reference traverses: a node's registered actions, in registration
    order, are what ``obs_node.get_child_nodes()`` iterates (selection order,
    ties, the softmax of ``sample_action``);
  * ``INTMCP.traverse`` = register every edge on the path (memoised per node).
"""
import math

from oracle.rng import S_ACT_BASE, S_BELIEF, S_SELECT, Streams, StreamRandom

INF = float("inf")
S_BELIEF_NESTED = 3   # the level-0 planner's random.Random(config.seed) (intmcp.py:66)
S_BELIEF_MID = 5      # a middle planner's random.Random(config.seed): level l (1 <= l < the
                      # nesting level) draws on S_BELIEF_MID + l - 1 for l <= 3 (5, 6, 7) and
S_BELIEF_MID_HI = 16  # on S_BELIEF_MID_HI + l beyond (20, 21: clear of the action streams 8 + i;
                      # csrc/philox.h belief_mid_stream)
MAX_NESTING = 5       # (the engine builds nesting levels 0-5: include/intmcp.h INTMCP_MAX_TREES)


def belief_stream(level: int, nesting_level: int) -> int:
    """The stream of the level-`level` planner's random.Random(seed) in a
    nesting-`nesting_level` chain (construction order, intmcp.py:964-986)."""
    if level == 0:
        return S_BELIEF_NESTED
    if level == nesting_level:
        return S_BELIEF
    return S_BELIEF_MID + level - 1 if level <= 3 else S_BELIEF_MID_HI + level


class _Tree:
    """One planner's search tree (``ObsNode``/``ActionNode``, ``node.py``)."""

    def __init__(self, A):
        self.A = A
        self.NONE = A                     # the None action of the initial observation
        self.parent = [(-1, -1)]
        self.obs = [None]
        self.okey = [None]
        self.t = [0]
        self.visits = [0]
        self.absorbing = [False]
        self.order = [[]]                 # registered actions, registration order
        self.path_ok = [True]
        self.belief = [[]]
        self.children = {}                # (node, action, obs key) -> node
        self.stats = {}                   # (node, action) -> [visits, value, total, agg]

    def child(self, n, a, obs, okey):
        """The obs child (n, a, obs), created (visits 0) if missing."""
        k = (n, a, okey)
        c = self.children.get(k)
        if c is None:
            c = len(self.t)
            self.children[k] = c
            self.parent.append((n, a))
            self.obs.append(obs)
            self.okey.append(okey)
            self.t.append(self.t[n] + 1)
            self.visits.append(0)
            self.absorbing.append(False)
            self.order.append([])
            self.path_ok.append(False)
            self.belief.append([])
        return c

    def register(self, n, a):              # ObsNode.add_child (node.py:68-80)
        if a not in self.order[n]:
            self.order[n].append(a)
            self.stats[(n, a)] = [0, 0.0, 0.0, 0]

    def traverse(self, n):                 # intmcp.py:797-809
        while not self.path_ok[n]:
            p, a = self.parent[n]
            self.register(p, a)
            self.path_ok[n] = True
            n = p

    def expand(self, n):                   # intmcp.py:453-458 / 416-418
        for a in range(self.A):
            self.register(n, a)


class _Planner:
    """One INTMCP instance (``intmcp.py:22-111``)."""

    def __init__(self, model, agent_id, cfg, level, streams, rng_stream, nested=None,
                 search_probs=None):
        self.model = model
        # search_policies of this level (intmcp.py:956-971): agent id -> None
        # (RandomSearchPolicy: Discrete.sample()) or the action distribution of a
        # SearchPolicyWrapper(FixedDistributionPolicy), drawn as random.choices on
        # the agent's action stream (oracle/ref_harness.py wires it so)
        self.search_probs = dict(search_probs or {})
        self.agent_id = agent_id
        self.ego = model.possible_agents.index(agent_id)
        self.other_id = model.possible_agents[1 - self.ego]
        self.cfg = cfg
        self.level = level
        self.s = streams
        self.rng = StreamRandom(streams, rng_stream)     # self._rng = random.Random(seed)
        self.rng_stream = rng_stream
        self.nested = nested                             # other_agent_policies[j] (level 0)
        self.A = model.action_spaces[agent_id].n
        self.A_other = model.action_spaces[self.other_id].n
        if cfg.step_limit is not None:                   # intmcp.py:70-75
            self.step_limit = cfg.step_limit
        elif getattr(model, "spec", None) is not None:
            self.step_limit = model.spec.max_episode_steps
        else:
            self.step_limit = INF
        self.reset()

    def reset(self):                                     # intmcp.py:154-176
        kb = self.cfg.known_bounds
        self.mm_max, self.mm_min = (kb[1], kb[0]) if kb else (-INF, INF)
        self.tree = _Tree(self.A)
        self.cur = 0
        self.last_action = None
        self.search_depth = 0
        if self.nested is not None:
            self.nested.reset()

    # -------------------------------------------------------------- helpers
    def _mm_update(self, v):
        if v > self.mm_max:
            self.mm_max = v
        if v < self.mm_min:
            self.mm_min = v

    def _normalize(self, v):
        if self.mm_max > self.mm_min:
            return (v - self.mm_min) / (self.mm_max - self.mm_min)
        return v

    def _key(self, obs):
        return self.model.pack_obs(obs)

    def _belief_sample(self, n):                        # belief.py:55
        b = self.tree.belief[n]
        return b[self.s.randint(self.rng_stream, len(b))]

    # ------------------------------------------------------------ selection
    def _select(self, n):
        tr = self.tree
        sel = self.cfg.action_selection
        if sel == "ucb":                                 # intmcp.py:670-684
            if tr.visits[n] == 0:
                return self.s.randint(S_SELECT, self.A)
            log_n = math.log(tr.visits[n])
            best_v, best_a = -INF, 0
            for a in tr.order[n]:
                st = tr.stats[(n, a)]
                if st[0] == 0:
                    return a
                v = self._normalize(st[1]) + self.cfg.c * math.sqrt(log_n / st[0])
                if v > best_v:
                    best_v, best_a = v, a
            return best_a
        if sel == "uniform":                             # intmcp.py:686-701
            if tr.visits[n] == 0:
                return self.s.randint(S_SELECT, self.A)
            min_n, nxt = tr.visits[n] + 1, 0
            for a in tr.order[n]:
                if tr.stats[(n, a)][0] < min_n:
                    min_n, nxt = tr.stats[(n, a)][0], a
            return nxt
        raise NotImplementedError("INTMCP pucb (intmcp.py:645 reads self.action_space)")

    def final_action(self):                              # intmcp.py:718-732
        tr, n = self.tree, self.cur
        if len(tr.order[n]) == 0:
            return self.s.randint(S_SELECT, self.A)
        best, mx = [], -INF
        for a in tr.order[n]:
            v = tr.stats[(n, a)][1]
            if v == mx:
                best.append(a)
            elif v > mx:
                mx, best = v, [a]
        return best[self.s.randint(S_SELECT, len(best))]

    # ---------------------------------------------- other agent (level 1 only)
    def _policy_action(self, agent_id, probs):
        if probs is None:
            return self.s.randint(S_ACT_BASE + int(agent_id), self.model.action_spaces[agent_id].n)
        return StreamRandom(self.s, S_ACT_BASE + int(agent_id)).choices(range(len(probs)),
                                                                       weights=probs)[0]

    def sample_action(self, n, caller_probs=None):
        """``INTMCP.sample_action`` of the level-0 planner (``intmcp.py:763-791``)
        for the node of the other agent's history."""
        tr = self.tree
        tr.traverse(n)
        if tr.visits[n] == 0 or len(tr.order[n]) == 0:
            # the caller's search_policies[j].sample_action (intmcp.py:780):
            # model.action_spaces[j].sample(), or a fixed distribution's draw
            return self._policy_action(self.agent_id, caller_probs)
        sq = math.sqrt(tr.visits[n])
        probs = [math.exp(tr.stats[(n, a)][0] / sq) for a in tr.order[n]]
        total = sum(probs)
        probs = [p / total for p in probs]
        return StreamRandom(self.s, S_SELECT).choices(tr.order[n], weights=probs)[0]

    def _other_action(self, particle):                   # intmcp.py:602-615, 891-905
        if self.level == 0 or self.cfg.state_belief_only:
            return self.s.randint(self.rng_stream, self.A_other)   # self._rng.choice
        return self.nested.sample_action(particle[1], self.search_probs.get(self.other_id))

    def _joint(self, ego_action, other_action):
        ja = {}
        for i in self.model.possible_agents:
            ja[i] = ego_action if i == self.agent_id else other_action
        return ja

    def _extend(self, particle, ja, ts):
        """The next particle (state, [other's history node,] t + 1)."""
        if self.level == 0:
            return (ts.state, particle[-1] + 1)
        o = ts.observations[self.other_id]
        nid = self.nested.tree.child(particle[1], ja[self.other_id], o, self._key(o))
        return (ts.state, nid, particle[2] + 1)

    # ---------------------------------------------------------- reinvigorate
    def _reinvigorate(self, n, action, obs, target):     # intmcp.py:815-862
        tr = self.tree
        to_add = target - len(tr.belief[n])
        if to_add <= 0:
            return
        parent = tr.parent[n][0]
        okey = self._key(obs)
        limit = self.cfg.reinvigoration_sample_limit_factor * to_add   # belief.py:152-194
        count, attempts, rejected, samples = 0, 0, [], []
        while count < to_add and attempts < limit:
            attempts += 1
            hps = self._belief_sample(parent)
            if self.ego == 0:   # joint action built in possible_agents order
                ja = {"0": action}
                ja[self.other_id] = self._other_action(hps)
            else:
                oa = self._other_action(hps)
                ja = {self.other_id: oa, self.agent_id: action}
            ts = self.model.step(hps[0], ja)
            nxt = self._extend(hps, ja, ts)
            if self._key(ts.observations[self.agent_id]) == okey:
                samples.append(nxt)
                count += 1
            else:
                rejected.append(nxt)
        if count < to_add:
            samples.extend(rejected[:to_add - count])
        tr.belief[n].extend(samples)

    # ---------------------------------------------------------------- search
    def _simulate(self, hps, n, depth):                   # intmcp.py:444-517
        tr, cfg = self.tree, self.cfg
        if depth > cfg.depth_limit or tr.t[n] + depth > self.step_limit:
            return 0, depth
        if len(tr.order[n]) < self.A:
            tr.expand(n)
            return self._rollout(hps, depth), depth
        a = self._select(n)
        if self.ego == 0:
            ja = {"0": a}
            ja[self.other_id] = self._other_action(hps)
        else:
            oa = self._other_action(hps)
            ja = {self.other_id: oa, self.agent_id: a}
        ts = self.model.step(hps[0], ja)
        obs = ts.observations[self.agent_id]
        r = ts.rewards[self.agent_id]
        done = (ts.terminations[self.agent_id] or ts.truncations[self.agent_id] or ts.all_done)
        nxt = self._extend(hps, ja, ts)
        okey = self._key(obs)
        c = tr.children.get((n, a, okey))
        if c is not None:                                # intmcp.py:484-498
            tr.visits[c] += 1
        else:                                            # _add_obs_node(init_visits=1)
            c = tr.child(n, a, obs, okey)
            tr.visits[c] = 1
        tr.path_ok[c] = tr.path_ok[c] or tr.path_ok[n]
        tr.absorbing[c] = done
        tr.belief[c].append(nxt)
        max_depth = depth
        if not done:
            fut, max_depth = self._simulate(nxt, c, depth + 1)
            r += cfg.discount * fut
        st = tr.stats[(n, a)]                             # node.py:166-178
        st[0] += 1
        st[2] += r
        delta = r - st[1]
        st[1] += delta / st[0]
        st[3] += delta * (r - st[1])
        self._mm_update(st[1])
        return r, max_depth

    def _rollout(self, hps, depth):                       # intmcp.py:547-593
        cfg = self.cfg
        ret = 0
        k = 0
        state, t = hps[0], hps[-1]
        while depth <= cfg.depth_limit and t <= self.step_limit:
            ja = {i: self._policy_action(i, self.search_probs.get(i))
                  for i in self.model.possible_agents}
            ts = self.model.step(state, ja)
            ret += cfg.discount ** k * ts.rewards[self.agent_id]
            if (ts.terminations[self.agent_id] or ts.truncations[self.agent_id]
                    or ts.all_done):
                break
            state, t = ts.state, t + 1
            depth += 1
            k += 1
        return ret

    def _nested_sim(self, n, search_level, top_level):    # intmcp.py:410-442
        tr = self.tree
        tr.traverse(n)
        if len(tr.order[n]) == 0:
            tr.expand(n)
        size = len(tr.belief[n])
        if size == 0 or (top_level and size < self.cfg.extra_particles):
            p, a = tr.parent[n]
            self._reinvigorate(n, a, tr.obs[n], self.cfg.extra_particles)
        hps = self._belief_sample(n)
        if self.level > search_level:
            self.nested._nested_sim(hps[1], search_level, False)
        else:
            _, d = self._simulate(hps, n, 0)
            tr.visits[n] += 1
            self.search_depth = max(self.search_depth, d)

    # --------------------------------------------------------------- update
    def _nested_dist(self, dist):                        # intmcp.py:334-362
        """The other agent's history distribution: every history of every
        particle of the dist's nodes, weighted prob * count / size, in first-
        occurrence order."""
        out = {}
        for n, prob in dist.items():
            self.tree.traverse(n)
            b = self.tree.belief[n]
            counts = {}
            for p in b:
                counts[p[1]] = counts.get(p[1], 0) + 1
            for h, c in counts.items():
                out[h] = out.get(h, 0) + prob * (c / len(b))
        return out

    def _initial_nested_update(self, dist):              # intmcp.py:216-268
        tr, m = self.tree, self.model
        first = next(iter(dist))
        m.sample_agent_initial_state(self.agent_id, tr.obs[first])   # probe (draws)
        target = self.cfg.num_particles + self.cfg.extra_particles
        for n, prob in dist.items():
            tr.traverse(n)
            init_obs = tr.obs[n]
            parts = []
            while len(parts) < prob * target:
                state = m.sample_agent_initial_state(self.agent_id, init_obs)
                jo = m.sample_initial_obs(state)
                jo[self.agent_id] = init_obs
                if self.level == 0:
                    parts.append((state, 1))
                else:
                    o = jo[self.other_id]
                    nid = self.nested.tree.child(0, self.nested.tree.NONE, o, self._key(o))
                    parts.append((state, nid, 1))
            tr.belief[n] = parts
        if self.level > 0:
            self.nested._initial_nested_update(self._nested_dist(dist))

    def _nested_update(self, dist):                      # intmcp.py:270-300
        tr = self.tree
        target = self.cfg.num_particles + self.cfg.extra_particles
        for n, prob in dist.items():
            tr.traverse(n)
            if tr.absorbing[n]:
                continue
            p, a = tr.parent[n]
            self._reinvigorate(n, a, tr.obs[n], math.ceil(prob * target))
        if self.level > 0:
            self.nested._nested_update(self._nested_dist(dist))

    def update(self, action, obs):                       # intmcp.py:198-214
        tr = self.tree
        if tr.absorbing[self.cur]:
            return
        if tr.t[self.cur] == 0:
            self.cur = tr.child(0, tr.NONE, obs, self._key(obs))
            self._initial_nested_update({self.cur: 1.0})
        else:
            self.cur = tr.child(self.cur, action, obs, self._key(obs))
            self._nested_update({self.cur: 1.0})

    def get_action(self, num_sims):                       # intmcp.py:368-408
        tr = self.tree
        self.num_sims = 0
        if tr.absorbing[self.cur]:
            return 0
        for level in range(self.level + 1):
            for _ in range(num_sims):
                self._nested_sim(self.cur, level, True)
                self.num_sims += 1
        return self.final_action()


class OracleINTMCP:
    """``INTMCP.initialize(model, ego, config, nesting_level, None)`` with fixed
    simulation counts per level, nesting level 1 (a level-1 planner over the
    other agent's level-0 planner) or 0 (one level-0 planner: the other agent
    acts by its own ``self._rng.choice``, intmcp.py:750-753).  ``step(obs)``
    follows ``intmcp.py:115-140``.  The planners' ``random.Random(seed)`` are
    streams in construction order (the lowest level first, intmcp.py:964-986):
    S_BELIEF_NESTED, then S_BELIEF."""

    def __init__(self, model, agent_id, cfg, streams: Streams, nesting_level: int = 1,
                 search_probs=None):
        """search_probs: {level: {agent id: None or action probabilities}}
        (the search_policies of INTMCP.initialize; None: all random)."""
        assert cfg.num_sims is not None
        if not 0 <= nesting_level <= MAX_NESTING:
            raise NotImplementedError(f"nesting levels 0-{MAX_NESTING}")
        sp = search_probs or {}
        ids = model.possible_agents
        ego = ids.index(agent_id)
        # construction order of INTMCP.initialize (intmcp.py:964-986): the
        # lowest level first; level 0 draws on S_BELIEF_NESTED, the top planner
        # on S_BELIEF (nesting 0: the one planner is level 0), a middle level-l
        # planner on S_BELIEF_MID + l - 1 (belief_stream).  Level k models agent
        # ego if L - k is even.
        planners = []
        below = None
        for level in range(nesting_level + 1):
            who = ids[ego if (nesting_level - level) % 2 == 0 else 1 - ego]
            stream = belief_stream(level, nesting_level)
            below = _Planner(model, who, cfg, level, streams, stream, nested=below,
                             search_probs=sp.get(level))
            planners.append(below)
        self.planners = planners                       # by level
        self.top = planners[-1]
        self.nested = planners[-2] if nesting_level > 0 else None
        self.nesting_level = nesting_level
        self.cfg = cfg
        self.model = model
        self.stats = {}

    def reset(self):
        self.top.reset()

    def step(self, obs):
        top = self.top
        if top.tree.absorbing[top.cur]:
            self.stats = {"searched": False}
            return top.last_action
        self.stats = {"searched": True}
        top.update(top.last_action, obs)
        top.search_depth = 0
        if self.nested is not None:
            self.nested.search_depth = 0
        top.last_action = top.get_action(self.cfg.num_sims)
        return top.last_action

    # ---------------------------------------------------------- observation
    def history(self, tree, n):
        """The (action, obs key) path of node n (None action -> -1)."""
        out = []
        while n != 0:
            p, a = tree.parent[n]
            out.append((-1 if a == tree.NONE else a, tree.okey[n]))
            n = p
        return tuple(reversed(out))
