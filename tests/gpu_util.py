"""Drive the product (GPU) planner in the oracle's record format."""
import hashlib
import struct

from oracle.episode import fhex, run_episode


def product_config(cfg_kwargs, num_sims):
    from posggym_baselines_amd.planning import KnownBounds, MCTSConfig
    kw = dict(cfg_kwargs)
    if kw.get("known_bounds") is not None:
        kw["known_bounds"] = KnownBounds(*kw["known_bounds"])
    return MCTSConfig(num_sims=num_sims, **kw)


def rows_digest(rows):
    """(size, sha1 over (t, v0, v1) u32 triples): oracle.episode.belief_digest of
    the packed particle words."""
    h = hashlib.sha1()
    for t, v0, v1 in rows:
        h.update(struct.pack("<III", int(t), int(v0), int(v1)))
    return len(rows), h.hexdigest()


def product_model(env):
    from posggym_baselines_amd.envs import DrivingModel, PursuitEvasionModel
    return PursuitEvasionModel() if env == "PursuitEvasion-v1" else DrivingModel()


def stats_record(st, A, searched, action, rows):
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    rec["belief_size"], rec["belief_digest"] = rows_digest(rows)
    rec["num_sims"] = int(st.num_sims)
    if rec["num_sims"] > 0:
        rec["search_depth"] = int(st.search_depth)
        rec["root_visits"] = int(st.root_visits)
        rec["child_visits"] = [int(x) for x in st.child_visits[:A]]
        rec["child_values"] = [fhex(x) for x in st.child_values[:A]]
        rec["child_totals"] = [fhex(x) for x in st.child_totals[:A]]
        rec["min_value"] = fhex(st.min_value)
        rec["max_value"] = fhex(st.max_value)
    return rec


def gpu_episode(cfg_kwargs, num_sims, env_seed, ego="0", max_steps=50, env="Driving-v1",
                planner_cls="POMCP", select_margin=None, exact=None):
    """select_margin: k_search's fast-selection margin (pomcp_debug_set_select_margin);
    exact: a list that receives each search's n_exact_selects."""
    from posggym_baselines_amd.planning import (IPOMCP, POMCP, RandomOtherAgentPolicy,
                                                RandomSearchPolicy)
    model = product_model(env)
    config = product_config(cfg_kwargs, num_sims)
    if planner_cls == "IPOMCP":
        others = {i: RandomOtherAgentPolicy(model, i) for i in model.possible_agents if i != ego}
        planner = IPOMCP(model, ego, config, others, RandomSearchPolicy(model, ego))
    else:
        planner = POMCP(model, ego, config, RandomSearchPolicy(model, ego))
    if select_margin is not None:
        from posggym_baselines_amd import _native as N
        assert N.load().pomcp_debug_set_select_margin(planner._engine._ctx,
                                                      float(select_margin)) == 0
    planner.reset()
    records = []
    A = model.action_spaces[ego].n

    def step(obs):
        searched = not planner.root.is_absorbing
        a = planner.step(obs)
        if not searched:
            records.append({"searched": False, "action": int(a)})
            return a
        rows = planner.root_belief()
        st = planner._engine.root_stats()[0]
        if exact is not None:
            exact.append(int(st.n_exact_selects))
        rec = stats_record(st, A, True, a, rows)
        rec["num_sims"] = int(planner.step_statistics["num_sims"])
        if rec["num_sims"] == 0:
            for k in ("search_depth", "root_visits", "child_visits", "child_values",
                      "child_totals", "min_value", "max_value"):
                rec.pop(k, None)
        records.append(rec)
        return a

    trace = run_episode(step, env_seed, ego=ego, max_steps=max_steps, env=env)
    planner.close()
    return trace, records


def _arena_usage(engine):
    import ctypes as C
    nb, nl = C.c_int32(), C.c_int32()
    assert engine._lib.pomcp_arena_usage(engine._ctx, C.byref(nb), C.byref(nl)) == 0
    return nb.value, nl.value


def batched_episodes(cfg_kwargs, num_sims, env_seeds, steps, capacities=None, usage=None,
                     inline_slots=None, probes=None, spin_limit=None, env="Driving-v1",
                     select_margin=None, counters=None, ego="0"):
    """Lockstep episodes of len(env_seeds) independent planners in ONE engine
    (tree b = planner b, env seed env_seeds[b]), `steps` real steps each.
    Returns per-tree record lists in the oracle format.  inline_slots: use only
    that many inline obs slots per action node (pomcp_debug_set_inline_slots);
    probes: a list that receives each search's overflow-map probes; spin_limit:
    k_search_lds's polls of a late step-tree hand-off (pomcp_debug_set_spin_limit);
    select_margin: k_search's fast-selection margin (pomcp_debug_set_select_margin);
    counters: a list that receives each search's summed (n_exact_selects,
    n_deferred, n_cutoff); ego: the planning agent (the other acts uniformly
    at random on the env's own stream, oracle/episode.py run_episode)."""
    import numpy as np
    from oracle.envs import make_model
    from oracle.episode import ENV_TREE_BASE
    from oracle.rng import S_ENV_POLICY_BASE, Streams
    from posggym_baselines_amd.planning import BatchedPOMCP
    model = product_model(env)
    A = model.action_spaces[ego].n
    B = len(env_seeds)
    bp = BatchedPOMCP(model, ego, product_config(cfg_kwargs, num_sims), B, num_sims,
                      searches=steps, reroot=True, capacities=capacities)
    if inline_slots is not None:
        from posggym_baselines_amd import _native as N
        assert N.load().pomcp_debug_set_inline_slots(bp.engine._ctx, int(inline_slots)) == 0
    if spin_limit is not None:
        from posggym_baselines_amd import _native as N
        assert N.load().pomcp_debug_set_spin_limit(bp.engine._ctx, int(spin_limit)) == 0
    if select_margin is not None:
        from posggym_baselines_amd import _native as N
        assert N.load().pomcp_debug_set_select_margin(bp.engine._ctx, float(select_margin)) == 0
    envs = []
    for s in env_seeds:
        es = Streams(s, ENV_TREE_BASE)
        e = make_model(env, es)
        st = e.sample_initial_state()
        envs.append([es, e, st, e.sample_initial_obs(st)])
    records = [[] for _ in range(B)]
    last = np.full(B, -1, dtype=np.int32)
    for t in range(steps):
        keys = np.array([e[1].pack_obs(e[3][ego]) for e in envs], dtype=np.uint64)
        if usage is not None:
            usage.append(("before_update", _arena_usage(bp.engine)))
        bp.engine.update(last, keys)
        if usage is not None:
            usage.append(("after_update", _arena_usage(bp.engine)))
        actions = bp.search()
        stats = bp.engine.root_stats()
        if probes is not None:
            probes.append(sum(int(st.n_probes) for st in stats))
        if counters is not None:
            counters.append((sum(int(st.n_exact_selects) for st in stats),
                             sum(int(st.n_deferred) for st in stats),
                             sum(int(st.n_cutoff) for st in stats)))
        for b in range(B):
            records[b].append(stats_record(stats[b], A, True, actions[b], bp.engine.root_belief(b)))
            es, e, st, obs = envs[b]
            acts = {i: int(actions[b]) if i == ego else
                    es.randint(S_ENV_POLICY_BASE + int(i), e.action_spaces[i].n)
                    for i in e.possible_agents}
            ts = e.step(st, acts)
            envs[b][2], envs[b][3] = ts.state, ts.observations
        last = actions.astype(np.int32)
    bp.close()
    return records


def intmcp_state_record(eng, pair, searched, action):
    """The oracle's I-NTMCP step record (oracle/run.py oracle_intmcp_record)
    rebuilt from the device state of one planner pair."""
    from oracle.intmcp_record import intmcp_record
    from posggym_baselines_amd.planning.intmcp import node_order
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    st = eng.root_stats()[pair]
    A = eng.A
    n1 = eng.nodes(pair, 1)
    s1 = eng.stats(pair, 1)
    ent, sparts = eng.support(pair)
    kids = [(int(st.child_action[i]), int(st.child_visits[i]), st.child_values[i],
             st.child_totals[i]) for i in range(st.num_children)]
    if eng.nesting_level == 0:   # the planner's tree (tree 1), its root belief = support entry 0
        t_root = int(n1[int(ent[0]["node"])]["t"])
        parts = [(t_root, (int(q[0]), int(q[1])), ()) for q in eng.root_belief(pair)]
        return intmcp_record(rec, int(st.num_sims), int(st.search_depth), int(st.root_visits),
                             kids, st.min_value, st.max_value, parts, [])
    rows = eng.root_belief(pair)

    def history(nodes, n):
        out = []
        while n != 0:
            a = int(nodes[n]["info"]) & 7
            out.append((-1 if a == A else a, int(nodes[n]["okey"])))
            n = int(nodes[n]["parent"])
        return tuple(reversed(out))

    def node(nodes, stats, n, ent_, parts_):
        """(visits, registered children, particles) of node n, its particles
        from its materialised belief entry"""
        nd = nodes[n]
        nk = [(a, int(stats[int(nd["stats"]) + a]["visits"]),
               float(stats[int(nd["stats"]) + a]["value"]))
              for a in node_order(int(nd["info"])) if a < A]
        hit = [e for e in ent_ if int(e["node"]) == n]
        rows_ = []
        if hit:
            e = hit[0]
            rows_ = parts_[int(e["off"]):int(e["off"]) + int(e["size"])]
        return (int(nd["visits"]), nk, [(int(nd["t"]), (int(q[0]), int(q[1]))) for q in rows_]), rows_

    L = eng.nesting_level

    def table(k):   # tree k's materialised beliefs: a middle tree's, else the level-0 support
        return eng.mid_support(pair, k) if 1 <= k <= L - 1 else (ent, sparts)

    ent1, parts1 = table(1)
    # the root's t: every root particle's other-agent history has that length
    t_root = int(n1[int(rows[0][2])]["t"]) if len(rows) else 0
    parts = [(t_root, (int(r[0]), int(r[1])), history(n1, int(r[2]))) for r in rows]
    nested, seen, mrows = [], [], []
    for r in rows:
        m = int(r[2])
        if m in seen:
            continue
        seen.append(m)
        nd, rows_ = node(n1, s1, m, ent1, parts1)
        nested.append((history(n1, m), nd))
        mrows.append(rows_)
    # the third tree on (nesting level >= 2): the histories carried by the
    # particles of the previous tree's recorded nodes, and those nodes
    chain, up_rows = [], mrows
    for k in range(2, L + 1):
        nk_, sk_ = eng.nodes(pair, k), eng.stats(pair, k)
        ek, pk = table(k)
        seqs, nodes2, seen2, rows2 = [], [], [], []
        for rows_ in up_rows:
            seq = []
            for q in rows_:
                h2 = int(q[2])
                seq.append(history(nk_, h2))
                if h2 not in seen2:
                    seen2.append(h2)
                    nd, r2 = node(nk_, sk_, h2, ek, pk)
                    nodes2.append((history(nk_, h2), nd))
                    rows2.append(r2)
            seqs.append(seq)
        chain.append((seqs, nodes2))
        up_rows = rows2
    return intmcp_record(rec, int(st.num_sims), int(st.search_depth), int(st.root_visits), kids,
                         st.min_value, st.max_value, parts, nested,
                         nested2=chain[0] if chain else None, deeper=chain[1:])


def _softmax_debug(ctx, slack):
    """Widen the I-NTMCP fast softmax bound (intmcp_debug_set_softmax_slack) and
    start counting exact-path draws."""
    from posggym_baselines_amd import _native as N
    assert N.load().intmcp_debug_set_softmax_slack(ctx, float(slack)) == 0


def _exact_draws(ctx):
    import ctypes as C
    from posggym_baselines_amd import _native as N
    n = C.c_uint64()
    assert N.load().intmcp_debug_exact_draws(ctx, C.byref(n)) == 0
    return int(n.value)


def intmcp_search_policies(model, search_probs):
    """{level: {agent: probs}} -> the product's INTMCP.initialize search_policies
    (SearchPolicyWrapper(FixedDistributionPolicy) / RandomSearchPolicy)."""
    if search_probs is None:
        return None
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
    from posggym_baselines_amd.planning.search_policy import (RandomSearchPolicy,
                                                               SearchPolicyWrapper)
    return {lv: {i: (RandomSearchPolicy(model, i) if pols.get(i) is None else
                     SearchPolicyWrapper(FixedDistributionPolicy(model, i, "search", pols[i])))
                 for i in model.possible_agents}
            for lv, pols in search_probs.items()}


def gpu_intmcp_episode(cfg_kwargs, num_sims, env_seed, ego="0", max_steps=50, env="Driving-v1",
                       softmax_slack=None, exact=None, nesting_level=1, search_probs=None):
    """softmax_slack: the fast softmax bound's widening (None: the product's);
    the exact-path draws of the episode are appended to `exact` (a list);
    search_probs: {level: {agent: probs}} fixed-distribution search policies."""
    from posggym_baselines_amd.planning import INTMCP
    model = product_model(env)
    planner = INTMCP.initialize(model, ego, product_config(cfg_kwargs, num_sims), nesting_level,
                                intmcp_search_policies(model, search_probs))
    if softmax_slack is not None:
        _softmax_debug(planner._engine._ctx, softmax_slack)
    planner.reset()
    records = []

    def step(obs):
        searched = not planner.root.is_absorbing
        a = planner.step(obs)
        records.append(intmcp_state_record(planner._engine, 0, searched, a))
        return a

    trace = run_episode(step, env_seed, ego=ego, max_steps=max_steps, env=env)
    if exact is not None:
        exact.append(_exact_draws(planner._engine._ctx))
    planner.close()
    return trace, records


def batched_intmcp_episodes(cfg_kwargs, num_sims, env_seeds, steps, env="Driving-v1", ego="0",
                            softmax_slack=None, exact=None, nesting_level=1):
    """Lockstep I-NTMCP episodes of len(env_seeds) planner pairs in ONE engine
    (pair b = tree key b, env seed env_seeds[b]), at most `steps` real steps;
    a pair whose episode ended is skipped (INTMCP_SKIP).  Per-pair record lists
    in the oracle format (oracle/run.py oracle_intmcp_episode)."""
    import numpy as np
    from oracle.envs import make_model
    from oracle.episode import ENV_TREE_BASE
    from oracle.rng import S_ENV_POLICY_BASE, Streams
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.planning import BatchedINTMCP
    model = product_model(env)
    B = len(env_seeds)
    bp = BatchedINTMCP(model, ego, product_config(cfg_kwargs, num_sims), B, num_sims,
                       searches=steps, nesting_level=nesting_level)
    if softmax_slack is not None:
        _softmax_debug(bp.engine._ctx, softmax_slack)
    envs = []
    for s in env_seeds:
        es = Streams(s, ENV_TREE_BASE)
        e = make_model(env, es)
        st = e.sample_initial_state()
        envs.append([es, e, st, e.sample_initial_obs(st), False])
    records = [[] for _ in range(B)]
    last = np.full(B, -1, dtype=np.int32)
    absorbing = np.zeros(B, dtype=bool)
    for t in range(steps):
        acts_in = last.copy()
        keys = np.zeros(B, dtype=np.uint64)
        searched = ~absorbing
        for b in range(B):
            if envs[b][4] or absorbing[b]:
                acts_in[b] = N.INTMCP_SKIP
            else:
                keys[b] = envs[b][1].pack_obs(envs[b][3][ego])
        absorbing = bp.engine.update(acts_in, keys)
        actions = bp.search()
        for b in range(B):
            if envs[b][4]:
                continue
            a = int(actions[b]) if searched[b] else int(last[b])
            records[b].append(intmcp_state_record(bp.engine, b, bool(searched[b]), a))
            es, e, st, obs, _ = envs[b]
            ja = {}
            for i in e.possible_agents:
                ja[i] = a if i == ego else es.randint(S_ENV_POLICY_BASE + int(i),
                                                      e.action_spaces[i].n)
            ts = e.step(st, ja)
            envs[b][2], envs[b][3] = ts.state, ts.observations
            envs[b][4] = bool(ts.all_done)
            last[b] = a
    if exact is not None:
        exact.append(_exact_draws(bp.engine._ctx))
    bp.close()
    return records
