"""Oracle-side episode / single-search drivers producing the fixture record format.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).
"""
from oracle.envs import make_model
from oracle.episode import belief_digest, fhex, run_episode
from oracle.pomcp import OracleConfig, OraclePOMCP
from oracle.rng import Streams


def oracle_record(p: OraclePOMCP, searched, action):
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    st = p.stats
    parts = st["belief"]
    rec["belief_size"] = len(parts)
    rec["belief_digest"] = belief_digest(parts, p.model.pack_words)
    rec["num_sims"] = int(st.get("num_sims", 0))
    if rec["num_sims"] > 0:
        rec["search_depth"] = st["search_depth"]
        rec["root_visits"] = st["root_visits"]
        rec["child_visits"] = list(st["child_visits"])
        rec["child_values"] = [fhex(v) for v in st["child_values"]]
        rec["child_totals"] = [fhex(v) for v in st["child_totals"]]
        rec["min_value"] = fhex(st["min_value"])
        rec["max_value"] = fhex(st["max_value"])
    return rec


def make_oracle(cfg_kwargs, num_sims, ego="0", grid=None, tree=0, env="Driving-v1"):
    streams = Streams(cfg_kwargs.get("seed") or 0, tree)
    model = make_model(env, streams, grid=grid)
    cfg = OracleConfig(num_sims=num_sims, **cfg_kwargs)
    return OraclePOMCP(model, ego, cfg, streams)


def oracle_episode(cfg_kwargs, num_sims, env_seed, ego="0", grid=None, tree=0,
                   max_steps=50, env="Driving-v1"):
    p = make_oracle(cfg_kwargs, num_sims, ego=ego, grid=grid, tree=tree, env=env)
    records = []

    def step(obs):
        searched = not p.on_abs[p.root]
        a = p.step(obs)
        records.append(oracle_record(p, searched, a))
        return a

    trace = run_episode(step, env_seed, ego=ego, grid=grid, max_steps=max_steps, env=env)
    return trace, records


def oracle_first_step(cfg_kwargs, num_sims, tree, env_seed, rekey=None, env="Driving-v1"):
    """Record of the first planner step of an episode (synthetic root), optionally
    with the search streams re-keyed after the initial update (root-parallel)."""
    p = make_oracle(cfg_kwargs, num_sims, tree=tree, env=env)
    recs = []

    def step(obs):
        p.update(None, obs)
        if rekey is not None:
            p.s.rekey(rekey)
        a = p.get_action()
        p.stats["searched"] = True
        recs.append(oracle_record(p, True, a))
        return a

    run_episode(step, env_seed, max_steps=1, env=env)
    return recs[0], p


# ----------------------------------------------------------------- I-NTMCP
def make_oracle_intmcp(cfg_kwargs, num_sims, ego="0", tree=0, env="Driving-v1", nesting_level=1,
                       search_probs=None):
    from oracle.intmcp import OracleINTMCP
    streams = Streams(cfg_kwargs.get("seed") or 0, tree)
    model = make_model(env, streams)
    cfg = OracleConfig(num_sims=num_sims, **cfg_kwargs)
    return OracleINTMCP(model, ego, cfg, streams, nesting_level, search_probs)


def oracle_intmcp_record(p, searched, action):
    from oracle.intmcp_record import intmcp_record
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    top, nested = p.top, p.nested
    tr, n = top.tree, top.cur
    kids = [(a,) + tuple(tr.stats[(n, a)][:3]) for a in tr.order[n]]
    if nested is None:   # nesting level 0: no other-agent histories
        parts = [(q[1], p.model.pack_words(q[0]), ()) for q in tr.belief[n]]
        return intmcp_record(rec, top.num_sims, top.search_depth, tr.visits[n], kids,
                             top.mm_min, top.mm_max, parts, [])
    parts = [(q[2], p.model.pack_words(q[0]), p.history(nested.tree, q[1])) for q in tr.belief[n]]

    def node(pl, m):
        t = pl.tree
        nkids = [(a, t.stats[(m, a)][0], t.stats[(m, a)][1]) for a in t.order[m]]
        nparts = [(r[-1], p.model.pack_words(r[0])) for r in t.belief[m]]
        return (t.visits[m], nkids, nparts)

    nested_nodes, seen = [], []
    for q in tr.belief[n]:
        if q[1] in seen:
            continue
        seen.append(q[1])
        nested_nodes.append((p.history(nested.tree, q[1]), node(nested, q[1])))
    # the third tree on (nesting level >= 2): the histories carried by the
    # particles of the previous tree's recorded nodes, and those nodes
    chain = []
    upper, seen_up = nested, seen
    for lvl in range(p.nesting_level - 2, -1, -1):
        low = p.planners[lvl]
        seqs, nodes2, seen2 = [], [], []
        for m in seen_up:
            seq = []
            for r in upper.tree.belief[m]:
                seq.append(p.history(low.tree, r[1]))
                if r[1] not in seen2:
                    seen2.append(r[1])
                    nodes2.append((p.history(low.tree, r[1]), node(low, r[1])))
            seqs.append(seq)
        chain.append((seqs, nodes2))
        upper, seen_up = low, seen2
    return intmcp_record(rec, top.num_sims, top.search_depth, tr.visits[n], kids,
                         top.mm_min, top.mm_max, parts, nested_nodes,
                         nested2=chain[0] if chain else None, deeper=chain[1:])


def oracle_intmcp_episode(cfg_kwargs, num_sims, env_seed, ego="0", tree=0, max_steps=50,
                          env="Driving-v1", nesting_level=1, search_probs=None):
    p = make_oracle_intmcp(cfg_kwargs, num_sims, ego=ego, tree=tree, env=env,
                           nesting_level=nesting_level, search_probs=search_probs)
    p.reset()
    records = []

    def step(obs):
        searched = not p.top.tree.absorbing[p.top.cur]
        a = p.step(obs)
        records.append(oracle_intmcp_record(p, searched, a))
        return a

    trace = run_episode(step, env_seed, ego=ego, max_steps=max_steps, env=env)
    return trace, records
