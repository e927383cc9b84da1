"""Drive the REAL reference planner (container-only) to produce golden fixtures.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).  Never runs on the GPU box:
``/root/reference`` does not exist there.  Contains no reference source: it
only creates empty stand-in modules for the absent third-party packages
(SURVEY Appendix A), then imports ``posggym_baselines.planning`` from
``/root/reference`` read-only (``sys.dont_write_bytecode``; the
``posggym_baselines.ppo`` package is stubbed so its ``results/`` mkdir side
effect never runs).

Injection:
  * ``posggym_baselines.planning.mcts.random`` -> a module object whose
    ``Random(seed)`` is the BELIEF stream and whose ``choice``/``choices`` are
    the SELECT stream of the planner's ``Streams``;
  * ``mcts.time`` -> a fake clock; the planner instance's ``_simulate`` is
    wrapped so that after ``num_sims`` depth-0 calls the clock jumps past
    ``search_time_limit`` and ``get_action``'s while loop (``mcts.py:285``)
    exits after exactly ``num_sims`` simulations;
  * the model is the build's restatement (``oracle.envs``: Driving-v1 or
    PursuitEvasion-v1) whose action spaces and RNG draw from the same ``Streams``.
"""
import os
import sys
import types

REF_ROOT = "/root/reference"


def reference_available() -> bool:
    return os.path.isdir(os.path.join(REF_ROOT, "posggym_baselines", "planning"))


_P = None


def import_reference():
    global _P
    if _P is not None:
        return _P
    sys.dont_write_bytecode = True

    def mod(name, **kw):
        m = types.ModuleType(name)
        m.__dict__.update(kw)
        sys.modules[name] = m
        return m

    class _Any:
        pass


    from oracle.driving import Discrete
    spaces = mod("gymnasium.spaces", Discrete=Discrete)
    mod("gymnasium").spaces = spaces
    pg = mod("posggym")
    pg.__path__ = []
    pg.model = mod("posggym.model", POSGModel=_Any, ObsType=object, ActType=object,
                   StateType=object)
    pg.agents = mod("posggym.agents", make=None, Policy=_Any)
    pg.agents.__path__ = []
    mod("posggym.agents.policy", Policy=_Any, PolicyState=dict)
    mod("posggym.agents.wrappers", AgentEnvWrapper=_Any)
    mod("posggym.agents.utils").__path__ = []
    mod("posggym.agents.utils.processors", Processor=_Any)
    mod("posggym.agents.utils.action_distributions", DiscreteActionDistribution=_Any)
    pg.utils = mod("posggym.utils")
    pg.utils.__path__ = []
    from oracle.history import AgentHistory, JointHistory
    mod("posggym.utils.history", JointHistory=JointHistory, AgentHistory=AgentHistory)
    mod("posggym_baselines.ppo").__path__ = [os.path.join(REF_ROOT, "posggym_baselines", "ppo")]
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import posggym_baselines.planning as P  # noqa: E402
    _P = P
    return P


class _FakeClock:
    def __init__(self):
        self.now = 0.0

    def time(self):
        return self.now


def make_reference_pomcp(model, agent_id, cfg_kwargs, num_sims, streams, planner_cls="POMCP"):
    """Build a reference ``POMCP`` (or ``IPOMCP`` with random other agents,
    ``ipomcp.py:11-38``) wired to ``streams`` and a fixed sim count."""
    P = import_reference()
    import posggym_baselines.planning.belief as B
    import posggym_baselines.planning.mcts as mcts_mod
    from oracle.rng import S_BELIEF, S_SELECT, StreamRandom

    select = StreamRandom(streams, S_SELECT)
    belief_rng = StreamRandom(streams, S_BELIEF)
    rnd = types.ModuleType("random_shim")
    rnd.Random = lambda seed=None: belief_rng
    rnd.choice = select.choice
    rnd.choices = select.choices
    rnd.random = select.random
    mcts_mod.random = rnd
    B.random = rnd
    clock = _FakeClock()
    mcts_mod.time = clock

    from posggym_baselines.planning.utils import KnownBounds
    kw = dict(cfg_kwargs)
    if kw.get("known_bounds") is not None:
        kw["known_bounds"] = KnownBounds(*kw["known_bounds"])
    config = P.MCTSConfig(**kw)
    if planner_cls == "IPOMCP":
        others = {i: P.RandomOtherAgentPolicy(model, i)
                  for i in model.possible_agents if i != agent_id}
        planner = P.IPOMCP(model, agent_id, config, others,
                           search_policy=P.RandomSearchPolicy(model, agent_id))
    else:
        planner = P.POMCP(model, agent_id, config,
                          search_policy=P.RandomSearchPolicy(model, agent_id))
    inner = planner._simulate
    count = [0]

    def simulate(hps, obs_node, depth, search_policy):
        if depth == 0:
            streams.align_sim()   # a simulation starts its step streams at a block (oracle/rng.py)
            count[0] += 1
            if count[0] >= num_sims:
                clock.now += 1e9
                count[0] = 0
        return inner(hps, obs_node, depth, search_policy)

    planner._simulate = simulate
    if num_sims <= 0:
        raise ValueError("num_sims must be positive")
    return planner


def reference_record(planner, searched, action):
    from oracle.episode import belief_digest, fhex
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    root = planner.root
    parts = [(p.state, p.t) for p in root.belief.particles]
    st = planner.step_statistics
    rec["belief_size"] = len(parts)
    rec["belief_digest"] = belief_digest(parts, planner.model.pack_words)
    rec["num_sims"] = int(st["num_sims"])
    if rec["num_sims"] > 0:
        kids = root.get_child_nodes()
        rec["search_depth"] = int(st["search_depth"])
        rec["root_visits"] = int(root.visits)
        rec["child_visits"] = [int(c.visits) for c in kids]
        rec["child_values"] = [fhex(c.value) for c in kids]
        rec["child_totals"] = [fhex(c.total_value) for c in kids]
        rec["min_value"] = fhex(st["min_value"])
        rec["max_value"] = fhex(st["max_value"])
    return rec


def reference_episode(cfg_kwargs, num_sims, env_seed, ego="0", grid=None,
                      tree=0, max_steps=50, env="Driving-v1", planner_cls="POMCP"):
    """One full episode with the real reference POMCP. Returns (trace, records)."""
    from oracle.envs import make_model
    from oracle.episode import run_episode
    from oracle.rng import Streams

    streams = Streams(cfg_kwargs.get("seed") or 0, tree)
    model = make_model(env, streams, grid=grid)
    planner = make_reference_pomcp(model, ego, cfg_kwargs, num_sims, streams, planner_cls)
    planner.reset()
    records = []

    def step(obs):
        searched = not planner.root.is_absorbing
        a = planner.step(obs)
        records.append(reference_record(planner, searched, a))
        return a

    trace = run_episode(step, env_seed, ego=ego, grid=grid, max_steps=max_steps, env=env)
    planner.close()
    return trace, records


# ----------------------------------------------------------------- I-NTMCP
def make_reference_intmcp(model, agent_id, cfg_kwargs, num_sims, streams, nesting_level=1,
                          search_probs=None):
    """``INTMCP.initialize(model, agent_id, config, nesting_level, search_policies)``
    wired to ``streams`` with ``num_sims`` simulations per nesting level
    (intmcp.py:385-399: the wrapped top-level ``_nested_sim`` jumps the fake
    clock after num_sims calls).  ``random.Random(seed)`` is called once per
    planner, the lowest level first (intmcp.py:964-986): first call ->
    S_BELIEF_NESTED, second -> S_BELIEF (nesting level 0: the one planner's is
    S_BELIEF_NESTED).  search_probs: None (``search_policies=None``: random at
    every level) or {level: {agent: None | probs}} -> ``RandomSearchPolicy`` /
    ``SearchPolicyWrapper(FixedDistributionPolicy)`` drawing on the agent's
    action stream (``S_ACT_BASE + agent``, the stream ``Discrete.sample()`` uses)."""
    P = import_reference()
    import posggym_baselines.planning.intmcp as im
    import posggym_baselines.planning.belief as B
    from oracle.intmcp import belief_stream
    from oracle.rng import S_SELECT, StreamRandom

    select = StreamRandom(streams, S_SELECT)
    # lowest level first: level 0, the middle levels, the top (belief_stream)
    order = [StreamRandom(streams, belief_stream(lv, nesting_level))
             for lv in range(nesting_level + 1)]
    made = []

    def new_random(seed=None):
        r = order[len(made)]
        made.append(r)
        return r

    rnd = types.ModuleType("random_shim")
    rnd.Random = new_random
    rnd.choice = select.choice
    rnd.choices = select.choices
    rnd.random = select.random
    im.random = rnd
    B.random = rnd
    clock = _FakeClock()
    im.time = clock
    from posggym_baselines.planning.utils import KnownBounds
    kw = dict(cfg_kwargs)
    if kw.get("known_bounds") is not None:
        kw["known_bounds"] = KnownBounds(*kw["known_bounds"])
    config = P.MCTSConfig(**kw)
    search_policies = None
    if search_probs is not None:
        import posggym_baselines.planning.search_policy as sp_mod
        from oracle.rng import S_ACT_BASE
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "posggym-baselines_amd"))
        from posggym_baselines_amd.planning.policies import FixedDistributionPolicy

        def policy(i, probs):
            if probs is None:
                return P.RandomSearchPolicy(model, i)
            return sp_mod.SearchPolicyWrapper(FixedDistributionPolicy(
                model, i, "search", probs, StreamRandom(streams, S_ACT_BASE + int(i))))

        search_policies = {lv: {i: policy(i, search_probs.get(lv, {}).get(i))
                                for i in model.possible_agents}
                           for lv in range(nesting_level + 1)}
    planner = P.INTMCP.initialize(model, agent_id, config, nesting_level=nesting_level,
                                  search_policies=search_policies)
    assert len(made) == nesting_level + 1
    inner = planner._nested_sim
    count = [0]

    def nested_sim(history, search_level, top_level=False):
        r = inner(history, search_level, top_level)
        if top_level:
            count[0] += 1
            if count[0] >= num_sims:
                clock.now += 1e9
                count[0] = 0
        return r

    planner._nested_sim = nested_sim
    return planner


def _hist_key(model, agent_hist):
    return tuple((-1 if a is None else int(a), model.pack_obs(o)) for a, o in agent_hist)


def _walk(root, agent_hist):
    node = root
    for a, o in agent_hist:
        an = node.children.get(a)
        if an is None:
            return None
        node = an.children.get(o)
        if node is None:
            return None
    return node


def reference_intmcp_record(planner, searched, action):
    from oracle.intmcp_record import intmcp_record
    model = planner.model
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    root = _walk(planner.root, planner.history)
    other = [i for i in model.possible_agents if i != planner.agent_id][0]
    kids = [(int(c.action), c.visits, c.value, c.total_value) for c in root.get_child_nodes()]
    st = planner.step_statistics
    if planner.nesting_level == 0:   # no other-agent histories (intmcp_record of the oracle)
        parts = [(p.t, model.pack_words(p.state), ()) for p in root.belief.particles]
        return intmcp_record(rec, int(st["num_sims"]), int(st["search_depth"]), root.visits, kids,
                             st["min_value"], st["max_value"], parts, [])
    nested = planner.other_agent_policies[other]
    parts = [(p.t, model.pack_words(p.state), _hist_key(model, p.history.get_agent_history(other)))
             for p in root.belief.particles]
    def node(n):
        nparts = [(q.t, model.pack_words(q.state)) for q in n.belief.particles]
        nkids = [(int(c.action), c.visits, c.value) for c in n.get_child_nodes()]
        return (n.visits, nkids, nparts)

    nested_nodes, seen, seen_nodes = [], [], []
    for p in root.belief.particles:
        h = p.history.get_agent_history(other)
        if h in seen:
            continue
        seen.append(h)
        n = _walk(nested.root, h)
        seen_nodes.append(n)
        nested_nodes.append((_hist_key(model, h), None if n is None else node(n)))
    # the third tree on (nesting level >= 2): the histories carried by the
    # particles of the previous tree's recorded nodes, and those nodes
    chain = []
    upper, up_agent, up_nodes = nested, other, seen_nodes
    for _ in range(planner.nesting_level - 1):
        low_agent = planner.agent_id if up_agent == other else other
        low = upper.other_agent_policies[low_agent]
        seqs, nodes2, seen2, seen2_nodes = [], [], [], []
        for n in up_nodes:
            seq = []
            for q in ([] if n is None else n.belief.particles):
                h2 = q.history.get_agent_history(low_agent)
                seq.append(_hist_key(model, h2))
                if h2 not in seen2:
                    seen2.append(h2)
                    n2 = _walk(low.root, h2)
                    seen2_nodes.append(n2)
                    nodes2.append((_hist_key(model, h2), None if n2 is None else node(n2)))
            seqs.append(seq)
        chain.append((seqs, nodes2))
        upper, up_agent, up_nodes = low, low_agent, seen2_nodes
    st = planner.step_statistics
    return intmcp_record(rec, int(st["num_sims"]), int(st["search_depth"]), root.visits, kids,
                         st["min_value"], st["max_value"], parts, nested_nodes,
                         nested2=chain[0] if chain else None, deeper=chain[1:])


def reference_intmcp_episode(cfg_kwargs, num_sims, env_seed, ego="0", tree=0, max_steps=50,
                             env="Driving-v1", nesting_level=1, search_probs=None):
    from oracle.envs import make_model
    from oracle.episode import run_episode
    from oracle.rng import Streams

    streams = Streams(cfg_kwargs.get("seed") or 0, tree)
    model = make_model(env, streams)
    planner = make_reference_intmcp(model, ego, cfg_kwargs, num_sims, streams, nesting_level,
                                    search_probs)
    planner.reset()
    records = []

    def step(obs):
        root = _walk(planner.root, planner.history)
        searched = not root.is_absorbing
        a = planner.step(obs)
        records.append(reference_intmcp_record(planner, searched, a))
        return a

    trace = run_episode(step, env_seed, ego=ego, max_steps=max_steps, env=env)
    planner.close()
    return trace, records


# ----------------------------------------------------------------- POTMMCP
def potmmcp_policies(model, agent_id, spec, streams=None):
    """The non-neural policy set of a POTMMCP case: ``spec`` = {"ego": {id: probs},
    "other": {id: probs}, "meta": {other id: {ego id: weight}}}.  Returns (ego
    policies, other-agent policies, meta_policy); a policy samples its actions
    on its agent's action stream (8 + agent index) when ``streams`` is given."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "posggym-baselines_amd"))
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
    from oracle.rng import S_ACT_BASE, StreamRandom
    other = [i for i in model.possible_agents if i != agent_id][0]

    def make(i, pid, probs):
        rng = StreamRandom(streams, S_ACT_BASE + int(i)) if streams is not None else None
        return FixedDistributionPolicy(model, i, pid, probs, rng)

    ego_pols = {k: make(agent_id, k, v) for k, v in spec["ego"].items()}
    oth_pols = {k: make(other, k, v) for k, v in spec["other"].items()}
    meta = {k: dict(v) for k, v in spec["meta"].items()}
    return ego_pols, oth_pols, meta


def make_reference_potmmcp(model, agent_id, cfg_kwargs, num_sims, streams, spec):
    """The reference ``POTMMCP`` (potmmcp.py:18-301) with a ``POTMMCPMetaPolicy``
    over fixed-distribution ego policies and an ``OtherAgentMixturePolicy`` over
    fixed-distribution other-agent policies, wired to ``streams``: mcts / potmmcp
    ``random`` -> SELECT stream (``sample_policy``'s ``random.choices`` included),
    other_policy ``random`` -> MIXTURE stream, planner Random -> BELIEF stream."""
    P = import_reference()
    import posggym_baselines.planning.belief as B
    import posggym_baselines.planning.mcts as mcts_mod
    import posggym_baselines.planning.other_policy as op_mod
    import posggym_baselines.planning.potmmcp as pt_mod
    from oracle.rng import S_BELIEF, S_MIXTURE, S_SELECT, StreamRandom

    select = StreamRandom(streams, S_SELECT)
    belief_rng = StreamRandom(streams, S_BELIEF)
    rnd = types.ModuleType("random_shim")
    rnd.Random = lambda seed=None: belief_rng
    rnd.choice = select.choice
    rnd.choices = select.choices
    rnd.random = select.random
    mcts_mod.random = rnd
    pt_mod.random = rnd
    B.random = rnd
    mix = types.ModuleType("random_shim_mixture")
    mix.choice = StreamRandom(streams, S_MIXTURE).choice
    op_mod.random = mix
    clock = _FakeClock()
    mcts_mod.time = clock
    pt_mod.time = clock
    from posggym_baselines.planning.utils import KnownBounds
    kw = dict(cfg_kwargs)
    if kw.get("known_bounds") is not None:
        kw["known_bounds"] = KnownBounds(*kw["known_bounds"])
    config = P.MCTSConfig(**kw)
    ego_pols, oth_pols, meta = potmmcp_policies(model, agent_id, spec, streams)
    other = [i for i in model.possible_agents if i != agent_id][0]
    others = {other: P.OtherAgentMixturePolicy(model, other, oth_pols)}
    search = P.POTMMCPMetaPolicy(model, agent_id, ego_pols, meta)
    planner = P.POTMMCP(model, agent_id, config, others, search)
    inner = planner._simulate
    count = [0]

    def simulate(hps, obs_node, depth, search_policy):
        if depth == 0:
            streams.align_sim()   # a simulation starts its step streams at a block (oracle/rng.py)
            count[0] += 1
            if count[0] >= num_sims:
                clock.now += 1e9
                count[0] = 0
        return inner(hps, obs_node, depth, search_policy)

    planner._simulate = simulate
    return planner


def potmmcp_belief_digest(particles, other_ids, pack_words):
    """sha1 over (t, v0, v1, other-agent policy index) u32 quadruples, insertion order."""
    import hashlib
    import struct
    h = hashlib.sha1()
    for st, t, pid in particles:
        v0, v1 = pack_words(st)
        h.update(struct.pack("<IIII", t, v0, v1, other_ids.index(pid)))
    return h.hexdigest()


def reference_potmmcp_record(planner, searched, action):
    from oracle.episode import fhex
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    root = planner.root
    other = [i for i in planner.model.possible_agents if i != planner.agent_id][0]
    oth_ids = list(planner.other_agent_policies[other].policies)
    parts = [(p.state, p.t, p.policy_state[other]["policy_id"]) for p in root.belief.particles]
    st = planner.step_statistics
    rec["belief_size"] = len(parts)
    rec["belief_digest"] = potmmcp_belief_digest(parts, oth_ids, planner.model.pack_words)
    rec["num_sims"] = int(st["num_sims"])
    rec["prior"] = [fhex(root.action_probs[a]) for a in range(len(root.action_probs))]
    if rec["num_sims"] > 0:
        kids = root.get_child_nodes()
        rec["search_depth"] = int(st["search_depth"])
        rec["root_visits"] = int(root.visits)
        rec["child_visits"] = [int(c.visits) for c in kids]
        rec["child_values"] = [fhex(c.value) for c in kids]
        rec["child_totals"] = [fhex(c.total_value) for c in kids]
        rec["min_value"] = fhex(st["min_value"])
        rec["max_value"] = fhex(st["max_value"])
    return rec


def reference_potmmcp_episode(cfg_kwargs, num_sims, env_seed, spec, ego="0", tree=0,
                              max_steps=50, env="Driving-v1"):
    """One full episode with the real reference POTMMCP. Returns (trace, records)."""
    from oracle.envs import make_model
    from oracle.episode import run_episode
    from oracle.rng import Streams

    streams = Streams(cfg_kwargs.get("seed") or 0, tree)
    model = make_model(env, streams)
    planner = make_reference_potmmcp(model, ego, cfg_kwargs, num_sims, streams, spec)
    planner.reset()
    records = []

    def step(obs):
        searched = not planner.root.is_absorbing
        a = planner.step(obs)
        records.append(reference_potmmcp_record(planner, searched, a))
        return a

    trace = run_episode(step, env_seed, ego=ego, max_steps=max_steps, env=env)
    planner.close()
    return trace, records


# ------------------------------------------- MCTS / IPOMCP / POMCP, any policies
def make_reference_mcts(model, agent_id, cfg_kwargs, num_sims, streams, spec,
                        planner_cls="IPOMCP"):
    """The reference base planner (``MCTS`` / ``IPOMCP`` / ``POMCP``,
    mcts.py:22-739, ipomcp.py:11-38, pomcp.py:9-35) with fixed-distribution
    policies, wired to ``streams`` like ``make_reference_potmmcp``:
      spec["search"]: None (``RandomSearchPolicy``) or the ego's action
        probabilities (``SearchPolicyWrapper`` of a ``FixedDistributionPolicy``,
        search_policy.py:188-224: prior of every node, rollouts);
      spec["other"]: {"kind": "random"} (``RandomOtherAgentPolicy``), {"kind":
        "fixed", "probs": [...]} (a stateless ``FixedDistributionPolicy``, used
        with state_belief_only=True) or {"kind": "mixture", "policies": {id:
        probs}} (``OtherAgentMixturePolicy``, state_belief_only=False)."""
    P = import_reference()
    import posggym_baselines.planning.belief as B
    import posggym_baselines.planning.mcts as mcts_mod
    import posggym_baselines.planning.other_policy as op_mod
    import posggym_baselines.planning.search_policy as sp_mod
    from oracle.rng import S_ACT_BASE, S_BELIEF, S_MIXTURE, S_SELECT, StreamRandom
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "posggym-baselines_amd"))
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy

    select = StreamRandom(streams, S_SELECT)
    belief_rng = StreamRandom(streams, S_BELIEF)
    rnd = types.ModuleType("random_shim")
    rnd.Random = lambda seed=None: belief_rng
    rnd.choice = select.choice
    rnd.choices = select.choices
    rnd.random = select.random
    mcts_mod.random = rnd
    B.random = rnd
    mix = types.ModuleType("random_shim_mixture")
    mix.choice = StreamRandom(streams, S_MIXTURE).choice
    op_mod.random = mix
    clock = _FakeClock()
    mcts_mod.time = clock
    from posggym_baselines.planning.utils import KnownBounds
    kw = dict(cfg_kwargs)
    if kw.get("known_bounds") is not None:
        kw["known_bounds"] = KnownBounds(*kw["known_bounds"])
    config = P.MCTSConfig(**kw)
    other = [i for i in model.possible_agents if i != agent_id][0]

    def fixed(i, pid, probs):
        return FixedDistributionPolicy(model, i, pid, probs,
                                       StreamRandom(streams, S_ACT_BASE + int(i)))

    if spec.get("search") is None:
        search = P.RandomSearchPolicy(model, agent_id)
    else:
        search = sp_mod.SearchPolicyWrapper(fixed(agent_id, "search", spec["search"]))
    o = spec["other"]
    if o["kind"] == "random":
        others = {other: P.RandomOtherAgentPolicy(model, other)}
    elif o["kind"] == "fixed":
        others = {other: fixed(other, "fixed", o["probs"])}
    else:
        others = {other: P.OtherAgentMixturePolicy(
            model, other, {k: fixed(other, k, v) for k, v in o["policies"].items()})}
    if planner_cls == "POMCP":
        assert o["kind"] == "random"
        planner = P.POMCP(model, agent_id, config, search_policy=search)
    else:
        planner = getattr(P, planner_cls)(model, agent_id, config, others, search)
    inner = planner._simulate
    count = [0]

    def simulate(hps, obs_node, depth, search_policy):
        if depth == 0:
            streams.align_sim()   # a simulation starts its step streams at a block (oracle/rng.py)
            count[0] += 1
            if count[0] >= num_sims:
                clock.now += 1e9
                count[0] = 0
        return inner(hps, obs_node, depth, search_policy)

    planner._simulate = simulate
    return planner


def reference_mcts_record(planner, searched, action, spec):
    """``reference_potmmcp_record`` for the base planner: the particles' other-
    agent policy index is 0 unless the other agent is a mixture."""
    from oracle.episode import fhex
    rec = {"searched": searched, "action": int(action)}
    if not searched:
        return rec
    root = planner.root
    other = [i for i in planner.model.possible_agents if i != planner.agent_id][0]
    if spec["other"]["kind"] == "mixture":
        oth_ids = list(planner.other_agent_policies[other].policies)
        parts = [(p.state, p.t, p.policy_state[other]["policy_id"]) for p in root.belief.particles]
    else:
        oth_ids = [0]
        parts = [(p.state, p.t, 0) for p in root.belief.particles]
    st = planner.step_statistics
    rec["belief_size"] = len(parts)
    rec["belief_digest"] = potmmcp_belief_digest(parts, oth_ids, planner.model.pack_words)
    rec["num_sims"] = int(st["num_sims"])
    rec["prior"] = [fhex(root.action_probs[a]) for a in range(len(root.action_probs))]
    if rec["num_sims"] > 0:
        kids = root.get_child_nodes()
        rec["search_depth"] = int(st["search_depth"])
        rec["root_visits"] = int(root.visits)
        rec["child_visits"] = [int(c.visits) for c in kids]
        rec["child_values"] = [fhex(c.value) for c in kids]
        rec["child_totals"] = [fhex(c.total_value) for c in kids]
        rec["min_value"] = fhex(st["min_value"])
        rec["max_value"] = fhex(st["max_value"])
    return rec


def reference_mcts_episode(cfg_kwargs, num_sims, env_seed, spec, ego="0", tree=0, max_steps=50,
                           env="Driving-v1", planner_cls="IPOMCP"):
    """One full episode with the real reference base planner. Returns (trace, records)."""
    from oracle.envs import make_model
    from oracle.episode import run_episode
    from oracle.rng import Streams

    streams = Streams(cfg_kwargs.get("seed") or 0, tree)
    model = make_model(env, streams)
    planner = make_reference_mcts(model, ego, cfg_kwargs, num_sims, streams, spec, planner_cls)
    planner.reset()
    records = []

    def step(obs):
        searched = not planner.root.is_absorbing
        a = planner.step(obs)
        records.append(reference_mcts_record(planner, searched, a, spec))
        return a

    trace = run_episode(step, env_seed, ego=ego, max_steps=max_steps, env=env)
    planner.close()
    return trace, records
