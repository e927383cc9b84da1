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
    mod("posggym.utils.history", JointHistory=_Any, AgentHistory=_Any)
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


def make_reference_pomcp(model, agent_id, cfg_kwargs, num_sims, streams):
    """Build a reference ``POMCP`` wired to ``streams`` and a fixed sim count."""
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
    planner = P.POMCP(model, agent_id, config, search_policy=P.RandomSearchPolicy(model, agent_id))
    inner = planner._simulate
    count = [0]

    def simulate(hps, obs_node, depth, search_policy):
        if depth == 0:
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
                      tree=0, max_steps=50, env="Driving-v1"):
    """One full episode with the real reference POMCP. Returns (trace, records)."""
    from oracle.envs import make_model
    from oracle.episode import run_episode
    from oracle.rng import Streams

    streams = Streams(cfg_kwargs.get("seed") or 0, tree)
    model = make_model(env, streams, grid=grid)
    planner = make_reference_pomcp(model, ego, cfg_kwargs, num_sims, streams)
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
