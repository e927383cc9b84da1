"""Episode loop + per-step records (shared by the reference harness, the oracle
and the parity tests).

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

The loop follows ``tests/planning/test_pomcp.py:16-33`` (reset, then
``planner.step(obs[ego])`` once per env step against a uniform-random other
agent, until ``all_done``; posggym's TimeLimit truncates at 50 steps).  The
"real" environment is its own ``DrivingModel`` instance on its own RNG key so
that the planner's model draws are never interleaved with the env's.
"""
import hashlib
import struct

from oracle.driving import DrivingModel
from oracle.envs import make_model
from oracle.rng import S_ENV_POLICY_BASE, Streams

ENV_TREE_BASE = 0x40000000


def fhex(x):
    return float(x).hex()


def belief_digest(particles, pack_words=DrivingModel.pack_words):
    """sha1 over (t, v0, v1) u32 little-endian triples, insertion order."""
    h = hashlib.sha1()
    for st, t in particles:
        v0, v1 = pack_words(st)
        h.update(struct.pack("<III", t, v0, v1))
    return h.hexdigest()


def run_episode(planner_step, env_seed, ego="0", num_agents=2, grid=None,
                max_steps=50, on_step=None, env="Driving-v1"):
    """Drive one episode.  ``planner_step(obs) -> action``; ``on_step(t, obs, action)``
    is called after each planner step (to capture planner-side records)."""
    env_streams = Streams(env_seed, ENV_TREE_BASE)
    env = make_model(env, env_streams, grid=grid)
    state = env.sample_initial_state()
    obs = env.sample_initial_obs(state)
    trace = {"env_seed": env_seed, "steps": []}
    ret = 0.0
    for t in range(max_steps):
        a_ego = planner_step(obs[ego])
        actions = {}
        for i in env.possible_agents:
            if i == ego:
                actions[i] = a_ego
            else:
                actions[i] = env_streams.randint(S_ENV_POLICY_BASE + int(i),
                                                 env.action_spaces[i].n)
        if on_step is not None:
            on_step(t, obs[ego], a_ego)
        ts = env.step(state, actions)
        ret += ts.rewards[ego]
        trace["steps"].append({"obs": env.pack_obs(obs[ego]), "actions": [actions[i] for i in env.possible_agents],
                               "reward": fhex(ts.rewards[ego])})
        state, obs = ts.state, ts.observations
        if ts.all_done:
            break
    trace["return"] = fhex(ret)
    trace["len"] = len(trace["steps"])
    return trace
