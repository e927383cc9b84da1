"""The invariant k_search_lds's step-tree producer waves rely on
(csrc/pomcp_search_lds.hip): a simulation that does not
terminate draws exactly depth_limit + 1 words from the model stream (Driving's
execution-order shuffle, one per joint step) and from the other agent's action
stream -- its tree levels plus its rollout reach the depth limit
(mcts.py:315-328, 405-452) -- and fewer when a step terminates it.  The
producers predict simulation k's words from that; a wrong prediction would only
cost speed (the search wave checks the counters), but the test pins why the
prediction holds.  Checked on the oracle (pinned to the reference goldens)."""
import math

import pytest

from oracle.episode import run_episode
from oracle.rng import S_ACT_BASE, S_MODEL
from oracle.run import make_oracle

CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
           action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
           step_limit=None, epsilon=0.92, seed=3, state_belief_only=True)


@pytest.mark.parametrize("epsilon,env", [(0.92, "Driving-v1"), (0.75, "Driving-v1"),
                                         (0.92, "PursuitEvasion-v1")])
def test_words_per_simulation_are_depth_limit_plus_one(epsilon, env):
    p = make_oracle(dict(CFG, epsilon=epsilon), 100, env=env)
    d1 = p.cfg.depth_limit + 1
    other = next(i for i in p.model.possible_agents if i != p.agent_id)
    s_oth = S_ACT_BASE + int(other)
    draws_model = 1 if env == "Driving-v1" else 0
    done_seen = []
    step = p.model.step

    def spy_step(state, actions):
        ts = step(state, actions)
        if ts.all_done or any(ts.terminations.values()) or any(ts.truncations.values()):
            done_seen.append(True)
        return ts

    p.model.step = spy_step
    sim = p._simulate
    deltas = []

    def spy_sim(st, t, node):
        c0 = p.s.counters()
        done_seen.clear()
        depth = sim(st, t, node)
        c1 = p.s.counters()
        dm = c1.get(S_MODEL, 0) - c0.get(S_MODEL, 0)
        do = c1.get(s_oth, 0) - c0.get(s_oth, 0)
        deltas.append((dm, do, bool(done_seen)))
        return depth

    p._simulate = spy_sim
    run_episode(p.step, 11, ego=p.agent_id, max_steps=3, env=env)
    assert len(deltas) >= 300
    full = [(dm, do) for dm, do, dn in deltas if not dn]
    assert full, "every simulation terminated"
    assert all(do == d1 and dm == draws_model * d1 for dm, do in full)
    assert all(do <= d1 and dm <= draws_model * d1 for dm, do, _ in deltas)
