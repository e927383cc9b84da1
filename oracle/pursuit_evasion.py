"""PursuitEvasion-v1 generative model — the build's restatement (pure Python).

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

posggym (``posggym[agents] >=0.5.0``, ``/root/reference/pyproject.toml:36``,
unpinned, not installed, no network) owns the real PursuitEvasion-v1.  What the
reference's own files pin:
  * env kwargs ``grid="16x16", max_obs_distance=12, use_progress_reward=True``
    (``baseline_exps/env_data/PursuitEvasion-v1_i0/env_kwargs.yaml:1-5``);
  * A = 4 actions and a 108-wide flattened observation
    (4 wall bits x 2 + 2 flags x 2 + three 16x16 coordinates x 32);
  * an episode limit of 100;
  * returns on a 1/124 lattice (``br_results.csv``, ``combined_belief_results.csv``):
    with R_MAX = 1, R_PROGRESS = 0.01 and every reward divided by
    1 + 0.01 * 24, a pursuer return is (100 - k)/124 when it catches an evader
    that made k progress steps and -(100 + k)/124 when the evader reaches its
    goal -- the rule below, with the grid's longest evader-start-to-goal
    shortest path (24 here) in the normaliser.
Everything else (the 16x16 layout, start and goal sets, turn-then-move actions,
the 3-lane field of view, hearing distance 2, simultaneous moves with capture on
meeting or swapping) is the build's documented choice: parity with posggym is
UNPINNED.  The HIP device model (``csrc/pursuit_evasion.h``) restates this file.

Agents: ``'0'`` evader, ``'1'`` pursuer.  The model step is deterministic (no
model-stream draw); initial states draw from the model stream.
"""
from collections import deque, namedtuple

from oracle.driving import Discrete
from oracle.rng import S_ACT_BASE, S_MODEL, Streams

NORTH, EAST, SOUTH, WEST = 0, 1, 2, 3
DIR_DX = (0, 1, 0, -1)
DIR_DY = (-1, 0, 1, 0)
FORWARD, BACKWARD, LEFT, RIGHT = 0, 1, 2, 3
NUM_ACTIONS = 4
TURN = (0, 2, 3, 1)            # direction change of each action (mod 4)
EVADER, PURSUER = 0, 1

R_MAX = 1.0
R_PROGRESS = 0.01
HEARING_DIST = 2
MAX_EPISODE_STEPS = 100

# '#' wall, '.' free, 'E' evader start, 'P' pursuer start, 'G' evader goal.
GRIDS = {
    "16x16": (
        "G......#.E.....G",
        ".##.##...##.##..",
        ".#...#.#.#...#..",
        "...#.#.#...#...#",
        "##.#...#.#.#.#..",
        "...#.###.#...#..",
        ".#.......###.##.",
        "E#.##.#P........",
        "...#..#.#.#.##.#",
        ".#.#.##.P.#....E",
        ".#...#..#.#.#.#.",
        ".###.#.##...#.#.",
        "..........#.#...",
        ".#.##.##.##.#.#.",
        ".#..........#.#.",
        "G...#.#.#E#....G",
    ),
    # small layout for fast unit tests
    "8x8": (
        "G..#...E",
        ".#...#..",
        ".#.##.#.",
        "...P....",
        ".##..#.#",
        "...#....",
        "E#...##.",
        "...#...G",
    ),
}

Spec = namedtuple("Spec", ["id", "max_episode_steps"])
JointTimestep = namedtuple(
    "JointTimestep",
    ["state", "observations", "rewards", "terminations", "truncations", "all_done", "infos"],
)


class PEGrid:
    def __init__(self, rows, max_obs_distance=12):
        self.height = len(rows)
        self.width = len(rows[0])
        assert self.width <= 16 and self.height <= 16
        self.wall = [[c == "#" for c in r] for r in rows]
        pick = lambda ch: [(x, y) for y, r in enumerate(rows) for x, c in enumerate(r) if c == ch]
        self.evader_starts = pick("E")
        self.pursuer_starts = pick("P")
        self.goals = pick("G")
        assert 1 <= len(self.evader_starts) <= 4 and 1 <= len(self.pursuer_starts) <= 4
        assert 1 <= len(self.goals) <= 4
        self.max_obs_distance = max_obs_distance
        self.goal_dist = [self._bfs(g) for g in self.goals]
        # longest shortest path from an evader start to a goal: reward normaliser
        self.max_sp = max(d[y][x] for d in self.goal_dist for (x, y) in self.evader_starts)

    def free(self, x, y):
        return 0 <= x < self.width and 0 <= y < self.height and not self.wall[y][x]

    def _bfs(self, src):
        inf = 127
        d = [[inf] * self.width for _ in range(self.height)]
        d[src[1]][src[0]] = 0
        q = deque([src])
        while q:
            x, y = q.popleft()
            for k in range(4):
                nx, ny = x + DIR_DX[k], y + DIR_DY[k]
                if self.free(nx, ny) and d[ny][nx] == inf:
                    d[ny][nx] = d[y][x] + 1
                    q.append((nx, ny))
        return d

    def wall_bits(self, x, y):
        return sum((0 if self.free(x + DIR_DX[k], y + DIR_DY[k]) else 1) << k for k in range(4))

    def lane_len(self, x, y, d, side):
        """Free cells straight ahead (<= max_obs_distance) in the lane `side`
        cells to the right (-1 left, 0 centre, +1 right) of heading d."""
        fx, fy = DIR_DX[d], DIR_DY[d]
        rx, ry = DIR_DX[(d + 1) & 3], DIR_DY[(d + 1) & 3]
        n = 0
        for k in range(1, self.max_obs_distance + 1):
            if not self.free(x + k * fx + side * rx, y + k * fy + side * ry):
                break
            n = k
        return n


# Evader: (x, y, dir, start_idx, goal_idx, min_goal_dist, caught, reached)
# Pursuer: (x, y, dir, start_idx)
def pack_evader(e) -> int:
    return (e[0] | (e[1] << 4) | (e[2] << 8) | (e[3] << 10) | (e[4] << 12) | (e[5] << 14)
            | (e[6] << 21) | (e[7] << 22))


def unpack_evader(u: int):
    return (u & 15, (u >> 4) & 15, (u >> 8) & 3, (u >> 10) & 3, (u >> 12) & 3,
            (u >> 14) & 127, (u >> 21) & 1, (u >> 22) & 1)


def pack_pursuer(p) -> int:
    return p[0] | (p[1] << 4) | (p[2] << 8) | (p[3] << 10)


def unpack_pursuer(u: int):
    return (u & 15, (u >> 4) & 15, (u >> 8) & 3, (u >> 10) & 3)


def pack_state_words(state):
    return pack_evader(state[0]), pack_pursuer(state[1])


def unpack_state_words(v0, v1):
    return (unpack_evader(v0), unpack_pursuer(v1))


def pack_obs(obs) -> int:
    walls, seen, heard, (x, y), (ax, ay), (bx, by) = obs
    return (walls | (seen << 4) | (heard << 5) | (x << 6) | (y << 10) | (ax << 14) | (ay << 18)
            | (bx << 22) | (by << 26))


def unpack_obs(key: int):
    return (key & 15, (key >> 4) & 1, (key >> 5) & 1, ((key >> 6) & 15, (key >> 10) & 15),
            ((key >> 14) & 15, (key >> 18) & 15), ((key >> 22) & 15, (key >> 26) & 15))


class PursuitEvasionModel:
    """PursuitEvasion-v1 restatement (2 agents: '0' evader, '1' pursuer)."""

    env_id = "PursuitEvasion-v1"
    pack_obs = staticmethod(pack_obs)
    pack_words = staticmethod(pack_state_words)

    def __init__(self, streams: Streams, grid="16x16", max_obs_distance=12,
                 use_progress_reward=True):
        self.grid_name = grid
        self.grid = PEGrid(GRIDS[grid], max_obs_distance)
        self.use_progress_reward = use_progress_reward
        self.reward_norm = R_MAX + self.grid.max_sp * R_PROGRESS
        self.possible_agents = ("0", "1")
        self.num_agents = 2
        self.streams = streams
        self.action_spaces = {str(i): Discrete(NUM_ACTIONS, streams, S_ACT_BASE + i)
                              for i in range(2)}
        self.spec = Spec("PursuitEvasion-v1", MAX_EPISODE_STEPS)

    def _evader(self, sidx, gidx, d):
        x, y = self.grid.evader_starts[sidx]
        gx, gy = self.grid.goals[gidx]
        return (x, y, d, sidx, gidx, self.grid.goal_dist[gidx][y][x], 0, 0)

    def _pursuer(self, sidx, d):
        x, y = self.grid.pursuer_starts[sidx]
        return (x, y, d, sidx)

    def sample_initial_state(self):
        g = self.grid
        r = lambda n: self.streams.randint(S_MODEL, n)
        es = r(len(g.evader_starts))
        ps = r(len(g.pursuer_starts))
        gi = r(len(g.goals))
        ed = r(4)
        pd = r(4)
        return (self._evader(es, gi, ed), self._pursuer(ps, pd))

    def sample_initial_obs(self, state):
        return {str(i): self._obs(state, i) for i in range(2)}

    def sample_agent_initial_state(self, agent_id, obs):
        """Ego's own start (and the evader's goal / start it observes) from its
        obs; the unknowns drawn and rejected until the obs matches (<= 64 tries,
        then the last draw)."""
        g = self.grid
        r = lambda n: self.streams.randint(S_MODEL, n)
        i = int(agent_id)
        _, _, _, own, c1, c2 = obs
        state = None
        for _ in range(64):
            if i == EVADER:
                es = g.evader_starts.index(own)
                gi = g.goals.index(c2)
                ed = r(4)
                ps = r(len(g.pursuer_starts))
                pd = r(4)
            else:
                ps = g.pursuer_starts.index(own)
                es = g.evader_starts.index(c2)
                gi = r(len(g.goals))
                ed = r(4)
                pd = r(4)
            state = (self._evader(es, gi, ed), self._pursuer(ps, pd))
            if self._obs(state, i) == obs:
                break
        return state

    def _obs(self, state, i):
        g = self.grid
        e, p = state
        me, other = (e, p) if i == EVADER else (p, e)
        x, y, d = me[0], me[1], me[2]
        fx, fy = DIR_DX[d], DIR_DY[d]
        rx, ry = DIR_DX[(d + 1) & 3], DIR_DY[(d + 1) & 3]
        dx, dy = other[0] - x, other[1] - y
        fwd = dx * fx + dy * fy
        side = dx * rx + dy * ry
        seen = 1 if (-1 <= side <= 1 and 1 <= fwd <= g.lane_len(x, y, d, side)) else 0
        man = abs(dx) + abs(dy)
        heard = 1 if 0 < man <= HEARING_DIST else 0
        if i == EVADER:
            c1 = g.evader_starts[e[3]]
            c2 = g.goals[e[4]]
        else:
            c1 = g.pursuer_starts[p[3]]
            c2 = g.evader_starts[e[3]]
        return (g.wall_bits(x, y), seen, heard, (x, y), c1, c2)

    def _move(self, x, y, d, a):
        nd = (d + TURN[a]) & 3
        nx, ny = x + DIR_DX[nd], y + DIR_DY[nd]
        if self.grid.free(nx, ny):
            return nx, ny, nd
        return x, y, nd

    def _evader_reward(self, e0, e1):
        r = 0.0
        if self.use_progress_reward and e1[5] < e0[5]:
            r += R_PROGRESS
        if e1[6]:
            r -= R_MAX
        elif e1[7]:
            r += R_MAX
        return r / self.reward_norm

    def step(self, state, actions):
        e, p = state
        if e[6] or e[7]:   # absorbing
            nxt = state
            re = 0.0
        else:
            ex, ey, ed = self._move(e[0], e[1], e[2], actions["0"])
            px, py, pd = self._move(p[0], p[1], p[2], actions["1"])
            caught = (ex, ey) == (px, py) or ((ex, ey) == (p[0], p[1]) and (px, py) == (e[0], e[1]))
            gx, gy = self.grid.goals[e[4]]
            reached = 0 if caught else int((ex, ey) == (gx, gy))
            mgd = min(e[5], self.grid.goal_dist[e[4]][ey][ex])
            ne = (ex, ey, ed, e[3], e[4], mgd, int(caught), reached)
            nxt = (ne, (px, py, pd, p[3]))
            re = self._evader_reward(e, ne)
        done = bool(nxt[0][6] or nxt[0][7])
        rewards = {"0": re, "1": 0.0 - re}
        terms = {"0": done, "1": done}
        obs = {str(i): self._obs(nxt, i) for i in range(2)}
        return JointTimestep(nxt, obs, rewards, terms, {"0": False, "1": False}, done, {})


def pack_state(state, t) -> tuple:
    """Particle record as the GPU stores it: (t, v0, v1) u32 words."""
    v0, v1 = pack_state_words(state)
    return (t, v0, v1)
