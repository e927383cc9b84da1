"""PursuitEvasion-v1 model, product side.

As for Driving-v1, the planner only needs the model's description (grid,
start / goal sets, observation distance, reward normaliser) to configure the
GPU engine; the dynamics run on the device (``csrc/pursuit_evasion.h``) and
the same header is exposed on the host through the C ABI
(``pomcp_pe_step`` / ``pomcp_pe_sample_initial_state`` / ``pomcp_pe_obs``)
for episode loops.

posggym's PursuitEvasion-v1 is not available in this build environment; the
dynamics are the build's documented restatement (DESIGN.md
"PursuitEvasion-v1"), parity with posggym unpinned; the reward lattice
(R_MAX = 1, R_PROGRESS = 0.01, normalised by 1 + 0.01 * longest start-goal
path) matches the returns the reference's own
``baseline_exps/env_data/PursuitEvasion-v1_i0`` files hold.  Agents: ``'0'``
evader, ``'1'`` pursuer; actions FORWARD, BACKWARD, LEFT, RIGHT (turn, then
move one cell).  Grid layouts are data: ``'#'`` wall, ``'.'`` free, ``'E'``
evader start, ``'P'`` pursuer start, ``'G'`` evader goal.
"""
import ctypes as C
from collections import deque

import numpy as np

from posggym_baselines_amd.envs.driving import Discrete, JointTimestep, Spec

NUM_ACTIONS = 4
MAX_EPISODE_STEPS = 100
ENV_TREE_KEY = 0x40000000
R_MAX, R_PROGRESS = 1.0, 0.01
_DX = (0, 1, 0, -1)
_DY = (-1, 0, 1, 0)

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


def pack_obs(obs) -> int:
    """(walls, seen, heard, (x, y), c1, c2) -> 30-bit key (pursuit_evasion.h layout)."""
    walls, seen, heard, (x, y), (ax, ay), (bx, by) = obs
    return (int(walls) | (int(seen) << 4) | (int(heard) << 5) | (int(x) << 6) | (int(y) << 10)
            | (int(ax) << 14) | (int(ay) << 18) | (int(bx) << 22) | (int(by) << 26))


def unpack_obs(key: int):
    key = int(key)
    return (key & 15, (key >> 4) & 1, (key >> 5) & 1, ((key >> 6) & 15, (key >> 10) & 15),
            ((key >> 14) & 15, (key >> 18) & 15), ((key >> 22) & 15, (key >> 26) & 15))


def build_pe_tables(rows):
    h, w = len(rows), len(rows[0])
    if w > 16 or h > 16:
        raise ValueError("grid must be at most 16x16")
    wall = [[c == "#" for c in r] for r in rows]
    pick = lambda ch: [(x, y) for y, r in enumerate(rows) for x, c in enumerate(r) if c == ch]
    es, ps, goals = pick("E"), pick("P"), pick("G")
    if not (1 <= len(es) <= 4 and 1 <= len(ps) <= 4 and 1 <= len(goals) <= 4):
        raise ValueError("grid needs 1..4 'E', 'P' and 'G' cells")

    def bfs(src):
        d = [[127] * w for _ in range(h)]
        d[src[1]][src[0]] = 0
        q = deque([src])
        while q:
            x, y = q.popleft()
            for k in range(4):
                nx, ny = x + _DX[k], y + _DY[k]
                if 0 <= nx < w and 0 <= ny < h and not wall[ny][nx] and d[ny][nx] == 127:
                    d[ny][nx] = d[y][x] + 1
                    q.append((nx, ny))
        return d

    dist = [bfs(g) for g in goals]
    max_sp = max(d[y][x] for d in dist for (x, y) in es)
    return w, h, wall, es, ps, goals, dist, max_sp


class PursuitEvasionModel:
    """PursuitEvasion-v1 (``grid``, ``max_obs_distance``, ``use_progress_reward``)."""

    env_id = "PursuitEvasion-v1"

    def __init__(self, grid="16x16", max_obs_distance=12, use_progress_reward=True, seed=0):
        self.grid_name = grid
        rows = GRIDS[grid] if isinstance(grid, str) else tuple(grid)
        (self.width, self.height, self._wall, self.evader_starts, self.pursuer_starts,
         self.goals, self._dist, self.max_sp) = build_pe_tables(rows)
        self.max_obs_distance = int(max_obs_distance)
        self.use_progress_reward = bool(use_progress_reward)
        self.reward_norm = R_MAX + self.max_sp * R_PROGRESS
        self.possible_agents = ("0", "1")
        self.action_spaces = {a: Discrete(NUM_ACTIONS, None if seed is None else seed + i)
                              for i, a in enumerate(self.possible_agents)}
        self.spec = Spec("PursuitEvasion-v1", MAX_EPISODE_STEPS)
        self._grid = None
        self.seed(seed)

    # -- engine description -------------------------------------------------
    def pomcp_pe_grid(self):
        from posggym_baselines_amd._native import PomcpPeGrid
        if self._grid is None:
            g = PomcpPeGrid()
            for y in range(self.height):
                for x in range(self.width):
                    g.wall[(y << 4) | x] = 1 if self._wall[y][x] else 0
            for k, d in enumerate(self._dist):
                for c in range(256):
                    g.goal_dist[k][c] = 127
                for y in range(self.height):
                    for x in range(self.width):
                        g.goal_dist[k][(y << 4) | x] = d[y][x]
            for k, (x, y) in enumerate(self.evader_starts):
                g.evader_start[k][0], g.evader_start[k][1] = x, y
            for k, (x, y) in enumerate(self.pursuer_starts):
                g.pursuer_start[k][0], g.pursuer_start[k][1] = x, y
            for k, (x, y) in enumerate(self.goals):
                g.goal[k][0], g.goal[k][1] = x, y
            g.width, g.height = self.width, self.height
            g.n_evader_start, g.n_pursuer_start = len(self.evader_starts), len(self.pursuer_starts)
            g.n_goal = len(self.goals)
            g.max_obs_distance = self.max_obs_distance
            g.use_progress_reward = 1 if self.use_progress_reward else 0
            g.reward_norm = self.reward_norm
            self._grid = g
        return self._grid

    def configure_engine(self, cfg):
        """Fill the environment part of a ``pomcp_config``."""
        from posggym_baselines_amd._native import ENV_PURSUIT_EVASION
        cfg.env_id = ENV_PURSUIT_EVASION
        cfg.pe_grid = self.pomcp_pe_grid()

    def obs_key(self, obs) -> int:
        return obs if isinstance(obs, (int, np.integer)) else pack_obs(obs)

    def obs_from_key(self, key: int):
        return unpack_obs(key)

    # -- host environment (same pursuit_evasion.h through the C ABI) --------
    def seed(self, seed=0):
        self._env_seed = 0 if seed is None else int(seed)
        self._model_ctr = C.c_uint32(0)

    def sample_initial_state(self):
        from posggym_baselines_amd._native import check, load
        out = (C.c_uint32 * 2)()
        check(load().pomcp_pe_sample_initial_state(
            C.byref(self.pomcp_pe_grid()), self._env_seed, ENV_TREE_KEY,
            C.byref(self._model_ctr), out))
        return (int(out[0]), int(out[1]))

    def sample_initial_obs(self, state):
        from posggym_baselines_amd._native import check, load
        st = (C.c_uint32 * 2)(*state)
        keys = (C.c_uint64 * 2)()
        check(load().pomcp_pe_obs(C.byref(self.pomcp_pe_grid()), st, keys))
        return {a: self.obs_from_key(keys[i]) for i, a in enumerate(self.possible_agents)}

    def step(self, state, actions):
        from posggym_baselines_amd._native import check, load
        st = (C.c_uint32 * 2)(*state)
        act = (C.c_int32 * 2)(*[int(actions[a]) for a in self.possible_agents])
        nxt = (C.c_uint32 * 2)()
        rew = (C.c_double * 2)()
        term = (C.c_int32 * 2)()
        keys = (C.c_uint64 * 2)()
        check(load().pomcp_pe_step(C.byref(self.pomcp_pe_grid()), st, act, nxt, rew, term, keys))
        agents = self.possible_agents
        terms = {a: bool(term[i]) for i, a in enumerate(agents)}
        return JointTimestep(
            (int(nxt[0]), int(nxt[1])),
            {a: self.obs_from_key(keys[i]) for i, a in enumerate(agents)},
            {a: float(rew[i]) for i, a in enumerate(agents)},
            terms, {a: False for a in agents}, all(terms.values()), {})
