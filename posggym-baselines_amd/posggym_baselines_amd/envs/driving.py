"""Driving-v1 model, product side.

The planner only needs the model's identity (grid, agents, action count,
observation window, episode limit) to configure the GPU engine; the dynamics
run on the device (``csrc/driving.h``).  For episode loops the same
``driving.h`` is exposed on the host through the C ABI
(``pomcp_driving_step`` / ``pomcp_driving_sample_initial_state``), so the
environment and the planner's generative model are one implementation.

posggym's own Driving-v1 is not available in this build environment; the
dynamics are the build's documented restatement (DESIGN.md "Driving-v1"),
parity with posggym unpinned.  Grid layouts are data: ``'#'`` wall, ``'.'``
road, ``'+'`` start/destination location.
"""
import ctypes as C
from collections import namedtuple

import numpy as np

NORTH, EAST, SOUTH, WEST = 0, 1, 2, 3
_DX = (0, 1, 0, -1)
_DY = (-1, 0, 1, 0)
NUM_ACTIONS = 5
MAX_EPISODE_STEPS = 50
ENV_TREE_KEY = 0x40000000

GRIDS = {
    "14x14RoundAbout": (
        "######++######",
        "######..######",
        "######..######",
        "###........###",
        "###........###",
        "###..####..###",
        "+....####....+",
        "+....####....+",
        "###..####..###",
        "###........###",
        "###........###",
        "######..######",
        "######..######",
        "######++######",
    ),
    "7x7RoundAbout": (
        "###+###",
        "##...##",
        "#.#.#.#",
        "+.....+",
        "#.#.#.#",
        "##...##",
        "###+###",
    ),
}

Spec = namedtuple("Spec", ["id", "max_episode_steps"])
JointTimestep = namedtuple(
    "JointTimestep",
    ["state", "observations", "rewards", "terminations", "truncations", "all_done", "infos"])


class Discrete:
    """Minimal ``gymnasium.spaces.Discrete`` (``n`` + ``sample``)."""

    def __init__(self, n, seed=None):
        self.n = n
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return int(self._rng.integers(self.n))


def build_grid_tables(rows):
    """Walls, location list, initial headings and BFS distance tables."""
    h, w = len(rows), len(rows[0])
    if w > 16 or h > 16:
        raise ValueError("grid must be at most 16x16")
    wall = [[c == "#" for c in r] for r in rows]
    locs = [(x, y) for y, r in enumerate(rows) for x, c in enumerate(r) if c == "+"]
    if not 2 <= len(locs) <= 8:
        raise ValueError("grid needs 2..8 '+' locations")

    def free(x, y):
        return 0 <= x < w and 0 <= y < h and not wall[y][x]

    dirs = []
    for (x, y) in locs:
        dirs.append(SOUTH if y == 0 else NORTH if y == h - 1 else EAST if x == 0
                    else WEST if x == w - 1 else NORTH)
    dist = []
    for (lx, ly) in locs:
        d = [[127] * w for _ in range(h)]
        d[ly][lx] = 0
        frontier = [(lx, ly)]
        while frontier:
            nxt = []
            for (x, y) in frontier:
                for k in range(4):
                    nx, ny = x + _DX[k], y + _DY[k]
                    if free(nx, ny) and d[ny][nx] == 127:
                        d[ny][nx] = d[y][x] + 1
                        nxt.append((nx, ny))
            frontier = nxt
        dist.append(d)
    return w, h, wall, locs, dirs, dist


def pack_obs(obs) -> int:
    """Ego observation tuple -> u64 key (layout of driving.h)."""
    cells, speed, (x, y), (dx, dy), reached, crashed = obs
    key = 0
    for c, v in enumerate(cells):
        key |= int(v) << (2 * c)
    return (key | (int(speed) << 30) | (int(x) << 32) | (int(y) << 36) | (int(dx) << 40)
            | (int(dy) << 44) | (int(reached) << 48) | (int(crashed) << 49))


def unpack_obs(key: int, ncells: int = 15):
    cells = tuple((key >> (2 * c)) & 3 for c in range(ncells))
    return (cells, (key >> 30) & 3, ((key >> 32) & 15, (key >> 36) & 15),
            ((key >> 40) & 15, (key >> 44) & 15), (key >> 48) & 1, (key >> 49) & 1)


class DrivingModel:
    """Driving-v1 (``grid``, ``num_agents=2``, ``obs_dim=(front, back, side)``)."""

    env_id = "Driving-v1"

    def __init__(self, grid="14x14RoundAbout", num_agents=2, obs_dim=(3, 1, 1), seed=0):
        if num_agents != 2:
            raise NotImplementedError("the GPU engine implements 2-agent Driving-v1")
        self.grid_name = grid
        rows = GRIDS[grid] if isinstance(grid, str) else tuple(grid)
        self.width, self.height, self._wall, self.locs, self.loc_dirs, self._dist = \
            build_grid_tables(rows)
        self.num_agents = num_agents
        self.obs_dim = tuple(obs_dim)
        self.ncells = (obs_dim[0] + obs_dim[1] + 1) * (2 * obs_dim[2] + 1)
        if self.ncells > 15:
            raise ValueError("observation window must have at most 15 cells")
        self.possible_agents = tuple(str(i) for i in range(num_agents))
        self.action_spaces = {a: Discrete(NUM_ACTIONS, None if seed is None else seed + i)
                              for i, a in enumerate(self.possible_agents)}
        self.spec = Spec("Driving-v1", MAX_EPISODE_STEPS)
        self._grid = None
        self.seed(seed)

    # -- engine description -------------------------------------------------
    def pomcp_grid(self):
        from posggym_baselines_amd._native import PomcpGrid
        if self._grid is None:
            g = PomcpGrid()
            for y in range(self.height):
                for x in range(self.width):
                    g.wall[(y << 4) | x] = 1 if self._wall[y][x] else 0
            for k, d in enumerate(self._dist):
                for y in range(self.height):
                    for x in range(self.width):
                        g.dist[k][(y << 4) | x] = d[y][x]
            for k, (x, y) in enumerate(self.locs):
                g.loc_x[k], g.loc_y[k], g.loc_dir[k] = x, y, self.loc_dirs[k]
            g.width, g.height, g.num_locs = self.width, self.height, len(self.locs)
            g.obs_front, g.obs_back, g.obs_side = self.obs_dim
            self._grid = g
        return self._grid

    def configure_engine(self, cfg):
        """Fill the environment part of a ``pomcp_config``."""
        from posggym_baselines_amd._native import ENV_DRIVING
        cfg.env_id = ENV_DRIVING
        cfg.grid = self.pomcp_grid()

    def obs_key(self, obs) -> int:
        return obs if isinstance(obs, (int, np.integer)) else pack_obs(obs)

    def obs_from_key(self, key: int):
        return unpack_obs(int(key), self.ncells)

    # -- host environment (same driving.h through the C ABI) ----------------
    def seed(self, seed=0):
        self._env_seed = 0 if seed is None else int(seed)
        self._model_ctr = C.c_uint32(0)

    def sample_initial_state(self):
        from posggym_baselines_amd._native import check, load
        out = (C.c_uint32 * 2)()
        check(load().pomcp_driving_sample_initial_state(
            C.byref(self.pomcp_grid()), self._env_seed, ENV_TREE_KEY, C.byref(self._model_ctr),
            out))
        return (int(out[0]), int(out[1]))

    def sample_initial_obs(self, state):
        from posggym_baselines_amd._native import check, load
        st = (C.c_uint32 * 2)(*state)
        keys = (C.c_uint64 * 2)()
        check(load().pomcp_driving_obs(C.byref(self.pomcp_grid()), st, keys))
        return {a: self.obs_from_key(keys[i]) for i, a in enumerate(self.possible_agents)}

    def step(self, state, actions):
        from posggym_baselines_amd._native import check, load
        st = (C.c_uint32 * 2)(*state)
        act = (C.c_int32 * 2)(*[int(actions[a]) for a in self.possible_agents])
        nxt = (C.c_uint32 * 2)()
        rew = (C.c_double * 2)()
        term = (C.c_int32 * 2)()
        keys = (C.c_uint64 * 2)()
        check(load().pomcp_driving_step(C.byref(self.pomcp_grid()), self._env_seed, ENV_TREE_KEY,
                                        C.byref(self._model_ctr), st, act, nxt, rew, term, keys))
        agents = self.possible_agents
        terms = {a: bool(term[i]) for i, a in enumerate(agents)}
        return JointTimestep(
            (int(nxt[0]), int(nxt[1])),
            {a: self.obs_from_key(keys[i]) for i, a in enumerate(agents)},
            {a: float(rew[i]) for i, a in enumerate(agents)},
            terms, {a: False for a in agents}, all(terms.values()), {})
