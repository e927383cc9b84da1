"""Driving-v1 generative model — the build's restatement (pure Python).

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

posggym (``posggym[agents] >=0.5.0``, ``/root/reference/pyproject.toml:36``,
unpinned, not installed, no network) owns the real Driving-v1.  Its source is
absent, so the dynamics below are restated from the environment's published
description and the invariants the reference's own data files pin
(SURVEY Appendix C): A = 5 actions, a 5x3 local window for
``obs_dim=(3, 1, 1)``, a 124-wide flattened observation
(15 cells x 4 classes + speed(4) + own coord (14+14) + dest coord (14+14) +
two flags), an episode limit of 50 and the return lattice
{1.0, 0.5*k/D, -1 + 0.5*k/D}.  Everything else (grid layout, move/collision
order, reward split) is the build's documented choice: parity with posggym is
UNPINNED.  The HIP device model (``csrc/driving.h``) restates this file.

Model interface used by the reference planner (call sites ``mcts.py:181,
191-198, 333, 418``; ``belief.py:165``): ``possible_agents``,
``action_spaces[i].sample()/.n``, ``spec.max_episode_steps``,
``sample_initial_state()``, ``sample_initial_obs(state)``,
``sample_agent_initial_state(agent_id, obs)``, ``step(state, joint_action)``
returning a ``JointTimestep`` with ``state, observations, rewards,
terminations, truncations, all_done, infos``.
"""
from collections import namedtuple

from oracle.rng import S_ACT_BASE, S_MODEL, StreamRandom, Streams

# --- constants (kept in sync with csrc/driving.h) ---------------------------
NORTH, EAST, SOUTH, WEST = 0, 1, 2, 3
DIR_DX = (0, 1, 0, -1)
DIR_DY = (-1, 0, 1, 0)

REVERSE, STOPPED, FORWARD_SLOW, FORWARD_FAST = 0, 1, 2, 3
DO_NOTHING, ACCELERATE, DECELERATE, TURN_RIGHT, TURN_LEFT = 0, 1, 2, 3, 4
NUM_ACTIONS = 5

VEHICLE, WALL, EMPTY, DESTINATION = 0, 1, 2, 3

R_CRASH_VEHICLE = -1.0
R_DESTINATION_REACHED = 0.5
R_PROGRESS_TOTAL = 0.5       # progress shaping sums to 0.5 over the initial distance

MAX_EPISODE_STEPS = 50

# '#' wall, '.' road, '+' road cell that is a start and destination location.
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
    # small layout used only by fast unit tests
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
    ["state", "observations", "rewards", "terminations", "truncations", "all_done", "infos"],
)


class Discrete:
    """gymnasium.spaces.Discrete stand-in; ``sample()`` draws from a stream."""

    def __init__(self, n: int, streams: Streams, stream_id: int):
        self.n = n
        self._streams = streams
        self._sid = stream_id

    def sample(self) -> int:
        return self._streams.randint(self._sid, self.n)


class Grid:
    def __init__(self, rows):
        self.height = len(rows)
        self.width = len(rows[0])
        assert self.width <= 16 and self.height <= 16
        self.wall = [[c == "#" for c in r] for r in rows]
        self.locs = [(x, y) for y, r in enumerate(rows) for x, c in enumerate(r) if c == "+"]
        assert 2 <= len(self.locs) <= 8
        self.init_dir = []
        for (x, y) in self.locs:
            if y == 0:
                d = SOUTH
            elif y == self.height - 1:
                d = NORTH
            elif x == 0:
                d = EAST
            elif x == self.width - 1:
                d = WEST
            else:
                d = NORTH
            self.init_dir.append(d)
        # BFS shortest-path distance (4-connected over road cells) to every location.
        inf = 127
        self.dist = []
        for (lx, ly) in self.locs:
            d = [[inf] * self.width for _ in range(self.height)]
            d[ly][lx] = 0
            frontier = [(lx, ly)]
            while frontier:
                nxt = []
                for (x, y) in frontier:
                    for k in range(4):
                        nx, ny = x + DIR_DX[k], y + DIR_DY[k]
                        if self.free(nx, ny) and d[ny][nx] == inf:
                            d[ny][nx] = d[y][x] + 1
                            nxt.append((nx, ny))
                frontier = nxt
            self.dist.append(d)

    def free(self, x, y):
        return 0 <= x < self.width and 0 <= y < self.height and not self.wall[y][x]


# Vehicle state: (x, y, dir, speed, dest, dest_reached, crashed, min_dest_dist, init_dest_dist)
VX, VY, VDIR, VSPEED, VDEST, VREACHED, VCRASHED, VMIN, VINIT = range(9)


def pack_vehicle(v) -> int:
    return (v[0] | (v[1] << 4) | (v[2] << 8) | (v[3] << 10) | (v[4] << 12)
            | (v[5] << 15) | (v[6] << 16) | (v[7] << 17) | (v[8] << 24))


def unpack_vehicle(u: int):
    return (u & 15, (u >> 4) & 15, (u >> 8) & 3, (u >> 10) & 3, (u >> 12) & 7,
            (u >> 15) & 1, (u >> 16) & 1, (u >> 17) & 127, (u >> 24) & 127)


def pack_obs(obs) -> int:
    cells, speed, (x, y), (dx, dy), reached, crashed = obs
    key = 0
    for c, v in enumerate(cells):
        key |= v << (2 * c)
    return key | (speed << 30) | (x << 32) | (y << 36) | (dx << 40) | (dy << 44) \
        | (reached << 48) | (crashed << 49)


class DrivingModel:
    """Driving-v1 restatement, 2+ agents, ``obs_dim=(front, back, side)``."""

    env_id = "Driving-v1"
    pack_obs = staticmethod(pack_obs)

    @staticmethod
    def pack_words(state):
        return pack_vehicle(state[0]), pack_vehicle(state[1])

    def __init__(self, streams: Streams, grid="14x14RoundAbout", num_agents=2,
                 obs_dim=(3, 1, 1)):
        self.grid_name = grid
        self.grid = Grid(GRIDS[grid])
        self.num_agents = num_agents
        self.obs_front, self.obs_back, self.obs_side = obs_dim
        self.possible_agents = tuple(str(i) for i in range(num_agents))
        self.streams = streams
        self.rng = StreamRandom(streams, S_MODEL)
        self.action_spaces = {
            str(i): Discrete(NUM_ACTIONS, streams, S_ACT_BASE + i) for i in range(num_agents)
        }
        self.spec = Spec("Driving-v1", MAX_EPISODE_STEPS)

    # -- initial state ------------------------------------------------------
    def _make_vehicle(self, loc, dest):
        d = self.grid.dist[dest][self.grid.locs[loc][1]][self.grid.locs[loc][0]]
        x, y = self.grid.locs[loc]
        return (x, y, self.grid.init_dir[loc], STOPPED, dest, 0, 0, d, d)

    def sample_initial_state(self):
        n_loc = len(self.grid.locs)
        starts, dests, state = [], [], []
        for _ in range(self.num_agents):
            avail = [k for k in range(n_loc) if k not in starts]
            s = avail[self.streams.randint(S_MODEL, len(avail))]
            starts.append(s)
            avail_d = [k for k in range(n_loc) if k not in dests and k != s]
            d = avail_d[self.streams.randint(S_MODEL, len(avail_d))]
            dests.append(d)
            state.append(self._make_vehicle(s, d))
        return tuple(state)

    def sample_initial_obs(self, state):
        return {str(i): self._obs(state, i) for i in range(self.num_agents)}

    def sample_agent_initial_state(self, agent_id, obs):
        """Ego vehicle from its own obs; other vehicles sampled, rejected until the
        ego's local window matches (bounded at 64 tries, then the last draw)."""
        ego = int(agent_id)
        (ex, ey), (edx, edy) = obs[2], obs[3]
        locs = self.grid.locs
        e_loc = locs.index((ex, ey))
        e_dest = locs.index((edx, edy))
        n_loc = len(locs)
        state = None
        for _ in range(64):
            starts, dests = [e_loc], [e_dest]
            vs = [None] * self.num_agents
            vs[ego] = self._make_vehicle(e_loc, e_dest)
            for j in range(self.num_agents):
                if j == ego:
                    continue
                avail = [k for k in range(n_loc) if k not in starts]
                s = avail[self.streams.randint(S_MODEL, len(avail))]
                starts.append(s)
                avail_d = [k for k in range(n_loc) if k not in dests and k != s]
                d = avail_d[self.streams.randint(S_MODEL, len(avail_d))]
                dests.append(d)
                vs[j] = self._make_vehicle(s, d)
            state = tuple(vs)
            if self._obs(state, ego) == obs:
                break
        return state

    # -- observation --------------------------------------------------------
    def _obs(self, state, i):
        v = state[i]
        x, y, d = v[VX], v[VY], v[VDIR]
        fx, fy = DIR_DX[d], DIR_DY[d]
        r = (d + 1) & 3
        rx, ry = DIR_DX[r], DIR_DY[r]
        dest_x, dest_y = self.grid.locs[v[VDEST]]
        cells = []
        for fwd in range(self.obs_front, -self.obs_back - 1, -1):
            for side in range(-self.obs_side, self.obs_side + 1):
                cx = x + fwd * fx + side * rx
                cy = y + fwd * fy + side * ry
                if not self.grid.free(cx, cy):
                    cells.append(WALL)
                elif any(j != i and state[j][VX] == cx and state[j][VY] == cy
                         for j in range(self.num_agents)):
                    cells.append(VEHICLE)
                elif cx == dest_x and cy == dest_y:
                    cells.append(DESTINATION)
                else:
                    cells.append(EMPTY)
        return (tuple(cells), v[VSPEED], (x, y), (dest_x, dest_y), v[VREACHED], v[VCRASHED])

    # -- dynamics -----------------------------------------------------------
    def step(self, state, actions):
        n = self.num_agents
        order = list(range(n))
        self.rng.shuffle(order)          # execution order: one model draw per swap
        nxt = list(state)
        for idx in order:
            v = nxt[idx]
            if v[VREACHED] or v[VCRASHED]:
                continue
            a = actions[str(idx)]
            d, speed = v[VDIR], v[VSPEED]
            if a == TURN_RIGHT:
                d = (d + 1) & 3
            elif a == TURN_LEFT:
                d = (d + 3) & 3
            elif a == ACCELERATE:
                speed = min(speed + 1, FORWARD_FAST)
            elif a == DECELERATE:
                speed = max(speed - 1, REVERSE)
            move = d if speed != REVERSE else (d + 2) & 3
            cells = abs(speed - STOPPED)
            x, y = v[VX], v[VY]
            hit = -1
            for _ in range(cells):
                nx, ny = x + DIR_DX[move], y + DIR_DY[move]
                if not self.grid.free(nx, ny):
                    speed = STOPPED
                    break
                for j in range(n):
                    if j != idx and nxt[j][VX] == nx and nxt[j][VY] == ny:
                        hit = j
                        break
                if hit >= 0:
                    speed = STOPPED
                    break
                x, y = nx, ny
            dist = self.grid.dist[v[VDEST]][y][x]
            reached = 1 if dist == 0 else 0
            crashed = 1 if hit >= 0 else 0
            nxt[idx] = (x, y, d, speed, v[VDEST], reached, crashed, min(v[VMIN], dist), v[VINIT])
            if crashed:
                h = nxt[hit]
                if not (h[VREACHED] or h[VCRASHED]):
                    nxt[hit] = h[:VCRASHED] + (1,) + h[VCRASHED + 1:]
        next_state = tuple(nxt)
        rewards, terms, truncs, obs = {}, {}, {}, {}
        for i in range(n):
            aid = str(i)
            v0, v1 = state[i], next_state[i]
            if v0[VREACHED] or v0[VCRASHED]:
                r = 0.0
            else:
                if v1[VCRASHED]:
                    base = R_CRASH_VEHICLE
                elif v1[VREACHED]:
                    base = R_DESTINATION_REACHED
                else:
                    base = 0.0
                progress = v0[VMIN] - v1[VMIN]
                r = base + (R_PROGRESS_TOTAL * progress) / v0[VINIT]
            rewards[aid] = r
            terms[aid] = bool(v1[VREACHED] or v1[VCRASHED])
            truncs[aid] = False
            obs[aid] = self._obs(next_state, i)
        all_done = all(terms.values())
        return JointTimestep(next_state, obs, rewards, terms, truncs, all_done, {})


def pack_state(state, t) -> tuple:
    """Particle record as the GPU stores it: (t, v0, v1) u32 words."""
    return (t, pack_vehicle(state[0]), pack_vehicle(state[1]))
