// Driving-v1 generative model (host + device), the build's restatement.
//
// posggym's Driving-v1 source is not available (posggym[agents]>=0.5.0,
// /root/reference/pyproject.toml:36, unpinned); the dynamics are the build's
// documented restatement (DESIGN.md "Driving-v1"), identical to
// oracle/driving.py.  Called by the reference planner at mcts.py:181,191-198
// (initial belief), mcts.py:333 (tree step), mcts.py:418 (rollout step) and
// belief.py:165 (reinvigoration).
//
// State: one packed u32 per vehicle
//   x:4 | y:4 | dir:2 | speed:2 | dest:3 | dest_reached:1 | crashed:1 |
//   min_dest_dist:7 | init_dest_dist:7
// Ego observation key (u64, <= 50 bits):
//   cells (2 bits each, window order) | speed<<30 | x<<32 | y<<36 |
//   dest_x<<40 | dest_y<<44 | dest_reached<<48 | crashed<<49
#pragma once
#include <stdint.h>

#include "philox.h"

namespace pb {

enum : int { NORTH = 0, EAST = 1, SOUTH = 2, WEST = 3 };
enum : int { REVERSE = 0, STOPPED = 1, FORWARD_SLOW = 2, FORWARD_FAST = 3 };
enum : int { DO_NOTHING = 0, ACCELERATE = 1, DECELERATE = 2, TURN_RIGHT = 3, TURN_LEFT = 4 };
enum : int { CELL_VEHICLE = 0, CELL_WALL = 1, CELL_EMPTY = 2, CELL_DEST = 3 };

// Grid tables, 16-wide row stride (index = y * 16 + x).  Uploaded by the host
// (built from the grid string in posggym_baselines_amd/envs/driving.py) and
// staged in LDS by every kernel.
struct DrvGrid {
  uint8_t wall[256];       // 1 = wall
  uint8_t dist[8][256];    // BFS distance to location k (127 = unreachable)
  uint8_t loc_x[8], loc_y[8], loc_dir[8];
  int32_t width, height, num_locs;
  int32_t obs_front, obs_back, obs_side;
  int32_t pad[2];
};

struct Veh {
  int x, y, dir, speed, dest, reached, crashed, mind, initd;
};

PB_HD Veh unpack_veh(uint32_t u) {
  Veh v;
  v.x = u & 15;
  v.y = (u >> 4) & 15;
  v.dir = (u >> 8) & 3;
  v.speed = (u >> 10) & 3;
  v.dest = (u >> 12) & 7;
  v.reached = (u >> 15) & 1;
  v.crashed = (u >> 16) & 1;
  v.mind = (u >> 17) & 127;
  v.initd = (u >> 24) & 127;
  return v;
}

PB_HD uint32_t pack_veh(const Veh& v) {
  return (uint32_t)v.x | ((uint32_t)v.y << 4) | ((uint32_t)v.dir << 8) |
         ((uint32_t)v.speed << 10) | ((uint32_t)v.dest << 12) | ((uint32_t)v.reached << 15) |
         ((uint32_t)v.crashed << 16) | ((uint32_t)v.mind << 17) | ((uint32_t)v.initd << 24);
}

PB_HD int dir_dx(int d) { return d == EAST ? 1 : (d == WEST ? -1 : 0); }
PB_HD int dir_dy(int d) { return d == SOUTH ? 1 : (d == NORTH ? -1 : 0); }

template <class G>
PB_HD bool grid_free(const G& g, int x, int y) {
  return x >= 0 && y >= 0 && x < g.width && y < g.height && !g.wall[(y << 4) | x];
}

PB_HD bool veh_done(uint32_t u) { return ((u >> 15) & 3) != 0; }

// One vehicle's move (exec order handled by the caller).  `other` is the
// other vehicle's CURRENT packed state (moved already or not).  Returns the
// new packed state of `self`; sets *hit when it drove into `other`.
template <class G>
PB_HD uint32_t move_vehicle(const G& g, uint32_t self, uint32_t other, int action, bool* hit) {
  *hit = false;
  Veh v = unpack_veh(self);
  if (v.reached || v.crashed) return self;
  int d = v.dir, speed = v.speed;
  if (action == TURN_RIGHT) d = (d + 1) & 3;
  else if (action == TURN_LEFT) d = (d + 3) & 3;
  else if (action == ACCELERATE) speed = speed + 1 < FORWARD_FAST ? speed + 1 : FORWARD_FAST;
  else if (action == DECELERATE) speed = speed - 1 > REVERSE ? speed - 1 : REVERSE;
  const int move = speed != REVERSE ? d : ((d + 2) & 3);
  const int cells = speed > STOPPED ? speed - STOPPED : STOPPED - speed;
  const int ox = other & 15, oy = (other >> 4) & 15;
  int x = v.x, y = v.y;
  for (int k = 0; k < cells; ++k) {
    const int nx = x + dir_dx(move), ny = y + dir_dy(move);
    if (!grid_free(g, nx, ny)) {
      speed = STOPPED;
      break;
    }
    if (nx == ox && ny == oy) {
      *hit = true;
      speed = STOPPED;
      break;
    }
    x = nx;
    y = ny;
  }
  const int dist = g.dist[v.dest][(y << 4) | x];
  Veh n;
  n.x = x;
  n.y = y;
  n.dir = d;
  n.speed = speed;
  n.dest = v.dest;
  n.reached = dist == 0 ? 1 : 0;
  n.crashed = *hit ? 1 : 0;
  n.mind = v.mind < dist ? v.mind : dist;
  n.initd = v.initd;
  return pack_veh(n);
}

// Joint step for 2 agents.  `j` is the model-stream draw of Python's
// random.shuffle([0, 1]) (j == 0 swaps -> agent 1 moves first).
template <class G>
PB_HD void drv_step2(const G& g, uint32_t s0, uint32_t s1, int a0, int a1, uint32_t j,
                     uint32_t* o0, uint32_t* o1) {
  uint32_t v[2] = {s0, s1};
  const int act[2] = {a0, a1};
  const int first = j == 0 ? 1 : 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = k == 0 ? first : 1 - first;
    const int oth = 1 - idx;
    if (veh_done(v[idx])) continue;
    bool hit;
    v[idx] = move_vehicle(g, v[idx], v[oth], act[idx], &hit);
    if (hit && !veh_done(v[oth])) v[oth] |= (1u << 16);
  }
  *o0 = v[0];
  *o1 = v[1];
}

// Reward of one agent for the transition prev -> next.
PB_HD double drv_reward(uint32_t prev, uint32_t next) {
  if (veh_done(prev)) return 0.0;
  const Veh a = unpack_veh(prev), b = unpack_veh(next);
  const double base = b.crashed ? -1.0 : (b.reached ? 0.5 : 0.0);
  const int progress = a.mind - b.mind;
  return base + (0.5 * (double)progress) / (double)a.initd;
}

// Observation cell `c` (window order: farthest-front row first, left to right)
// of vehicle `self` given the other vehicle.
template <class G>
PB_HD int obs_cell(const G& g, uint32_t self, uint32_t other, int c) {
  const int W = 2 * g.obs_side + 1;
  const int fwd = g.obs_front - c / W;
  const int side = c % W - g.obs_side;
  const int x = self & 15, y = (self >> 4) & 15, d = (self >> 8) & 3;
  const int r = (d + 1) & 3;
  const int cx = x + fwd * dir_dx(d) + side * dir_dx(r);
  const int cy = y + fwd * dir_dy(d) + side * dir_dy(r);
  if (!grid_free(g, cx, cy)) return CELL_WALL;
  if ((int)(other & 15) == cx && (int)((other >> 4) & 15) == cy) return CELL_VEHICLE;
  const int dest = (self >> 12) & 7;
  if (g.loc_x[dest] == cx && g.loc_y[dest] == cy) return CELL_DEST;
  return CELL_EMPTY;
}

template <class G>
PB_HD uint64_t obs_tail(const G& g, uint32_t self) {
  const Veh v = unpack_veh(self);
  return ((uint64_t)v.speed << 30) | ((uint64_t)v.x << 32) | ((uint64_t)v.y << 36) |
         ((uint64_t)g.loc_x[v.dest] << 40) | ((uint64_t)g.loc_y[v.dest] << 44) |
         ((uint64_t)v.reached << 48) | ((uint64_t)v.crashed << 49);
}

// Serial (one-thread) observation key.
template <class G>
PB_HD uint64_t obs_key_serial(const G& g, uint32_t self, uint32_t other) {
  const int n = (g.obs_front + g.obs_back + 1) * (2 * g.obs_side + 1);
  uint64_t key = 0;
  for (int c = 0; c < n; ++c) key |= (uint64_t)obs_cell(g, self, other, c) << (2 * c);
  return key | obs_tail(g, self);
}

template <class G>
PB_HD uint32_t make_vehicle(const G& g, int loc, int dest) {
  Veh v;
  v.x = g.loc_x[loc];
  v.y = g.loc_y[loc];
  v.dir = g.loc_dir[loc];
  v.speed = STOPPED;
  v.dest = dest;
  v.reached = 0;
  v.crashed = 0;
  v.mind = g.dist[dest][(v.y << 4) | v.x];
  v.initd = v.mind;
  return pack_veh(v);
}

// k-th set bit (k < popcount(mask)) of an 8-bit mask.
PB_HD int kth_bit(uint32_t mask, uint32_t k) {
  for (int i = 0; i < 8; ++i) {
    if (mask & (1u << i)) {
      if (k == 0) return i;
      --k;
    }
  }
  return -1;
}

PB_HD int popc8(uint32_t m) {
  int n = 0;
  for (int i = 0; i < 8; ++i) n += (m >> i) & 1;
  return n;
}

// sample_initial_state for 2 agents; `draw(n)` returns a model-stream int.
template <class G, class Draw>
PB_HD void drv_sample_initial_state2(const G& g, Draw draw, uint32_t* s0, uint32_t* s1) {
  const uint32_t all = (1u << g.num_locs) - 1u;
  uint32_t starts = 0, dests = 0;
  uint32_t out[2];
  for (int i = 0; i < 2; ++i) {
    const uint32_t av = all & ~starts;
    const int s = kth_bit(av, draw((uint32_t)popc8(av)));
    starts |= 1u << s;
    const uint32_t avd = all & ~dests & ~(1u << s);
    const int d = kth_bit(avd, draw((uint32_t)popc8(avd)));
    dests |= 1u << d;
    out[i] = make_vehicle(g, s, d);
  }
  *s0 = out[0];
  *s1 = out[1];
}

template <class G>
PB_HD int loc_index(const G& g, int x, int y) {
  for (int k = 0; k < g.num_locs; ++k)
    if (g.loc_x[k] == x && g.loc_y[k] == y) return k;
  return -1;
}

}  // namespace pb

namespace pb {

// ---------------------------------------------------------------------------
// Table-driven fast path (identical results to the functions above; the CPU
// tests compare the host build of these against oracle/driving.py and the GPU
// tests the device build against the reference goldens).
//   nbr2[cell * 4 + dir]     : low byte = next free cell in dir (or 0xFF), high
//                              byte = the cell after it (or 0xFF)
//   win_wall[cell * 4 + dir] : bit c set when window cell c is a wall / outside
//   prog[k * 128 + initd]    : (0.5 * k) / initd for progress k = 1, 2 (k = 0 -> 0.0)
struct DrvModel {
  DrvGrid g;
  uint16_t win_wall[1024];
  uint16_t nbr2[1024];
  double prog[3 * 128];
};

template <class G>
PB_HD void build_model_tables(const G& g, DrvModel* m) {
  const int ncells = (g.obs_front + g.obs_back + 1) * (2 * g.obs_side + 1);
  for (int cell = 0; cell < 256; ++cell) {
    const int x = cell & 15, y = cell >> 4;
    for (int d = 0; d < 4; ++d) {
      const int nx = x + dir_dx(d), ny = y + dir_dy(d);
      int n1 = 0xFF, n2 = 0xFF;
      if (grid_free(g, nx, ny)) {
        n1 = (ny << 4) | nx;
        const int mx = nx + dir_dx(d), my = ny + dir_dy(d);
        if (grid_free(g, mx, my)) n2 = (my << 4) | mx;
      }
      m->nbr2[cell * 4 + d] = (uint16_t)(n1 | (n2 << 8));
      uint32_t w = 0;
      const int W = 2 * g.obs_side + 1;
      const int r = (d + 1) & 3;
      for (int c = 0; c < ncells; ++c) {
        const int fwd = g.obs_front - c / W;
        const int side = c % W - g.obs_side;
        const int cx = x + fwd * dir_dx(d) + side * dir_dx(r);
        const int cy = y + fwd * dir_dy(d) + side * dir_dy(r);
        if (!grid_free(g, cx, cy)) w |= 1u << c;
      }
      m->win_wall[cell * 4 + d] = (uint16_t)w;
    }
  }
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < 128; ++i)
      m->prog[k * 128 + i] = i == 0 ? 0.0 : (0.5 * (double)k) / (double)i;
}

// Window index of absolute cell (tx, ty) seen from (x, y) facing d, or -1.
PB_HD int window_index(const DrvGrid& g, int x, int y, int d, int tx, int ty) {
  const int rx = tx - x, ry = ty - y;
  const int r = (d + 1) & 3;
  const int fwd = rx * dir_dx(d) + ry * dir_dy(d);
  const int side = rx * dir_dx(r) + ry * dir_dy(r);
  if (fwd < -g.obs_back || fwd > g.obs_front || side < -g.obs_side || side > g.obs_side) return -1;
  return (g.obs_front - fwd) * (2 * g.obs_side + 1) + (side + g.obs_side);
}

PB_HD uint32_t spread_bits16(uint32_t x) {
  x &= 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}

// Ego observation key without per-cell work: walls from the window table,
// then the destination cell (11) and the other vehicle (00) patched in.
PB_HD uint64_t obs_key_fast(const DrvModel& m, uint32_t self, uint32_t other) {
  const DrvGrid& g = m.g;
  const int ncells = (g.obs_front + g.obs_back + 1) * (2 * g.obs_side + 1);
  const uint32_t full = (1u << ncells) - 1u;
  const int x = self & 15, y = (self >> 4) & 15, d = (self >> 8) & 3;
  const uint32_t wall = m.win_wall[(((y << 4) | x) << 2) | d];
  uint32_t cells = spread_bits16(wall) | (spread_bits16(~wall & full) << 1);
  const int dest = (self >> 12) & 7;
  const int cd = window_index(g, x, y, d, g.loc_x[dest], g.loc_y[dest]);
  if (cd >= 0 && !((wall >> cd) & 1u)) cells |= 3u << (2 * cd);
  const int cv = window_index(g, x, y, d, (int)(other & 15), (int)((other >> 4) & 15));
  if (cv >= 0 && !((wall >> cv) & 1u)) cells &= ~(3u << (2 * cv));
  return (uint64_t)cells | obs_tail(g, self);
}

// A vehicle's intended move before collision resolution.
struct MovePlan {
  uint32_t self;   // packed state before the move
  int d, speed, cells;
  uint32_t path;   // nbr2 entry along the move direction
  bool done;
};

PB_HD MovePlan plan_move(const DrvModel& m, uint32_t self, int action) {
  MovePlan p;
  p.self = self;
  p.done = veh_done(self);
  int d = (self >> 8) & 3, speed = (self >> 10) & 3;
  if (action == TURN_RIGHT) d = (d + 1) & 3;
  else if (action == TURN_LEFT) d = (d + 3) & 3;
  else if (action == ACCELERATE) speed = speed + 1 < FORWARD_FAST ? speed + 1 : FORWARD_FAST;
  else if (action == DECELERATE) speed = speed - 1 > REVERSE ? speed - 1 : REVERSE;
  const int move = speed != REVERSE ? d : ((d + 2) & 3);
  p.d = d;
  p.speed = speed;
  p.cells = speed > STOPPED ? speed - STOPPED : STOPPED - speed;
  p.path = m.nbr2[((self & 0xFF) << 2) | (uint32_t)move];
  return p;
}

// Resolve a planned move against the other vehicle's current cell; returns the
// final cell, updates *speed and *hit.
PB_HD int resolve_move(const MovePlan& p, int ocell, int* speed, bool* hit) {
  int cell = (int)(p.self & 0xFF);
  *speed = p.speed;
  *hit = false;
  if (p.cells >= 1) {
    const int c1 = (int)(p.path & 0xFF);
    if (c1 == 0xFF) {
      *speed = STOPPED;
    } else if (c1 == ocell) {
      *hit = true;
      *speed = STOPPED;
    } else {
      cell = c1;
      if (p.cells >= 2) {
        const int c2 = (int)(p.path >> 8);
        if (c2 == 0xFF) {
          *speed = STOPPED;
        } else if (c2 == ocell) {
          *hit = true;
          *speed = STOPPED;
        } else {
          cell = c2;
        }
      }
    }
  }
  return cell;
}

PB_HD uint32_t finish_move(const DrvModel& m, const MovePlan& p, int cell, int speed, bool hit) {
  const uint32_t self = p.self;
  const int dest = (self >> 12) & 7;
  const int dist = m.g.dist[dest][cell];
  const int mind0 = (self >> 17) & 127;
  const int mind = mind0 < dist ? mind0 : dist;
  return (self & 0x7F007000u) | (uint32_t)cell | ((uint32_t)p.d << 8) | ((uint32_t)speed << 10) |
         ((uint32_t)(dist == 0) << 15) | ((uint32_t)hit << 16) | ((uint32_t)mind << 17);
}

// Joint step for 2 agents (same semantics as drv_step2): both plans (one table
// read each) first, then collisions in execution order.
PB_HD void drv_step2_fast(const DrvModel& m, uint32_t s0, uint32_t s1, int a0, int a1, uint32_t j,
                          uint32_t* o0, uint32_t* o1) {
  const MovePlan p0 = plan_move(m, s0, a0);
  const MovePlan p1 = plan_move(m, s1, a1);
  const bool first1 = j == 0;   // shuffle swapped: agent 1 moves first
  const MovePlan& pf = first1 ? p1 : p0;
  const MovePlan& ps = first1 ? p0 : p1;
  uint32_t vf = pf.self, vs = ps.self;
  int cf = (int)(vf & 0xFF), cs = (int)(vs & 0xFF);
  int spf = 0, sps = 0;
  bool hf = false, hs = false, sec_crashed = false, fst_crashed = false;
  bool movedf = false, moveds = false;
  if (!pf.done) {
    cf = resolve_move(pf, cs, &spf, &hf);
    movedf = true;
    if (hf && !ps.done) sec_crashed = true;
  }
  if (!ps.done && !sec_crashed) {
    cs = resolve_move(ps, cf, &sps, &hs);
    moveds = true;
    if (hs) fst_crashed = true;   // the first mover is hit (it may be done: no effect then)
  }
  if (movedf) vf = finish_move(m, pf, cf, spf, hf);
  if (moveds) vs = finish_move(m, ps, cs, sps, hs);
  if (sec_crashed) vs |= 1u << 16;
  if (fst_crashed && !veh_done(vf)) vf |= 1u << 16;
  *o0 = first1 ? vs : vf;
  *o1 = first1 ? vf : vs;
}

// Ego reward for prev -> next (drv_reward), the division from the table.
PB_HD double drv_reward_fast(const DrvModel& m, uint32_t prev, uint32_t next) {
  if (veh_done(prev)) return 0.0;
  const double base = ((next >> 16) & 1) ? -1.0 : (((next >> 15) & 1) ? 0.5 : 0.0);
  const int progress = (int)((prev >> 17) & 127) - (int)((next >> 17) & 127);
  return base + m.prog[progress * 128 + (int)((prev >> 24) & 127)];
}

}  // namespace pb
