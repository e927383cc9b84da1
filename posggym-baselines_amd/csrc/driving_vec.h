// Driving-v1 step / reward / observation key on the VECTOR ALU (device only).
//
// Same results as the table-driven scalar functions in driving.h (and hence as
// oracle/driving.py); written branch-free with selects so every lane of the
// wave evaluates the identical values in VGPRs.  Why: one CU has one scalar
// ALU shared by its 4 SIMDs but 4 vector ALUs; with every tree's serial logic
// on SALU the scalar unit saturated first.  `vary()` hides the
// wave-uniformity of a value from the compiler so that it stays in a VGPR and
// the arithmetic on it is issued as VALU instead of being scalarised.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "driving.h"

namespace pb {

__device__ __forceinline__ uint32_t vary(uint32_t x) {
  uint32_t r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

struct VPlan {
  uint32_t self, path;
  uint32_t d, speed, cells, done;
};

__device__ __forceinline__ VPlan vplan(const DrvModel& m, uint32_t self, uint32_t act) {
  VPlan p;
  p.self = self;
  p.done = ((self >> 15) & 3u) != 0u;
  const uint32_t d0 = (self >> 8) & 3u, s0 = (self >> 10) & 3u;
  const uint32_t d = act == (uint32_t)TURN_RIGHT ? ((d0 + 1u) & 3u)
                     : act == (uint32_t)TURN_LEFT ? ((d0 + 3u) & 3u) : d0;
  const uint32_t sp = act == (uint32_t)ACCELERATE ? (s0 < 3u ? s0 + 1u : 3u)
                      : act == (uint32_t)DECELERATE ? (s0 > 0u ? s0 - 1u : 0u) : s0;
  const uint32_t move = sp != 0u ? d : ((d + 2u) & 3u);
  p.d = d;
  p.speed = sp;
  p.cells = sp == 0u ? 1u : sp - 1u;   // |speed - STOPPED|
  p.path = m.nbr2[((self & 0xFFu) << 2) | move];
  return p;
}

struct VMove {
  uint32_t cell, speed, hit;
};

// Cells traversed until a wall or the other vehicle (cell `ocell`).
__device__ __forceinline__ VMove vresolve(const VPlan& p, uint32_t ocell) {
  const uint32_t c1 = p.path & 0xFFu, c2 = p.path >> 8;
  const uint32_t start = p.self & 0xFFu;
  const bool s1 = p.cells >= 1u;
  const bool w1 = c1 == 0xFFu, h1 = !w1 && c1 == ocell;
  const bool a1 = s1 && !w1 && !h1;
  const bool s2 = p.cells >= 2u && a1;
  const bool w2 = c2 == 0xFFu, h2 = !w2 && c2 == ocell;
  const bool a2 = s2 && !w2 && !h2;
  VMove r;
  r.cell = a2 ? c2 : (a1 ? c1 : start);
  r.hit = ((s1 && h1) || (s2 && h2)) ? 1u : 0u;
  r.speed = ((s1 && (w1 || h1)) || (s2 && (w2 || h2))) ? (uint32_t)STOPPED : p.speed;
  return r;
}

__device__ __forceinline__ uint32_t vfinish(const DrvModel& m, const VPlan& p, const VMove& mv) {
  const uint32_t dest = (p.self >> 12) & 7u;
  const uint32_t dist = m.g.dist[dest][mv.cell];
  const uint32_t mind0 = (p.self >> 17) & 127u;
  const uint32_t mind = mind0 < dist ? mind0 : dist;
  return (p.self & 0x7F007000u) | mv.cell | (p.d << 8) | (mv.speed << 10) |
         ((dist == 0u ? 1u : 0u) << 15) | (mv.hit << 16) | (mind << 17);
}

// Joint step (drv_step2 semantics).  j: the model-stream draw of the shuffle.
__device__ __forceinline__ void drv_step2_vec(const DrvModel& m, uint32_t s0, uint32_t s1,
                                              uint32_t a0, uint32_t a1, uint32_t j, uint32_t* o0,
                                              uint32_t* o1) {
  const VPlan q0 = vplan(m, s0, a0), q1 = vplan(m, s1, a1);
  const bool first1 = j == 0u;   // shuffle swapped: agent 1 moves first
  VPlan pf, ps;
  pf.self = first1 ? q1.self : q0.self;
  pf.path = first1 ? q1.path : q0.path;
  pf.d = first1 ? q1.d : q0.d;
  pf.speed = first1 ? q1.speed : q0.speed;
  pf.cells = first1 ? q1.cells : q0.cells;
  pf.done = first1 ? q1.done : q0.done;
  ps.self = first1 ? q0.self : q1.self;
  ps.path = first1 ? q0.path : q1.path;
  ps.d = first1 ? q0.d : q1.d;
  ps.speed = first1 ? q0.speed : q1.speed;
  ps.cells = first1 ? q0.cells : q1.cells;
  ps.done = first1 ? q0.done : q1.done;
  // first mover against the second's current cell
  const VMove mf = vresolve(pf, ps.self & 0xFFu);
  const bool movef = !pf.done;
  const bool sec_crash = movef && mf.hit && !ps.done;
  const uint32_t cellf = movef ? mf.cell : (pf.self & 0xFFu);
  // second mover against the first's new cell
  const VMove ms = vresolve(ps, cellf);
  const bool moves = !ps.done && !sec_crash;
  uint32_t vf = movef ? vfinish(m, pf, mf) : pf.self;
  uint32_t vs = moves ? vfinish(m, ps, ms) : ps.self;
  vs |= sec_crash ? (1u << 16) : 0u;
  const bool fst_crash = moves && ms.hit && ((vf >> 15) & 3u) == 0u;
  vf |= fst_crash ? (1u << 16) : 0u;
  *o0 = first1 ? vs : vf;
  *o1 = first1 ? vf : vs;
}

__device__ __forceinline__ double drv_reward_vec(const DrvModel& m, uint32_t prev, uint32_t next) {
  const bool done0 = ((prev >> 15) & 3u) != 0u;
  const double base = ((next >> 16) & 1u) ? -1.0 : (((next >> 15) & 1u) ? 0.5 : 0.0);
  const uint32_t progress = ((prev >> 17) & 127u) - ((next >> 17) & 127u);
  const double r = base + m.prog[progress * 128u + ((prev >> 24) & 127u)];
  return done0 ? 0.0 : r;
}

__device__ __forceinline__ int vwindow_index(const DrvGrid& g, int x, int y, int fx, int fy, int rx,
                                             int ry, int tx, int ty) {
  const int dx = tx - x, dy = ty - y;
  const int fwd = dx * fx + dy * fy;
  const int side = dx * rx + dy * ry;
  const bool in = fwd >= -g.obs_back && fwd <= g.obs_front && side >= -g.obs_side &&
                  side <= g.obs_side;
  return in ? (g.obs_front - fwd) * (2 * g.obs_side + 1) + (side + g.obs_side) : -1;
}

__device__ __forceinline__ uint64_t obs_key_vec(const DrvModel& m, uint32_t self, uint32_t other) {
  const DrvGrid& g = m.g;
  const int ncells = (g.obs_front + g.obs_back + 1) * (2 * g.obs_side + 1);
  const uint32_t full = (1u << ncells) - 1u;
  const int x = (int)(self & 15u), y = (int)((self >> 4) & 15u), d = (int)((self >> 8) & 3u);
  const uint32_t wall = m.win_wall[(self & 0xFFu) << 2 | (uint32_t)d];
  uint32_t cells = spread_bits16(wall) | (spread_bits16(~wall & full) << 1);
  const int fx = d == EAST ? 1 : (d == WEST ? -1 : 0);
  const int fy = d == SOUTH ? 1 : (d == NORTH ? -1 : 0);
  const int rx = -fy, ry = fx;   // right of heading d = heading d + 1
  const uint32_t dest = (self >> 12) & 7u;
  const int dxl = g.loc_x[dest], dyl = g.loc_y[dest];
  const int cd = vwindow_index(g, x, y, fx, fy, rx, ry, dxl, dyl);
  const uint32_t dmask = (cd >= 0 && !((wall >> (cd & 31)) & 1u)) ? (3u << (2 * (cd & 15))) : 0u;
  cells |= dmask;
  const int cv = vwindow_index(g, x, y, fx, fy, rx, ry, (int)(other & 15u), (int)((other >> 4) & 15u));
  const uint32_t vmask = (cv >= 0 && !((wall >> (cv & 31)) & 1u)) ? (3u << (2 * (cv & 15))) : 0u;
  cells &= ~vmask;
  const uint64_t tail = ((uint64_t)((self >> 10) & 3u) << 30) | ((uint64_t)x << 32) |
                        ((uint64_t)y << 36) | ((uint64_t)dxl << 40) | ((uint64_t)dyl << 44) |
                        ((uint64_t)((self >> 15) & 1u) << 48) | ((uint64_t)((self >> 16) & 1u) << 49);
  return (uint64_t)cells | tail;
}

}  // namespace pb
