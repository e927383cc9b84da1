// PursuitEvasion-v1 generative model (host + device), the build's restatement.
//
// posggym's PursuitEvasion-v1 source is not available (posggym[agents]>=0.5.0,
// /root/reference/pyproject.toml:36, unpinned); the dynamics restate
// oracle/pursuit_evasion.py exactly (DESIGN.md "PursuitEvasion-v1"; parity
// with posggym unpinned, reward lattice pinned by the reference's own
// baseline_exps/env_data/PursuitEvasion-v1_i0 returns).  Called by the
// reference planner at the same sites as Driving-v1 (mcts.py:181,191-198,333,
// 418; belief.py:165).
//
// Agents: 0 evader, 1 pursuer.  Cells are (y << 4) | x (16-wide stride).
// State words:
//   v0 (evader) : cell:8 | dir:2 | start:2 | goal:2 | min_goal_dist:7 | caught:1 | reached:1
//   v1 (pursuer): cell:8 | dir:2 | start:2
// Observation key (30 bits): walls:4 | seen:1 | heard:1 | x:4 | y:4 | c1x:4 |
//   c1y:4 | c2x:4 | c2y:4 with (c1, c2) = (own start, goal) for the evader and
//   (own start, evader start) for the pursuer.
// The step is deterministic: no model-stream draw.
#pragma once
#include <stdint.h>

#include "philox.h"

namespace pb {

constexpr int kPeMaxStarts = 4;
constexpr int kPeMaxGoals = 4;
constexpr int kPeHearing = 2;

// Device tables (staged in LDS by every kernel).
struct PeModel {
  uint8_t next[256][4];        // cell after turning to heading d and moving (itself if blocked)
  uint16_t lanes[256][4];      // free length (<= max_obs_distance) of lanes -1, 0, +1: 4 bits each
  uint8_t goal_dist[kPeMaxGoals][256];
  uint8_t wallbits[256];       // bit d: the neighbour in heading d is blocked
  uint8_t estart[kPeMaxStarts], pstart[kPeMaxStarts], goal[kPeMaxGoals];
  int32_t n_estart, n_pstart, n_goal, pad;
  double rew[2][2][3];         // [agent][progress][outcome: none, caught, reached]
};

PB_HD int pe_dx(int d) { return d == 1 ? 1 : (d == 3 ? -1 : 0); }
PB_HD int pe_dy(int d) { return d == 2 ? 1 : (d == 0 ? -1 : 0); }
PB_HD uint32_t pe_turn(uint32_t a) { return (0x78u >> (2u * a)) & 3u; }   // {0, 2, 3, 1}

// Host: tables from the grid description (include/pomcp.h pomcp_pe_grid).
template <class G>
inline void build_pe_model(const G& g, PeModel* m) {
  auto free_ = [&](int x, int y) {
    return x >= 0 && y >= 0 && x < g.width && y < g.height && !g.wall[(y << 4) | x];
  };
  for (int c = 0; c < 256; ++c) {
    const int x = c & 15, y = c >> 4;
    uint32_t wb = 0;
    for (int d = 0; d < 4; ++d) {
      const int nx = x + pe_dx(d), ny = y + pe_dy(d);
      const bool f = free_(nx, ny);
      m->next[c][d] = (uint8_t)(f ? ((ny << 4) | nx) : c);
      if (!f) wb |= 1u << d;
      uint32_t lanes = 0;
      const int r = (d + 1) & 3;
      for (int s = -1; s <= 1; ++s) {
        int n = 0;
        for (int k = 1; k <= g.max_obs_distance; ++k) {
          if (!free_(x + k * pe_dx(d) + s * pe_dx(r), y + k * pe_dy(d) + s * pe_dy(r))) break;
          n = k;
        }
        lanes |= (uint32_t)n << (4 * (s + 1));
      }
      m->lanes[c][d] = (uint16_t)lanes;
    }
    m->wallbits[c] = (uint8_t)wb;
  }
  for (int k = 0; k < kPeMaxGoals; ++k)
    for (int c = 0; c < 256; ++c) m->goal_dist[k][c] = k < g.n_goal ? g.goal_dist[k][c] : 127;
  for (int k = 0; k < kPeMaxStarts; ++k) {
    m->estart[k] = k < g.n_evader_start ? (uint8_t)((g.evader_start[k][1] << 4) | g.evader_start[k][0]) : 0;
    m->pstart[k] = k < g.n_pursuer_start ? (uint8_t)((g.pursuer_start[k][1] << 4) | g.pursuer_start[k][0]) : 0;
  }
  for (int k = 0; k < kPeMaxGoals; ++k)
    m->goal[k] = k < g.n_goal ? (uint8_t)((g.goal[k][1] << 4) | g.goal[k][0]) : 0;
  m->n_estart = g.n_evader_start;
  m->n_pstart = g.n_pursuer_start;
  m->n_goal = g.n_goal;
  m->pad = 0;
  // oracle/pursuit_evasion.py _evader_reward, same operation order:
  // r = 0.0; r += 0.01 (progress); r -= / += 1.0 (caught / reached); r / norm;
  // the pursuer's reward is 0.0 - r
  for (int prog = 0; prog < 2; ++prog) {
    for (int o = 0; o < 3; ++o) {
      double r = 0.0;
      if (prog && g.use_progress_reward) r += 0.01;
      if (o == 1) r -= 1.0;
      else if (o == 2) r += 1.0;
      r = r / g.reward_norm;
      m->rew[0][prog][o] = r;
      m->rew[1][prog][o] = 0.0 - r;
    }
  }
}

PB_HD bool pe_done(uint32_t v0) { return ((v0 >> 21) & 3u) != 0u; }

// Joint step; returns the next words and the evader's (progress, outcome).
PB_HD void pe_step(const PeModel& m, uint32_t v0, uint32_t v1, uint32_t ae, uint32_t ap,
                   uint32_t* n0, uint32_t* n1, uint32_t* prog, uint32_t* outcome) {
  const uint32_t ec = v0 & 0xFFu, pc = v1 & 0xFFu;
  const uint32_t ed = (((v0 >> 8) & 3u) + pe_turn(ae)) & 3u;
  const uint32_t pd = (((v1 >> 8) & 3u) + pe_turn(ap)) & 3u;
  const uint32_t ne = m.next[ec][ed], np = m.next[pc][pd];
  const bool caught = ne == np || (ne == pc && np == ec);
  const uint32_t gi = (v0 >> 12) & 3u;
  const bool reached = !caught && ne == m.goal[gi];
  const uint32_t mgd0 = (v0 >> 14) & 127u;
  const uint32_t gd = m.goal_dist[gi][ne];
  const uint32_t mgd = mgd0 < gd ? mgd0 : gd;
  const bool done0 = pe_done(v0);
  const uint32_t w0 = ne | (ed << 8) | (v0 & 0x3C00u) | (mgd << 14) | ((caught ? 1u : 0u) << 21) |
                      ((reached ? 1u : 0u) << 22);
  const uint32_t w1 = np | (pd << 8) | (v1 & 0xC00u);
  *n0 = done0 ? v0 : w0;
  *n1 = done0 ? v1 : w1;
  *prog = (!done0 && mgd < mgd0) ? 1u : 0u;
  *outcome = done0 ? 0u : (caught ? 1u : (reached ? 2u : 0u));
}

// Reward of agent `agent` for a step that started in v0 (absorbing -> 0.0).
PB_HD double pe_reward(const PeModel& m, int agent, uint32_t v0, uint32_t prog, uint32_t outcome) {
  return pe_done(v0) ? 0.0 : m.rew[agent][prog][outcome];
}

PB_HD uint64_t pe_obs_key(const PeModel& m, int agent, uint32_t v0, uint32_t v1) {
  const uint32_t me = agent == 0 ? v0 : v1, ot = agent == 0 ? v1 : v0;
  const uint32_t cell = me & 0xFFu;
  const int x = (int)(cell & 15u), y = (int)(cell >> 4), d = (int)((me >> 8) & 3u);
  const int ox = (int)(ot & 15u), oy = (int)((ot >> 4) & 15u);
  const int dx = ox - x, dy = oy - y;
  const int r = (d + 1) & 3;
  const int fwd = dx * pe_dx(d) + dy * pe_dy(d);
  const int side = dx * pe_dx(r) + dy * pe_dy(r);
  const bool in_lane = side >= -1 && side <= 1;
  const int L = (int)((m.lanes[cell][d] >> (4 * ((in_lane ? side : 0) + 1))) & 15u);
  const uint32_t seen = (in_lane && fwd >= 1 && fwd <= L) ? 1u : 0u;
  const int man = (dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy);
  const uint32_t heard = (man > 0 && man <= kPeHearing) ? 1u : 0u;
  uint32_t c1, c2;
  if (agent == 0) {
    c1 = m.estart[(v0 >> 10) & 3u];
    c2 = m.goal[(v0 >> 12) & 3u];
  } else {
    c1 = m.pstart[(v1 >> 10) & 3u];
    c2 = m.estart[(v0 >> 10) & 3u];
  }
  return (uint64_t)(m.wallbits[cell] | (seen << 4) | (heard << 5) | ((uint32_t)x << 6) |
                    ((uint32_t)y << 10) | ((c1 & 15u) << 14) | ((c1 >> 4) << 18) |
                    ((c2 & 15u) << 22) | ((c2 >> 4) << 26));
}

PB_HD uint32_t pe_make_evader(const PeModel& m, uint32_t es, uint32_t gi, uint32_t d) {
  const uint32_t c = m.estart[es];
  return c | (d << 8) | (es << 10) | (gi << 12) | ((uint32_t)m.goal_dist[gi][c] << 14);
}

PB_HD uint32_t pe_make_pursuer(const PeModel& m, uint32_t ps, uint32_t d) {
  return (uint32_t)m.pstart[ps] | (d << 8) | (ps << 10);
}

// sample_initial_state: evader start, pursuer start, goal, evader heading,
// pursuer heading (model stream, in this order).
template <class Draw>
PB_HD void pe_sample_initial_state(const PeModel& m, Draw draw, uint32_t* v0, uint32_t* v1) {
  const uint32_t es = draw((uint32_t)m.n_estart);
  const uint32_t ps = draw((uint32_t)m.n_pstart);
  const uint32_t gi = draw((uint32_t)m.n_goal);
  const uint32_t ed = draw(4u);
  const uint32_t pd = draw(4u);
  *v0 = pe_make_evader(m, es, gi, ed);
  *v1 = pe_make_pursuer(m, ps, pd);
}

PB_HD int pe_index_of(const uint8_t* cells, int n, uint32_t cell) {
  int k = -1;
  for (int i = n - 1; i >= 0; --i)
    if (cells[i] == cell) k = i;
  return k;
}

// sample_agent_initial_state (oracle/pursuit_evasion.py): the ego's known
// indices from its obs, the unknowns drawn and rejected until the obs matches
// (<= 64 tries, then the last draw).  false: the obs names no start / goal.
template <class Draw>
PB_HD bool pe_sample_agent_initial(const PeModel& m, int agent, uint64_t obs, Draw draw,
                                   uint32_t* v0, uint32_t* v1) {
  const uint32_t own = (uint32_t)(((obs >> 6) & 15u) | (((obs >> 10) & 15u) << 4));
  const uint32_t c2 = (uint32_t)(((obs >> 22) & 15u) | (((obs >> 26) & 15u) << 4));
  uint32_t es = 0, ps = 0, gi = 0;
  if (agent == 0) {
    const int e = pe_index_of(m.estart, m.n_estart, own), g = pe_index_of(m.goal, m.n_goal, c2);
    if (e < 0 || g < 0) return false;
    es = (uint32_t)e;
    gi = (uint32_t)g;
  } else {
    const int p = pe_index_of(m.pstart, m.n_pstart, own), e = pe_index_of(m.estart, m.n_estart, c2);
    if (p < 0 || e < 0) return false;
    ps = (uint32_t)p;
    es = (uint32_t)e;
  }
  for (int tr = 0; tr < 64; ++tr) {
    uint32_t ed, pd;
    if (agent == 0) {
      ed = draw(4u);
      ps = draw((uint32_t)m.n_pstart);
      pd = draw(4u);
    } else {
      gi = draw((uint32_t)m.n_goal);
      ed = draw(4u);
      pd = draw(4u);
    }
    *v0 = pe_make_evader(m, es, gi, ed);
    *v1 = pe_make_pursuer(m, ps, pd);
    if (pe_obs_key(m, agent, *v0, *v1) == obs) break;
  }
  return true;
}

}  // namespace pb
