// POMCP per-simulation loop as hand-written HIP kernels for gfx950 (CDNA4).
//
// Replaces posggym_baselines/planning/mcts.py:269-452 (get_action, _simulate,
// _rollout, UCB/PUCB/min-visit selection, final action choice),
// node.py (ObsNode/ActionNode -> SoA arena), belief.py (ParticleBelief ->
// particle log + root belief buffer, BeliefRejectionSampler -> k_update) and
// utils.py:15-42 (MinMaxStats -> two registers).  One wavefront per tree.
//
// FP64 arithmetic follows the reference's operation order exactly and is built
// with -ffp-contract=off; log(N) and discount**k come from host tables computed
// with Python's own math.log / float.__pow__ (DESIGN.md "bit-exactness").
#pragma clang fp contract(off)

#include "pomcp_device.h"

namespace pb {

__device__ __forceinline__ void stage_grid(const DrvGrid* src, DrvGrid& dst) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(&dst);
  for (int i = threadIdx.x; i < (int)(sizeof(DrvGrid) / 4); i += blockDim.x) d[i] = s[i];
  __syncthreads();
}

// Everything one wave needs about its tree, header fields held in registers.
struct Tree {
  const DevParams& p;
  const DrvGrid& g;
  int tree, lane;
  int2* onode;
  int32_t* ometa;
  ActRec* an;
  uint4* hash;
  uint4* plog;
  uint4* bel;          // 2 * Nr records
  int root, n_obs, n_blocks, n_log, bsize, bsel, epoch, err, root_t, root_abs;
  double mm_min, mm_max;
  Streams rs;
  int64_t c_levels, c_expand, c_new, c_rollout, c_probes;

  __device__ Tree(const DevParams& pp, const DrvGrid& gg, int t) : p(pp), g(gg), tree(t) {
    lane = lane_id();
    onode = p.onode + (int64_t)t * p.No;
    ometa = p.ometa + (int64_t)t * p.No;
    an = p.an + (int64_t)t * p.Nb * p.A;
    hash = reinterpret_cast<uint4*>(p.hash + (int64_t)t * p.H);
    plog = p.plog + (int64_t)t * p.Np;
    bel = p.belief + (int64_t)t * 2 * p.Nr;
    const TreeHdr h = p.hdr[t];
    root = uni(h.root);
    n_obs = uni(h.n_obs);
    n_blocks = uni(h.n_blocks);
    n_log = uni(h.n_log);
    bsize = uni(h.belief_size);
    bsel = uni(h.belief_sel);
    epoch = uni(h.epoch);
    err = uni(h.error);
    root_t = uni(h.root_t);
    root_abs = uni(h.root_abs);
    mm_min = h.mm_min;
    mm_max = h.mm_max;
    rs.seed = h.seed;
    rs.tree = h.tree_key;
#pragma unroll
    for (int k = 0; k < 5; ++k) rs.ctr[k] = (uint32_t)uni((int)h.ctr[k]);
    c_levels = c_expand = c_new = c_rollout = c_probes = 0;
  }

  __device__ void store_header() {
    if (lane != 0) return;
    TreeHdr h;
    h.root = root;
    h.n_obs = n_obs;
    h.n_blocks = n_blocks;
    h.n_log = n_log;
    h.belief_size = bsize;
    h.belief_sel = bsel;
    h.epoch = epoch;
    h.error = err;
    h.root_t = root_t;
    h.root_abs = root_abs;
    h.pad0 = h.pad1 = 0;
    h.mm_min = mm_min;
    h.mm_max = mm_max;
    h.seed = rs.seed;
    h.tree_key = rs.tree;
    for (int k = 0; k < 5; ++k) h.ctr[k] = rs.ctr[k];
    p.hdr[tree] = h;
  }

  __device__ uint4* root_belief() { return bel + (int64_t)bsel * p.Nr; }
  __device__ uint4* other_belief() { return bel + (int64_t)(bsel ^ 1) * p.Nr; }

  // ObsNode(...) (node.py:32-56)
  __device__ int new_obs_node(int t, int visits, int absorbing) {
    if (n_obs >= p.No) {
      err = POMCP_E_ARENA;
      return -1;
    }
    const int i = n_obs++;
    if (lane == 0) {
      onode[i] = make_int2(-1, visits);
      ometa[i] = (t << 1) | absorbing;
    }
    ++c_new;
    return i;
  }

  // ObsNode.add_child for every action (mcts.py:279-281, 318-321).
  __device__ int expand(int node) {
    if (n_blocks >= p.Nb) {
      err = POMCP_E_ARENA;
      return -1;
    }
    const int b = n_blocks++;
    if (lane < p.A) {
      ActRec z;
      z.visits = 0;
      z.pad = 0;
      z.value = 0.0;
      z.total = 0.0;
      z.agg = 0.0;
      an[(int64_t)b * p.A + lane] = z;
    }
    if (lane == 0) onode[node].x = b;
    ++c_expand;
    return b;
  }

  // ActionNode.children[obs] lookup, inserting a new ObsNode when absent.
  __device__ int find_or_insert(uint32_t ani, uint64_t okey, bool insert, int t_child,
                                int visits, int absorbing, bool* is_new) {
    const uint64_t key = okey | ((uint64_t)epoch << kEpochShift);
    uint32_t b = slot_hash(ani, okey) & p.bucket_mask;
    *is_new = false;
    for (uint32_t probe = 0; probe <= p.bucket_mask; ++probe) {
      ++c_probes;
      uint4 s = make_uint4(0, 0, 0, 0);
      if (lane < kBucket) s = hash[(int64_t)b * kBucket + lane];
      const uint64_t skey = (uint64_t)s.x | ((uint64_t)s.y << 32);
      const bool valid = lane < kBucket && (uint32_t)(skey >> kEpochShift) == (uint32_t)epoch;
      const uint64_t m = __ballot(valid && skey == key && s.z == ani);
      if (m) return rl((int)s.w, __ffsll((long long)m) - 1);
      const uint64_t e = __ballot(lane < kBucket && !valid);
      if (e) {
        if (!insert) return -1;
        const int c = new_obs_node(t_child, visits, absorbing);
        if (c < 0) return -1;
        if (lane == __ffsll((long long)e) - 1)
          hash[(int64_t)b * kBucket + lane] =
              make_uint4((uint32_t)key, (uint32_t)(key >> 32), ani, (uint32_t)c);
        *is_new = true;
        return c;
      }
      b = (b + 1) & p.bucket_mask;
    }
    err = POMCP_E_ARENA;
    return -1;
  }

  __device__ void mm_update(double v) {     // utils.py:29-32
    if (v > mm_max) mm_max = v;
    if (v < mm_min) mm_min = v;
  }

  __device__ double normalize(double v) const {   // utils.py:34-39
    if (mm_max > mm_min) return (v - mm_min) / (mm_max - mm_min);
    return v;
  }

  // Joint step with random other agent; returns the packed next state.
  __device__ void joint_step(uint32_t s0, uint32_t s1, int ego_a, int oth_a, uint32_t* n0,
                             uint32_t* n1) {
    const uint32_t j = rs.model(2);   // Python random.shuffle of the exec order
    const int a0 = p.ego == 0 ? ego_a : oth_a;
    const int a1 = p.ego == 0 ? oth_a : ego_a;
    drv_step2(g, s0, s1, a0, a1, j, n0, n1);
  }

  // _search_action_selection (mcts.py:492-563); lanes 0..A-1 score children.
  __device__ int select(int blk, int visits) {
    const int A = p.A;
    // (PUCB with visits == 0 is handled by pucb_prior_draw before this call.)
    if (visits == 0) return (int)rs.select((uint32_t)A);   // mcts.py:532, 555
    const ActRec* rec = an + (int64_t)blk * A;
    int n = 0;
    double v = 0.0;
    if (lane < A) {
      const int4 q = *reinterpret_cast<const int4*>(rec + lane);   // {visits, pad, value}
      n = q.x;
      v = __hiloint2double(q.w, q.z);
    }
    if (p.sel == POMCP_SEL_UNIFORM) {   // min_visit_action_selection
      int min_n = visits + 1, best = 0;
      for (int a = 0; a < A; ++a) {
        const int na = rl(n, a);
        if (na < min_n) {
          min_n = na;
          best = a;
        }
      }
      return best;
    }
    double score = -__builtin_inf();
    if (p.sel == POMCP_SEL_UCB) {
      const uint64_t unv = __ballot(lane < A && n == 0);   // mcts.py:539-540
      if (unv) return __ffsll((long long)unv) - 1;
      if (visits >= p.logtab_n) {
        err = POMCP_E_ARENA;
        return 0;
      }
      const double log_n = p.logtab[visits];
      if (lane < A) score = normalize(v) + p.c * sqrt(log_n / (double)n);   // mcts.py:541-542
    } else {   // PUCB, mcts.py:502-527
      const double noise = 1.0 / (double)A;
      const double prior = (1.0 / (double)A) * (1.0 - p.pucb_f) + p.pucb_f * noise;
      const double sqrt_n = sqrt((double)visits);
      if (lane < A) {
        const double explore = p.c * prior * (sqrt_n / (double)(1 + n));
        score = (n > 0 ? normalize(v) : 0.0) + explore;
      }
    }
    double best_v = -__builtin_inf();
    int best = 0;
    for (int a = 0; a < A; ++a) {   // strict '>' in action order
      const double sa = rl_d(score, a);
      if (sa > best_v) {
        best_v = sa;
        best = a;
      }
    }
    return best;
  }

  // PUCB with N == 0 (mcts.py:494-500): random.choices(actions, weights=prior),
  // cum_weights by itertools.accumulate, bisect(cum, random() * total, 0, A-1).
  __device__ int pucb_prior_draw() {
    const int A = p.A;
    const double w = 1.0 / (double)A;
    double cum[POMCP_MAX_ACTIONS];
    double acc = w;
    cum[0] = acc;
    for (int k = 1; k < A; ++k) {
      acc = acc + w;
      cum[k] = acc;
    }
    const double total = cum[A - 1] + 0.0;
    const double x = rs.select_float() * total;
    for (int k = 0; k < A - 1; ++k)   // bisect_right(cum, x, 0, A-1)
      if (x < cum[k]) return k;
    return A - 1;
  }

  __device__ int choose_action(int blk, int visits) {
    if (p.sel == POMCP_SEL_PUCB && visits == 0) return pucb_prior_draw();
    return select(blk, visits);
  }

  // _final_action_selection (mcts.py:565-600).
  __device__ int final_action(int blk, int visits) {
    const int A = p.A;
    if (p.sel == POMCP_SEL_PUCB) {
      if (visits == 0) return (int)rs.select((uint32_t)A);
      int mx = 0, nt = 0;
      uint32_t ties = 0;
      for (int a = 0; a < A; ++a) {
        const int na = an[(int64_t)blk * A + a].visits;
        if (na == mx) {
          ties |= 1u << a;
          ++nt;
        } else if (na > mx) {
          mx = na;
          ties = 1u << a;
          nt = 1;
        }
      }
      return kth_bit(ties, rs.select((uint32_t)nt));
    }
    if (blk < 0) return (int)rs.select((uint32_t)A);
    double mx = -__builtin_inf();
    int nt = 0;
    uint32_t ties = 0;
    for (int a = 0; a < A; ++a) {
      const double va = an[(int64_t)blk * A + a].value;
      if (va == mx) {
        ties |= 1u << a;
        ++nt;
      } else if (va > mx) {
        mx = va;
        ties = 1u << a;
        nt = 1;
      }
    }
    return kth_bit(ties, rs.select((uint32_t)nt));
  }

  // MCTS._rollout (mcts.py:405-452), random search policy.
  __device__ double rollout(uint32_t s0, uint32_t s1, int t, int depth) {
    double ret = 0.0;
    int k = 0;
    while (depth <= p.depth_limit && t <= p.step_limit) {
      const int ae = (int)rs.act(p.ego, (uint32_t)p.A);     // search_policy.py:177
      const int ao = (int)rs.act(p.other, (uint32_t)p.A);   // other_policy.py:151
      uint32_t n0, n1;
      joint_step(s0, s1, ae, ao, &n0, &n1);
      const uint32_t e0 = p.ego == 0 ? s0 : s1, e1 = p.ego == 0 ? n0 : n1;
      const double r = drv_reward(e0, e1);
      if (k >= p.dpow_n) {
        err = POMCP_E_ARENA;
        break;
      }
      ret += p.dpow[k] * r;   // mcts.py:420-422
      ++c_rollout;
      if (veh_done(e1) || (veh_done(n0) && veh_done(n1))) break;
      s0 = n0;
      s1 = n1;
      ++t;
      ++depth;
      ++k;
    }
    return ret;
  }

  // One simulation from the root (mcts.py:286-290 + _simulate 308-382).
  __device__ int simulate(int root_blk, int root_visits) {
    const uint32_t k = rs.belief((uint32_t)bsize);   // belief.py:55
    const uint4 pr = root_belief()[k];
    int t = (int)pr.x;
    uint32_t s0 = pr.y, s1 = pr.z;
    int node = root, depth = 0, plen = 0;
    int blk = root_blk, nvis = root_visits;
    double leaf = 0.0;
    int p_an = 0, p_done = 0;
    double p_r = 0.0;
    while (true) {
      if (depth > p.depth_limit || t > p.step_limit) break;   // mcts.py:315
      if (blk < 0) {                                            // mcts.py:318-328
        if (expand(node) < 0) return -1;
        leaf = rollout(s0, s1, t, depth);
        break;
      }
      const int a = choose_action(blk, nvis);                  // mcts.py:330
      const int ao = (int)rs.act(p.other, (uint32_t)p.A);      // mcts.py:331
      uint32_t n0, n1;
      joint_step(s0, s1, a, ao, &n0, &n1);                     // mcts.py:333
      const uint32_t e0 = p.ego == 0 ? s0 : s1;
      const uint32_t e1 = p.ego == 0 ? n0 : n1;
      const uint32_t o1 = p.ego == 0 ? n1 : n0;
      const double r = drv_reward(e0, e1);
      const int done = (veh_done(e1) || (veh_done(n0) && veh_done(n1))) ? 1 : 0;
      const uint64_t okey = obs_key_wave(g, e1, o1, p.ncells);
      const uint32_t ani = (uint32_t)(blk * p.A + a);
      bool is_new;
      const int child = find_or_insert(ani, okey, true, t + 1, 1, done, &is_new);
      if (child < 0) return -1;
      int cvis = 1, cblk = -1;
      if (!is_new) {                                            // mcts.py:358-367
        const int2 cn = onode[child];
        cvis = cn.y + 1;
        cblk = cn.x;
        if (lane == 0) {
          onode[child].y = cvis;
          ometa[child] = ((t + 1) << 1) | done;                 // mcts.py:370
        }
      }
      if (n_log >= p.Np) {
        err = POMCP_E_ARENA;
        return -1;
      }
      if (lane == 0) plog[n_log] = make_uint4((uint32_t)child, (uint32_t)(t + 1), n0, n1);
      ++n_log;                                                  // mcts.py:371
      if (lane == plen) {
        p_an = (int)ani;
        p_r = r;
        p_done = done;
      }
      ++plen;
      ++c_levels;
      if (done) break;
      if (plen >= kMaxPath) {
        err = POMCP_E_ARENA;
        return -1;
      }
      node = child;
      s0 = n0;
      s1 = n1;
      ++t;
      ++depth;
      nvis = cvis;
      blk = cblk;
    }
    // backup, deepest level first (mcts.py:374-381, node.py:166-178)
    double gr = leaf;
    for (int i = plen - 1; i >= 0; --i) {
      const int ani = rl(p_an, i);
      const double r = rl_d(p_r, i);
      gr = rl(p_done, i) ? r : r + p.discount * gr;
      ActRec rec = an[ani];
      const int n = rec.visits + 1;
      const double total = rec.total + gr;
      const double delta = gr - rec.value;
      const double value = rec.value + delta / (double)n;
      const double agg = rec.agg + delta * (gr - value);
      if (lane == 0) {
        rec.visits = n;
        rec.value = value;
        rec.total = total;
        rec.agg = agg;
        an[ani] = rec;
      }
      mm_update(value);
    }
    return depth;
  }

  // sample_agent_initial_state (oracle/driving.py): ego from its obs, the other
  // vehicle rejected until the ego window matches (<= 64 tries).
  __device__ bool sample_agent_initial(uint64_t obs, uint32_t* s0, uint32_t* s1) {
    const int eloc = loc_index(g, (int)((obs >> 32) & 15), (int)((obs >> 36) & 15));
    const int edest = loc_index(g, (int)((obs >> 40) & 15), (int)((obs >> 44) & 15));
    if (eloc < 0 || edest < 0) return false;
    const uint32_t all = (1u << g.num_locs) - 1u;
    const uint32_t ev = make_vehicle(g, eloc, edest);
    uint32_t ov = 0;
    for (int tr = 0; tr < 64; ++tr) {
      const uint32_t av = all & ~(1u << eloc);
      const int s = kth_bit(av, rs.model((uint32_t)popc8(av)));
      const uint32_t avd = all & ~(1u << edest) & ~(1u << s);
      const int d = kth_bit(avd, rs.model((uint32_t)popc8(avd)));
      ov = make_vehicle(g, s, d);
      if (obs_key_wave(g, ev, ov, p.ncells) == obs) break;
    }
    *s0 = p.ego == 0 ? ev : ov;
    *s1 = p.ego == 0 ? ov : ev;
    return true;
  }
};

// ---------------------------------------------------------------- kernels

__global__ __launch_bounds__(256) void k_reset(DevParams p) {
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  const int lane = lane_id();
  TreeHdr h = p.hdr[tree];
  int epoch = (h.epoch + 1) & (int)kEpochMask;
  if (epoch == 0) {   // generation counter wrapped: clear this tree's map
    uint4* hs = reinterpret_cast<uint4*>(p.hash + (int64_t)tree * p.H);
    for (int64_t i = lane; i < p.H; i += kWave) hs[i] = make_uint4(0, 0, 0, 0);
    epoch = 1;
  }
  if (lane == 0) {
    h.root = 0;
    h.n_obs = 1;
    h.n_blocks = 0;
    h.n_log = 0;
    h.belief_size = 0;
    h.epoch = epoch;
    h.error = 0;
    h.root_t = 0;
    h.root_abs = 0;
    h.mm_max = p.has_kb ? p.kb_max : -__builtin_inf();   // utils.py:21-27
    h.mm_min = p.has_kb ? p.kb_min : __builtin_inf();
    p.hdr[tree] = h;
    p.onode[(int64_t)tree * p.No] = make_int2(-1, 0);
    p.ometa[(int64_t)tree * p.No] = 0;
  }
}

__global__ __launch_bounds__(256) void k_update(DevParams p) {
  __shared__ DrvGrid sg;
  stage_grid(p.grid, sg);
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  Tree T(p, sg, tree);
  const int lane = T.lane;
  if (T.err == 0 && !T.root_abs) {   // mcts.py:161-162
    const uint64_t obs = p.in_obs[tree];
    if (T.root_t == 0) {
      // _initial_update (mcts.py:175-227)
      const int node = T.new_obs_node(T.root_t + 1, 0, 0);
      uint32_t s0, s1;
      if (node >= 0 && !T.sample_agent_initial(obs, &s0, &s1)) T.err = POMCP_E_INVALID;  // probe
      uint4* nb = T.other_belief();
      int n = 0;
      while (T.err == 0 && n < p.n_target) {
        if (n >= p.Nr) {
          T.err = POMCP_E_ARENA;
          break;
        }
        T.sample_agent_initial(obs, &s0, &s1);
        if (lane == 0) nb[n] = make_uint4(1u, s0, s1, 0u);
        ++n;
      }
      if (T.err == 0) {
        T.root = node;
        T.root_t = 1;
        T.root_abs = 0;
        T.bsel ^= 1;
        T.bsize = n;
      }
    } else {
      // _update (mcts.py:229-263)
      const int action = p.in_actions[tree];
      const int blk = T.onode[T.root].x;
      if (blk < 0 || action < 0 || action >= p.A) {
        T.err = POMCP_E_NOT_FOUND;
      } else {
        const uint32_t ani = (uint32_t)(blk * p.A + action);
        bool is_new;
        const int child =
            T.find_or_insert(ani, obs, true, T.root_t + 1, 0, T.root_abs, &is_new);
        if (child >= 0) {
          const int cabs = T.ometa[child] & 1;
          // the child's belief: its particles from the log, insertion order
          uint4* nb = T.other_belief();
          int n = 0;
          for (int base = 0; base < T.n_log; base += kWave) {
            const int i = base + lane;
            uint4 rec = make_uint4(0xFFFFFFFFu, 0, 0, 0);
            if (i < T.n_log) rec = T.plog[i];
            const bool m = i < T.n_log && rec.x == (uint32_t)child;
            const uint64_t mask = __ballot(m);
            const int pos = n + (int)__popcll(mask & ((1ull << lane) - 1ull));
            if (m && pos < p.Nr) nb[pos] = make_uint4(rec.y, rec.z, rec.w, 0u);
            n += (int)__popcll(mask);
          }
          if (n > p.Nr) T.err = POMCP_E_ARENA;
          // _reinvigorate (mcts.py:651-700) -> BeliefRejectionSampler (belief.py:145-194)
          const int need = p.n_target - n;
          if (T.err == 0 && !cabs && need > 0) {
            if (n + 2 * need > p.Nr) {
              T.err = POMCP_E_ARENA;
            } else {
              const uint4* pb_ = T.root_belief();
              const double limit = p.limit_factor * (double)need;
              int got = 0, tries = 0, nrej = 0;
              while (got < need && (double)tries < limit) {
                ++tries;
                const uint4 hp = pb_[T.rs.belief((uint32_t)T.bsize)];
                const int ao = (int)T.rs.act(p.other, (uint32_t)p.A);
                uint32_t n0, n1;
                T.joint_step(hp.y, hp.z, action, ao, &n0, &n1);
                const uint32_t e1 = p.ego == 0 ? n0 : n1, o1 = p.ego == 0 ? n1 : n0;
                const uint64_t k = obs_key_wave(sg, e1, o1, p.ncells);
                const uint4 rec = make_uint4(hp.x + 1u, n0, n1, 0u);
                if (k == obs) {
                  if (lane == 0) nb[n + got] = rec;
                  ++got;
                } else if (nrej < need) {
                  if (lane == 0) nb[n + need + nrej] = rec;
                  ++nrej;
                }
              }
              int fill = need - got;
              if (fill > nrej) fill = nrej;
              for (int q = 0; q < fill; ++q)
                if (lane == 0) nb[n + got + q] = nb[n + need + q];
              n += got + fill;
            }
          }
          if (T.err == 0) {
            T.root = child;
            T.root_t += 1;
            T.root_abs = cabs;
            T.bsel ^= 1;
            T.bsize = n;
          }
        }
      }
    }
  }
  T.store_header();
  if (lane == 0) {
    p.upd_out[2 * tree] = T.root_abs;
    p.upd_out[2 * tree + 1] = T.err;
  }
}

__global__ __launch_bounds__(256) void k_search(DevParams p, int num_sims) {
  __shared__ DrvGrid sg;
  stage_grid(p.grid, sg);
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  Tree T(p, sg, tree);
  const int lane = T.lane;
  int action = 0, max_depth = 0, sims = 0, blk = -1, visits = 0;
  if (T.err == 0 && T.root_t == 0) T.err = POMCP_E_STATE;
  if (T.err == 0 && !T.root_abs) {   // mcts.py:270-272
    const int2 rn = T.onode[T.root];
    blk = rn.x;
    visits = rn.y;
    if (blk < 0) blk = T.expand(T.root);   // mcts.py:279-281
    if (blk >= 0 && T.bsize <= 0) T.err = POMCP_E_STATE;
    for (int s = 0; s < num_sims && T.err == 0; ++s) {
      const int d = T.simulate(blk, visits);
      if (d < 0) break;
      ++visits;                               // mcts.py:288
      max_depth = d > max_depth ? d : max_depth;
      ++sims;
    }
    if (T.err == 0) action = T.final_action(blk, visits);
    if (lane == 0 && blk >= 0) T.onode[T.root] = make_int2(blk, visits);
  }
  T.store_header();
  // root statistics: MCTS.step_statistics + root children
  pomcp_root_stats* st = p.stats + tree;
  const int A = p.A;
  if (lane < A) {
    ActRec r;
    r.visits = 0;
    r.value = 0.0;
    r.total = 0.0;
    if (blk >= 0) r = T.an[(int64_t)blk * A + lane];
    st->child_visits[lane] = r.visits;
    st->child_values[lane] = r.value;
    st->child_totals[lane] = r.total;
    p.merge[((int64_t)tree * A + lane) * 2] = (double)r.visits;
    p.merge[((int64_t)tree * A + lane) * 2 + 1] = r.total;
  }
  if (lane == 0) {
    st->action = action;
    st->num_sims = sims;
    st->search_depth = max_depth;
    st->root_visits = visits;
    st->root_absorbing = T.root_abs;
    st->belief_size = T.bsize;
    st->error = T.err;
    st->num_children = blk >= 0 ? A : 0;
    st->min_value = T.mm_min;
    st->max_value = T.mm_max;
    st->n_levels = T.c_levels;
    st->n_expansions = T.c_expand;
    st->n_new_nodes = T.c_new;
    st->n_rollout_steps = T.c_rollout;
    st->n_probes = T.c_probes;
    st->n_obs_nodes = T.n_obs;
    st->n_blocks = T.n_blocks;
    st->n_log = T.n_log;
    st->pad = 0;
  }
}

// Synthetic Driving-v1 roots: env b0 sample for tree b under key
// (env_seed_base + b, 0x40000000), ego's initial observation.
__global__ __launch_bounds__(256) void k_synthetic_obs(DevParams p, uint64_t env_seed_base) {
  __shared__ DrvGrid sg;
  stage_grid(p.grid, sg);
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  Streams env;
  env.seed = env_seed_base + (uint64_t)tree;
  env.tree = 0x40000000u;
  for (int k = 0; k < 5; ++k) env.ctr[k] = 0;
  uint32_t s0, s1;
  drv_sample_initial_state2(sg, [&](uint32_t n) { return env.model(n); }, &s0, &s1);
  const uint32_t e = p.ego == 0 ? s0 : s1, o = p.ego == 0 ? s1 : s0;
  const uint64_t key = obs_key_wave(sg, e, o, p.ncells);
  if (lane_id() == 0) p.out_obs[tree] = key;
}

// Snapshot / restore of the post-initial-update root state.
__global__ __launch_bounds__(256) void k_restore(DevParams p, const TreeHdr* snap,
                                                 const int2* snap_root) {
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  const int lane = lane_id();
  int epoch = (p.hdr[tree].epoch + 1) & (int)kEpochMask;
  if (epoch == 0) {
    uint4* hs = reinterpret_cast<uint4*>(p.hash + (int64_t)tree * p.H);
    for (int64_t i = lane; i < p.H; i += kWave) hs[i] = make_uint4(0, 0, 0, 0);
    epoch = 1;
  }
  if (lane == 0) {
    TreeHdr h = snap[tree];
    h.epoch = epoch;
    p.hdr[tree] = h;
    p.onode[(int64_t)tree * p.No + h.root] = snap_root[tree];
  }
}

__global__ void k_fp_selftest(const double* a, const double* b, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[4 * i + 0] = sqrt(a[i]);
  out[4 * i + 1] = a[i] / b[i];
  out[4 * i + 2] = a[i] + 0.95 * b[i];
  out[4 * i + 3] = (a[i] - b[i]) / (a[i] + b[i]);
}

}  // namespace pb
