// k_search: the POMCP simulation loop with FOUR trees per wavefront.
//
// Replaces posggym_baselines/planning/mcts.py:269-452 (get_action, _simulate,
// _rollout, the three selection rules, the final action choice) and the
// search-side parts of node.py / belief.py / utils.py:15-42.
//
// Why 4 trees per wave: a simulation is a long chain of dependent scalar-ish
// operations (select -> step -> observe -> descend -> back up); with one tree
// per wave every instruction of the chain served one tree and the kernel was
// bound by per-wave issue latency.  Here each 16-lane group owns one tree and
// holds that tree's scalars as group-uniform VGPRs, so every instruction of
// the chain advances four independent trees.  Trees that are in different
// phases of a simulation (descending, rolling out, backing up, starting the
// next one) run under exec masks: one loop iteration executes each phase
// block once for the groups that are in it.
//
// Block layout (one expanded obs node, A action nodes, A x 128 B):
//   part a            : stats0 of action a {visits, pad, value}
//   part A + a        : stats1 of action a {total, agg}
//   part 2A + 6a + k  : child slot k of action a {obs key|valid|absorbing, block, visits}
// Lane i of a group holds parts i, 16 + i, 32 + i of the block being visited.
#pragma clang fp contract(off)

namespace pb {

constexpr int kG = 4;             // trees per wavefront
constexpr int kL = 16;            // lanes per tree
constexpr int kGroupsPerBlock = kG * (256 / kWave);   // 16 trees per 256-thread workgroup
constexpr uint32_t kGPage = 32;   // RNG page per stream: 8 Philox blocks
constexpr int kPathMax = 64;

enum : int { PH_LEVEL = 0, PH_ROLL = 1, PH_BACKUP = 2, PH_START = 3, PH_DONE = 4 };

__device__ __forceinline__ int glane() { return lane_id() & (kL - 1); }
__device__ __forceinline__ int gbase() { return lane_id() & ~(kL - 1); }

// value of `v` on lane `src` (0..15) of this lane's group
__device__ __forceinline__ uint32_t gshfl(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((gbase() + src) << 2, (int)v);
}
__device__ __forceinline__ double gshfl_d(double v, int src) {
  const int a = (gbase() + src) << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(a, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(a, __double2hiint(v));
  return __hiloint2double(hi, lo);
}
// this group's 16 bits of a wave ballot
__device__ __forceinline__ uint32_t gballot(bool pred) {
  const uint64_t m = __ballot(pred);
  return (uint32_t)(m >> gbase()) & 0xFFFFu;
}
__device__ __forceinline__ int ffs16(uint32_t m) { return m ? __ffs((int)m) - 1 : -1; }

__device__ __forceinline__ uint4 sel_part(const uint4& q0, const uint4& q1, const uint4& q2, int r) {
  return r == 0 ? q0 : (r == 1 ? q1 : q2);
}
// part p (group-uniform) of the block held in q0..q2
__device__ __forceinline__ uint4 get_part(const uint4& q0, const uint4& q1, const uint4& q2, int p) {
  const uint4 v = sel_part(q0, q1, q2, p >> 4);
  const int s = p & 15;
  return make_uint4(gshfl(v.x, s), gshfl(v.y, s), gshfl(v.z, s), gshfl(v.w, s));
}

struct GTree {
  const DevParams& p;
  const DrvModel& m;
  int tree;
  bool valid;
  ActNode* an;
  uint4* plog;
  uint4* rbel;
  OvfSlot* ovf;
  uint32_t* rng;     // LDS: 4 pages of kGPage words (belief, model, act0, act1)
  uint32_t* path;    // LDS: kPathMax x {stats byte offset | done << 31, r lo, r hi}
  int root_blk, root_visits, n_blocks, n_log, n_nodes, bsize, err;
  double mm_min, mm_max;
  uint64_t seed;
  uint32_t tkey;
  uint32_t c_bel, c_sel, c_mod, c_a0, c_a1;
  int32_t c_rollout, c_probes;

  __device__ GTree(const DevParams& pp, const DrvModel& mm, int t, uint32_t* rng_lds,
                   uint32_t* path_lds)
      : p(pp), m(mm), tree(t), rng(rng_lds), path(path_lds) {
    valid = t < p.B;
    const int tt = valid ? t : 0;
    an = p.an + (int64_t)tt * p.Nb * p.A;
    plog = p.plog + (int64_t)tt * p.Np;
    ovf = p.ovf + (int64_t)tt * p.H;
    const TreeHdr* h = p.hdr + tt;
    rbel = p.belief + (int64_t)tt * 2 * p.Nr + (int64_t)h->belief_sel * p.Nr;
    root_blk = h->root_blk;
    root_visits = h->root_visits;
    n_blocks = h->n_blocks;
    n_log = h->n_log;
    n_nodes = h->n_nodes;
    bsize = h->belief_size;
    err = h->error;
    mm_min = h->mm_min;
    mm_max = h->mm_max;
    seed = h->seed;
    tkey = h->tree_key;
    c_bel = h->ctr[0];
    c_sel = h->ctr[1];
    c_mod = h->ctr[2];
    c_a0 = h->ctr[3];
    c_a1 = h->ctr[4];
    c_rollout = c_probes = 0;
  }

  // fields the search changes (field stores: no header copy is kept live)
  __device__ void store_header() {
    if (glane() != 0 || !valid) return;
    TreeHdr* h = p.hdr + tree;
    h->n_blocks = n_blocks;
    h->n_log = n_log;
    h->n_nodes = n_nodes;
    h->error = err;
    h->root_blk = root_blk;
    h->root_visits = root_visits;
    h->mm_min = mm_min;
    h->mm_max = mm_max;
    h->ctr[0] = c_bel;
    h->ctr[1] = c_sel;
    h->ctr[2] = c_mod;
    h->ctr[3] = c_a0;
    h->ctr[4] = c_a1;
  }

  // ---- RNG: per tree and stream a kGPage-word LDS page, lanes 0..7 refill it
  __device__ void refill(int slot, uint32_t stream, uint32_t pg) {
    const int i = glane();
    if (i < (int)(kGPage / 4)) {
      uint32_t c[4] = {pg * (kGPage / 4) + (uint32_t)i, 0u, stream, (uint32_t)(seed >> 32)};
      philox4x32_10(c, (uint32_t)seed, tkey);
      reinterpret_cast<uint4*>(rng + slot * kGPage)[i] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  }
  __device__ void warm_rng() {
    refill(0, S_BELIEF, c_bel / kGPage);
    refill(1, S_MODEL, c_mod / kGPage);
    refill(2, S_ACT_BASE, c_a0 / kGPage);
    refill(3, S_ACT_BASE + 1, c_a1 / kGPage);
  }
  __device__ uint32_t draw(int slot, uint32_t& ctr, uint32_t stream) {
    const uint32_t j = ctr++;
    if ((j & (kGPage - 1)) == 0u) refill(slot, stream, j / kGPage);
    return rng[slot * kGPage + (j & (kGPage - 1))];
  }
  __device__ uint32_t d_belief(uint32_t n) { return uniform_int(draw(0, c_bel, S_BELIEF), n); }
  __device__ uint32_t d_model(uint32_t n) { return uniform_int(draw(1, c_mod, S_MODEL), n); }
  __device__ uint32_t d_act(int agent, uint32_t n) {
    return agent == 0 ? uniform_int(draw(2, c_a0, S_ACT_BASE), n)
                      : uniform_int(draw(3, c_a1, S_ACT_BASE + 1), n);
  }
  __device__ uint32_t d_select(uint32_t n) {
    return uniform_int(philox_word(seed, tkey, S_SELECT, c_sel++), n);
  }
  __device__ double d_select_float() {
    return uniform_float(philox_word(seed, tkey, S_SELECT, c_sel++));
  }

  __device__ void load_block(int blk, uint4* q0, uint4* q1, uint4* q2) const {
    const uint4* b = reinterpret_cast<const uint4*>(an + (int64_t)blk * p.A);
    const int i = glane(), np = kLanesPerAct * p.A;
    *q0 = i < np ? b[i] : make_uint4(0, 0, 0, 0);
    *q1 = 16 + i < np ? b[16 + i] : make_uint4(0, 0, 0, 0);
    *q2 = 32 + i < np ? b[32 + i] : make_uint4(0, 0, 0, 0);
  }

  // ObsNode.add_child for every action (mcts.py:279-281, 318-321): zeroed block.
  __device__ int alloc_block() {
    if (n_blocks >= p.Nb) {
      err = POMCP_E_ARENA;
      return -1;
    }
    const int b = n_blocks++;
    uint4* d = reinterpret_cast<uint4*>(an + (int64_t)b * p.A);
    const int i = glane(), np = kLanesPerAct * p.A;
    for (int k = i; k < np; k += kL) d[k] = make_uint4(0, 0, 0, 0);
    return b;
  }

  __device__ void mm_update(double v) {   // utils.py:29-32
    if (v > mm_max) mm_max = v;
    if (v < mm_min) mm_min = v;
  }
  __device__ double normalize(double v) const {   // utils.py:34-39
    return mm_max > mm_min ? (v - mm_min) / (mm_max - mm_min) : v;
  }

  // PUCB with N == 0 (mcts.py:494-500): random.choices over the uniform prior.
  __device__ int pucb_prior_draw() {
    const int A = p.A;
    const double w = 1.0 / (double)A;
    double total = w;
    for (int k = 1; k < A; ++k) total = total + w;
    const double x = d_select_float() * (total + 0.0);
    double acc = w;
    int r = A - 1;
    bool found = false;
    for (int k = 0; k < A - 1; ++k) {
      if (!found && x < acc) {
        r = k;
        found = true;
      }
      acc = acc + w;
    }
    return r;
  }

  // _search_action_selection (mcts.py:492-563).  Parts 0..A-1 (lanes 0..A-1 of
  // q0) hold {visits, value} of the A children.
  template <int SEL>
  __device__ int choose(const uint4& q0, int visits) {
    const int A = p.A, i = glane();
    if (SEL == POMCP_SEL_PUCB && visits == 0) return pucb_prior_draw();
    if (visits == 0) return (int)d_select((uint32_t)A);
    const bool head = i < A;
    const int n = head ? (int)q0.x : 0;
    const double v = hilo_d(q0.z, q0.w);
    if (SEL == POMCP_SEL_UNIFORM) {   // min_visit_action_selection
      int min_n = visits + 1, best = 0;
      for (int a = 0; a < A; ++a) {
        const int na = (int)gshfl((uint32_t)n, a);
        if (na < min_n) {
          min_n = na;
          best = a;
        }
      }
      return best;
    }
    double score = -__builtin_inf();
    if (SEL == POMCP_SEL_UCB) {
      const uint32_t unv = gballot(head && n == 0);   // mcts.py:539-540
      if (unv) return ffs16(unv);
      const double log_n = p.logtab[visits < p.logtab_n ? visits : 0];
      if (visits >= p.logtab_n) err = POMCP_E_ARENA;
      if (head) score = normalize(v) + p.c * sqrt(log_n / (double)n);   // mcts.py:541-542
    } else {   // PUCB, mcts.py:502-527
      const double noise = 1.0 / (double)A;
      const double prior = (1.0 / (double)A) * (1.0 - p.pucb_f) + p.pucb_f * noise;
      const double sqrt_n = sqrt((double)visits);
      if (head) score = (n > 0 ? normalize(v) : 0.0) + p.c * prior * (sqrt_n / (double)(1 + n));
    }
    double best_v = -__builtin_inf();
    int best = 0;
    for (int a = 0; a < A; ++a) {   // strict '>' in action order
      const double sa = gshfl_d(score, a);
      if (sa > best_v) {
        best_v = sa;
        best = a;
      }
    }
    return best;
  }

  // _final_action_selection (mcts.py:565-600) on the root block.
  template <int SEL>
  __device__ int final_action() {
    const int A = p.A;
    uint4 q0, q1, q2;
    load_block(root_blk, &q0, &q1, &q2);
    uint32_t ties = 0;
    int nt = 0;
    if (SEL == POMCP_SEL_PUCB) {
      if (root_visits == 0) return (int)d_select((uint32_t)A);
      int mx = 0;
      for (int a = 0; a < A; ++a) {
        const int na = (int)gshfl(q0.x, a);
        if (na == mx) {
          ties |= 1u << a;
          ++nt;
        } else if (na > mx) {
          mx = na;
          ties = 1u << a;
          nt = 1;
        }
      }
    } else {
      double mx = -__builtin_inf();
      for (int a = 0; a < A; ++a) {
        const double va = hilo_d(gshfl(q0.z, a), gshfl(q0.w, a));
        if (va == mx) {
          ties |= 1u << a;
          ++nt;
        } else if (va > mx) {
          mx = va;
          ties = 1u << a;
          nt = 1;
        }
      }
    }
    return kth_bit(ties, d_select((uint32_t)nt));
  }

  // overflow map (children beyond the 6 inline slots), 16 lanes per probe
  __device__ bool ovf_ref(uint32_t ani, uint64_t okey, int done, uint32_t* id, int* cblk,
                          int* cvis, int32_t** blk_ptr) {
    const int epoch = p.hdr[tree].epoch;
    const uint64_t key = okey | ((uint64_t)epoch << kEpochShift);
    uint32_t b = ovf_hash(ani, okey) & p.bucket_mask;
    const int i = glane();
    for (uint32_t probe = 0; probe <= p.bucket_mask; ++probe) {
      ++c_probes;
      OvfSlot* e = ovf + (int64_t)b * kBucket + i;
      const uint4 s = reinterpret_cast<const uint4*>(e)[0];
      const uint4 s2 = reinterpret_cast<const uint4*>(e)[1];
      const uint64_t skey = (uint64_t)s.x | ((uint64_t)s.y << 32);
      const bool ok = (uint32_t)(skey >> kEpochShift) == (uint32_t)epoch;
      const uint32_t mm = gballot(ok && skey == key && s.z == ani);
      const uint32_t em = gballot(!ok);
      const int L = mm ? ffs16(mm) : ffs16(em);
      if (mm || em) {
        OvfSlot* t = ovf + (int64_t)b * kBucket + L;
        *id = p.ovf_base + b * kBucket + (uint32_t)L;
        *blk_ptr = &t->block;
        if (mm) {
          *cblk = (int)gshfl(s2.x, L);
          *cvis = (int)gshfl(s2.y, L) + 1;
        } else {
          *cblk = -1;
          *cvis = 1;
          ++n_nodes;
        }
        if (i == 0) {
          reinterpret_cast<uint4*>(t)[0] =
              make_uint4((uint32_t)key, (uint32_t)(key >> 32), ani, (uint32_t)done);
          reinterpret_cast<uint4*>(t)[1] = make_uint4((uint32_t)*cblk, (uint32_t)*cvis, 0u, 0u);
        }
        return true;
      }
      b = (b + 1) & p.bucket_mask;
    }
    err = POMCP_E_ARENA;
    return false;
  }
};

// simulation state of one tree (group-uniform registers)
struct Sim {
  int phase, t, depth, plen, blk, nvis, k, sims, max_depth, rdepth;
  uint32_t s0, s1;
  int32_t* leaf_ptr;
  double ret;
};

template <int SEL>
__global__ __launch_bounds__(256, POMCP_SEARCH_WAVES_PER_SIMD) void k_search(DevParams p,
                                                                            int num_sims) {
  __shared__ DrvModel sm;
  __shared__ uint32_t rng_lds[kGroupsPerBlock][4 * kGPage];
  __shared__ uint32_t path_lds[kGroupsPerBlock][kPathMax * 3];
  stage_model(p.model, sm);
  const int g_in_block = threadIdx.x / kL;
  const int tree = blockIdx.x * kGroupsPerBlock + g_in_block;
  GTree T(p, sm, tree, rng_lds[g_in_block], path_lds[g_in_block]);
  const int i = glane();
  // counters derived from arena growth: one particle per tree level stepped,
  // one block per expansion, one node per new obs child
  const int log0 = T.n_log, blocks0 = T.n_blocks, nodes0 = T.n_nodes;
  const int A = p.A;
  Sim S;
  S.phase = PH_START;
  S.sims = 0;
  S.max_depth = 0;
  S.t = S.depth = S.plen = S.blk = S.nvis = S.k = S.rdepth = 0;
  S.s0 = S.s1 = 0;
  S.leaf_ptr = nullptr;
  S.ret = 0.0;
  const int root_abs = T.valid ? p.hdr[tree].root_abs : 0;
  if (!T.valid || T.err != 0 || root_abs) S.phase = PH_DONE;   // mcts.py:270-272
  if (S.phase != PH_DONE && p.hdr[tree].root_t == 0) {
    T.err = POMCP_E_STATE;
    S.phase = PH_DONE;
  }
  if (S.phase != PH_DONE) {
    if (T.root_blk < 0) T.root_blk = T.alloc_block();   // mcts.py:279-281
    if (T.root_blk < 0 || T.bsize <= 0) {
      if (T.err == 0) T.err = POMCP_E_STATE;
      S.phase = PH_DONE;
    }
  }
  T.warm_rng();
  const bool any_sims = num_sims > 0;
  if (!any_sims && S.phase != PH_DONE) S.phase = PH_DONE;
  // Arrival at an obs node (start of _simulate, mcts.py:315-328): depth/step
  // cutoff -> back up 0; unexpanded -> expand and roll out; else select there.
  auto arrive = [&]() {
    if (S.depth > p.depth_limit || S.t > p.step_limit) {     // mcts.py:315
      S.ret = 0.0;
      S.phase = PH_BACKUP;
    } else if (S.blk < 0) {                                   // mcts.py:318-328
      const int b = T.alloc_block();
      if (b < 0) {
        S.phase = PH_DONE;
      } else {
        if (i == 0) *S.leaf_ptr = b;
        S.ret = 0.0;
        S.k = 0;
        S.rdepth = S.depth;   // the rollout's own depth counter (mcts.py:449)
        S.phase = PH_ROLL;
      }
    }
  };
  // Loop iteration = one step of every tree: start a simulation (and select at
  // the root), one tree level, one rollout step, the backup (in this order, so a
  // depth-2 search takes 3 iterations per simulation).
  while (__ballot(S.phase != PH_DONE)) {
    // ---------------------------------------------------------- start a simulation
    if (S.phase == PH_START) {
      if (S.sims >= num_sims) {
        S.phase = PH_DONE;
      } else {
        const uint32_t k = T.d_belief((uint32_t)T.bsize);   // belief.py:55
        const uint4 pr = T.rbel[k];
        S.t = (int)pr.x;
        S.s0 = pr.y;
        S.s1 = pr.z;
        S.blk = T.root_blk;
        S.nvis = T.root_visits;
        S.depth = 0;
        S.plen = 0;
        S.phase = PH_LEVEL;
        arrive();
      }
    }
    // ---------------------------------------------------------- one tree level
    if (S.phase == PH_LEVEL) {
      {
        uint4 q0, q1, q2;
        T.load_block(S.blk, &q0, &q1, &q2);
        const int a = T.choose<SEL>(q0, S.nvis);                      // mcts.py:330
        const uint32_t ao = T.d_act(p.other, (uint32_t)A);            // mcts.py:331
        const uint32_t j = T.d_model(2);                              // exec-order shuffle
        uint32_t n0, n1;
        const uint32_t ea = (uint32_t)a;
        drv_step2_vec(sm, S.s0, S.s1, p.ego == 0 ? ea : ao, p.ego == 0 ? ao : ea, j, &n0, &n1);
        const uint32_t e0 = p.ego == 0 ? S.s0 : S.s1;
        const uint32_t e1 = p.ego == 0 ? n0 : n1;
        const uint32_t o1 = p.ego == 0 ? n1 : n0;
        const double r = drv_reward_vec(sm, e0, e1);
        const int done = (((e1 >> 15) & 3u) != 0u ||
                          (((n0 >> 15) & 3u) != 0u && ((n1 >> 15) & 3u) != 0u)) ? 1 : 0;
        const uint64_t okey = obs_key_vec(sm, e1, o1);
        // ActionNode.children[obs] among the 6 inline slots (mcts.py:356-370)
        const int lo = 2 * A + kSlots * a;
#define POMCP_SLOT_TEST(Q, R, MT, EM)                                              \
  bool MT, EM;                                                                     \
  {                                                                                \
    const int part = 16 * (R) + i;                                                 \
    const bool in = part >= lo && part < lo + kSlots;                              \
    const uint64_t sk = (uint64_t)(Q).x | ((uint64_t)(Q).y << 32);                 \
    const bool vb = (sk & kValidBit) != 0;                                         \
    MT = in && vb && (sk & kObsMask) == okey;                                      \
    EM = in && !vb;                                                                \
  }
        POMCP_SLOT_TEST(q0, 0, mt0, em0)
        POMCP_SLOT_TEST(q1, 1, mt1, em1)
        POMCP_SLOT_TEST(q2, 2, mt2, em2)
#undef POMCP_SLOT_TEST
        const uint64_t mm = (uint64_t)gballot(mt0) | ((uint64_t)gballot(mt1) << 16) |
                            ((uint64_t)gballot(mt2) << 32);
        const uint64_t ee = (uint64_t)gballot(em0) | ((uint64_t)gballot(em1) << 16) |
                            ((uint64_t)gballot(em2) << 32);
        const uint32_t ani = (uint32_t)(S.blk * A + a);
        uint32_t cid = 0;
        int cblk = -1, cvis = 1;
        int32_t* cptr = nullptr;
        bool ok = true;
        if (mm || ee) {
          const int P = mm ? (int)__builtin_ctzll(mm) : (int)__builtin_ctzll(ee);
          const uint4 sl = get_part(q0, q1, q2, P);
          const int ks = P - lo;
          if (mm) {
            cblk = (int)sl.z;
            cvis = (int)sl.w + 1;
          } else {
            ++T.n_nodes;
          }
          const uint64_t nk = okey | kValidBit | ((uint64_t)done << 63);
          uint4* slot = reinterpret_cast<uint4*>(T.an + (int64_t)S.blk * A) + P;
          if (i == 0)
            *slot = make_uint4((uint32_t)nk, (uint32_t)(nk >> 32), (uint32_t)cblk, (uint32_t)cvis);
          cid = ani * kSlots + (uint32_t)ks + 1u;
          cptr = reinterpret_cast<int32_t*>(slot) + 2;
        } else {
          ok = T.ovf_ref(ani, okey, done, &cid, &cblk, &cvis, &cptr);
        }
        if (!ok || T.err != 0 || T.n_log >= p.Np || S.plen >= kPathMax) {
          if (T.err == 0) T.err = POMCP_E_ARENA;
          S.phase = PH_DONE;
        } else {
          if (i == 0) T.plog[T.n_log] = make_uint4(cid, (uint32_t)(S.t + 1), n0, n1);   // mcts.py:371
          ++T.n_log;
          // path entry: byte offset of the action node's stats0 | done, reward
          const uint32_t off = (uint32_t)((S.blk * A) * 128 + a * 16);
          if (i == 0) {
            uint32_t* pe = T.path + 3 * S.plen;
            pe[0] = off | ((uint32_t)done << 31);
            pe[1] = (uint32_t)__double2loint(r);
            pe[2] = (uint32_t)__double2hiint(r);
          }
          ++S.plen;
          if (done) {
            S.ret = 0.0;
            S.phase = PH_BACKUP;
          } else {
            S.blk = cblk;
            S.nvis = cvis;
            S.leaf_ptr = cptr;
            S.s0 = n0;
            S.s1 = n1;
            ++S.t;
            ++S.depth;
            arrive();
          }
        }
      }
    }
    // ---------------------------------------------------------- one rollout step
    if (S.phase == PH_ROLL) {                                  // mcts.py:414-450
      if (!(S.rdepth <= p.depth_limit && S.t <= p.step_limit)) {
        S.phase = PH_BACKUP;
      } else {
        const uint32_t ae = T.d_act(p.ego, (uint32_t)A);       // search_policy.py:177
        const uint32_t ao = T.d_act(p.other, (uint32_t)A);     // other_policy.py:151
        const uint32_t j = T.d_model(2);
        uint32_t n0, n1;
        drv_step2_vec(sm, S.s0, S.s1, p.ego == 0 ? ae : ao, p.ego == 0 ? ao : ae, j, &n0, &n1);
        const uint32_t e0 = p.ego == 0 ? S.s0 : S.s1, e1 = p.ego == 0 ? n0 : n1;
        const double r = drv_reward_vec(sm, e0, e1);
        if (S.k >= p.dpow_n) {
          T.err = POMCP_E_ARENA;
          S.phase = PH_DONE;
        } else {
          S.ret += p.dpow[S.k] * r;   // mcts.py:420-422
          ++T.c_rollout;
          const bool done = ((e1 >> 15) & 3u) != 0u ||
                            (((n0 >> 15) & 3u) != 0u && ((n1 >> 15) & 3u) != 0u);
          if (done) {
            S.phase = PH_BACKUP;
          } else {
            S.s0 = n0;
            S.s1 = n1;
            ++S.t;
            ++S.rdepth;
            ++S.k;
          }
        }
      }
    }
    // ---------------------------------------------------------- backup
    if (S.phase == PH_BACKUP) {                                // mcts.py:374-381
      double gr = S.ret;
      const char* base = reinterpret_cast<const char*>(T.an);
      for (int c0 = ((S.plen - 1) / kL) * kL; c0 >= 0; c0 -= kL) {
        // statistics of the levels of this chunk, lane i -> level c0 + i
        uint4 st0 = make_uint4(0, 0, 0, 0), st1 = make_uint4(0, 0, 0, 0);
        if (c0 + i < S.plen) {
          const uint32_t off = T.path[3 * (c0 + i)] & 0x7FFFFFFFu;
          st0 = *reinterpret_cast<const uint4*>(base + off);
          st1 = *reinterpret_cast<const uint4*>(base + off + 16 * A);
        }
        const int top = (S.plen - 1 - c0) < (kL - 1) ? (S.plen - 1 - c0) : (kL - 1);
        for (int li = top; li >= 0; --li) {
          const uint32_t* pe = T.path + 3 * (c0 + li);
          const uint32_t w0 = pe[0];
          const double r = hilo_d(pe[1], pe[2]);
          gr = (w0 >> 31) ? r : r + p.discount * gr;
          const int n = (int)gshfl(st0.x, li) + 1;
          const double value0 = hilo_d(gshfl(st0.z, li), gshfl(st0.w, li));
          const double total = hilo_d(gshfl(st1.x, li), gshfl(st1.y, li)) + gr;
          const double delta = gr - value0;
          const double value = value0 + delta / (double)n;
          const double agg = hilo_d(gshfl(st1.z, li), gshfl(st1.w, li)) + delta * (gr - value);
          const uint32_t off = w0 & 0x7FFFFFFFu;
          if (i == 0)
            *reinterpret_cast<uint4*>(const_cast<char*>(base) + off) = make_uint4(
                (uint32_t)n, 0u, (uint32_t)__double2loint(value), (uint32_t)__double2hiint(value));
          if (i == 1)
            *reinterpret_cast<uint4*>(const_cast<char*>(base) + off + 16 * A) =
                make_uint4((uint32_t)__double2loint(total), (uint32_t)__double2hiint(total),
                           (uint32_t)__double2loint(agg), (uint32_t)__double2hiint(agg));
          T.mm_update(value);
        }
      }
      ++T.root_visits;                                          // mcts.py:288
      S.max_depth = S.depth > S.max_depth ? S.depth : S.max_depth;
      ++S.sims;
      S.phase = PH_START;
    }
  }
  // ------------------------------------------------------------------ results
  int action = 0;
  const bool have = T.valid && T.err == 0 && !root_abs && T.root_blk >= 0;
  if (have) action = T.final_action<SEL>();
  T.store_header();
  if (!T.valid) return;
  pomcp_root_stats* st = p.stats + tree;
  uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0;
  if (have) T.load_block(T.root_blk, &q0, &q1, &q2);
  for (int a = 0; a < A; ++a) {
    const uint4 a0 = get_part(q0, q1, q2, a);
    const uint4 a1 = get_part(q0, q1, q2, A + a);
    if (i == a) {
      const double va = hilo_d(a0.z, a0.w), tot = hilo_d(a1.x, a1.y);
      st->child_visits[a] = (int)a0.x;
      st->child_values[a] = va;
      st->child_totals[a] = tot;
      p.merge[((int64_t)tree * A + a) * 2] = (double)a0.x;
      p.merge[((int64_t)tree * A + a) * 2 + 1] = tot;
    }
  }
  if (i == 0) {
    st->action = action;
    st->num_sims = S.sims;
    st->search_depth = S.max_depth;
    st->root_visits = T.root_visits;
    st->root_absorbing = root_abs;
    st->belief_size = T.bsize;
    st->error = T.err;
    st->num_children = have ? A : 0;
    st->min_value = T.mm_min;
    st->max_value = T.mm_max;
    st->n_levels = T.n_log - log0;
    st->n_expansions = T.n_blocks - blocks0;
    st->n_new_nodes = T.n_nodes - nodes0;
    st->n_rollout_steps = T.c_rollout;
    st->n_probes = T.c_probes;
    st->n_obs_nodes = T.n_nodes;
    st->n_blocks = T.n_blocks;
    st->n_log = T.n_log;
    st->pad = 0;
  }
}

template __global__ void k_search<POMCP_SEL_PUCB>(DevParams, int);
template __global__ void k_search<POMCP_SEL_UCB>(DevParams, int);
template __global__ void k_search<POMCP_SEL_UNIFORM>(DevParams, int);

}  // namespace pb
