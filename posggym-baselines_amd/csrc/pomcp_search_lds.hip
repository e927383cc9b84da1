// k_search_lds: the POMCP simulation loop with ONE WAVE per tree and the
// tree in LDS -- the exact single tree (BASELINE config 2 as ONE planner, the
// drop-in POMCP's default mode) and small batches of planners.
//
// Replaces posggym_baselines/planning/mcts.py:269-452 (get_action, _simulate,
// _rollout, the selection rules, the final action choice) like k_search
// (pomcp_search.hip), with the same results bit for bit: the same simulations
// in the same order, the same draws of every stream, the same FP64 operations
// in the same order.  k_search runs one tree per LANE and is the throughput
// kernel for thousands of trees; a lone tree there is one lane waiting on
// ~6 dependent HBM round trips per simulation (~11 us).  Here the whole wave
// works on one simulation at a time:
//   * the tree's blocks live in LDS for the launch (staged in from the HBM
//     arena at the start, written back at the end), so a tree level is a few
//     LDS reads; blocks beyond the LDS pool stay in HBM (a uniform branch per
//     access), so any tree size runs, the overflowing part at HBM speed;
//   * lane 8a + q holds part q of action a's 128 B LDS line (q = 0 statistics
//     {visits, -, value}, 1 {total, -}, 2..7 the six inline child slots): one
//     LDS read per lane gives the selection its statistics and every action's
//     child slots at once;
//   * lane group a (8 lanes) runs the generative step and the observation key
//     for action a -- for EVERY action, before the selection has picked one
//     (the step's draws come from the other agent's and the model's streams,
//     which the selection does not touch), so the step overlaps the FP64
//     selection instead of following it; the child lookup of all actions is
//     one ballot; the chosen action's results are read out of its lane group;
//   * the UCB / PUCB scores of the A actions are computed in parallel lanes
//     (lane 8a), then scanned in action order with the reference's strict '>'
//     (mcts.py:541-545);
//   * RNG (philox.h): a page of 64 Philox blocks per stream in VGPRs (lane l:
//     block page*64 + l), refilled every 256 draws; a draw is one readlane;
//   * loads one simulation ahead: the next belief particle (belief.py:55: its
//     index depends only on the belief stream); a node's visits and the
//     math.log(N) of its next arrival sit beside its LDS block (nl_n, nl_v;
//     the node line's bytes 20..31 in HBM), the log loaded during a level and
//     stored one level later;
//   * particle-log records (mcts.py:371) go to a per-tree scratch log (no
//     atomics); k_log_merge then appends every tree's records to the search
//     waves' shared logs (pomcp_device.h WaveLog) in tree order, so re-root,
//     extraction and compaction read the same log as after k_search.
//   * with NP step-tree producer waves in the tree's workgroup (NP > 0, depth
//     limits <= 8): the producers evaluate every action sequence of each
//     coming simulation's first three levels and hand over its particle, so the
//     search wave reads a level's steps from LDS (kSpecLevels, below).
// Block layout in LDS: [block][action] 128 B lines {stats, total, slots 0..5}
// plus the node's {N, log N}; in HBM the (A + 1)-line layout of
// pomcp_device.h, converted part by part when staged in and written back.
// Child slots are rewritten on every arrival here (their visits are used only
// while the child has no block, as in k_search).
#pragma clang fp contract(off)

namespace pb {

#ifndef PB_SPEC_PRODUCERS   // measurement builds only (tools/dbg/st4.sh)
#define PB_SPEC_PRODUCERS 2
#endif
#ifndef PB_SPEC_SLOTS
#define PB_SPEC_SLOTS 3
#endif
#ifndef PB_SPEC_POOL_KB
#define PB_SPEC_POOL_KB 128
#endif
// tree blocks (+ model, path, caches below); with step-tree producers (NP > 0)
// their slots take 15 KB of it
__host__ __device__ constexpr int lds_pool_bytes(int NP) { return (NP > 0 ? PB_SPEC_POOL_KB : 136) * 1024; }
constexpr int kLdsDpow = 256;                      // discount powers cached in LDS
constexpr int kLdsBelief = 128;                    // root beliefs up to this size live in LDS
__host__ __device__ constexpr int lds_pool_blocks(int A, int NP = 0) {
  return lds_pool_bytes(NP) / 16 / (8 * A);
}
// Speculative step tree (NP producer waves): for simulation k the producers
// evaluate the generative step of every action sequence of the first
// kSpecLevels tree levels (A + A^2 + A^3 steps and observation keys) with the
// draws simulation k will use -- the model and the other agent's streams
// advance by exactly depth_limit + 1 words per simulation that does not
// terminate (mcts.py:315-328, 405-452: the tree levels plus the rollout reach
// the depth limit), and the belief stream by one -- into one of kSpecSlots LDS
// slots; the search wave checks the slot's counters against its own at the
// start of the simulation and reads a level's steps out of the slot instead of
// computing them (a mismatch, after a terminated simulation: it computes them
// as before and re-bases the producers' prediction).
constexpr int kSpecLevels = 3;
constexpr int kSpecProducers = PB_SPEC_PRODUCERS;
constexpr int kSpinMax = 1 << 22;   // s_sleep 1 polls (~0.1 s) before a hand-off counts as broken
constexpr int kSpecSlots = PB_SPEC_SLOTS;
__host__ __device__ constexpr int spec_entries(int A) { return A + A * A + A * A * A; }
enum : int { SP_NEXT = 0, SP_CONSUMED = 1, SP_STOP = 2, SP_SYNC_K = 3, SP_SYNC_M = 4, SP_SYNC_O = 5 };

// wave-uniform (the whole wave reads the same word): scalar branches on it
__device__ __forceinline__ int lds_acquire(int* x) {
  return uni(__hip_atomic_load(x, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_release(int* x, int v) {
  __hip_atomic_store(x, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One RNG stream as a VGPR page of 64 consecutive draws (philox.h: draw j =
// word j & 3 of block j >> 2): lane i holds draw base + i; a draw is one
// readlane, a refill (every 64 draws) one Philox block per lane.
struct VStream {
  uint32_t w;      // lane i: draw base + i
  uint32_t base;   // first draw in w (ctr - 64 initially: nothing held)
  uint32_t ctr;    // next draw
};

__device__ __forceinline__ void vs_fill(VStream& s, uint64_t seed, uint32_t tkey, uint32_t sid) {
  const uint32_t base = s.ctr & ~63u;
  const uint32_t i = (uint32_t)lane_id();
  uint32_t c[4] = {(base >> 2) + (i >> 2), 0u, sid, (uint32_t)(seed >> 32)};
  philox4x32(c, (uint32_t)seed, tkey);
  const uint32_t q = i & 3u;
  s.w = q == 0u ? c[0] : (q == 1u ? c[1] : (q == 2u ? c[2] : c[3]));
  s.base = base;
}

__device__ __forceinline__ uint32_t vs_next(VStream& s, uint64_t seed, uint32_t tkey, uint32_t sid) {
  if (s.ctr - s.base >= 64u) vs_fill(s, seed, tkey, sid);
  const uint32_t j = s.ctr++;
  return rlu(s.w, (int)(j - s.base));
}

__device__ __forceinline__ uint4 rl4(uint4 v, int l) {
  return make_uint4(rlu(v.x, l), rlu(v.y, l), rlu(v.z, l), rlu(v.w, l));
}

template <class Env, int SEL, int NA, int NP>
__global__ __launch_bounds__(64 * (NP + 1)) void k_search_lds(DevParams p, int num_sims, int final_sel) {
  static_assert(NA >= 2 && NA <= kMaxA, "action count");
  static_assert(NA * NA * NA <= 2 * kWave, "step tree: two level-2 passes");
  constexpr int A = NA;   // == p.A (host dispatch)
  constexpr int C = lds_pool_blocks(A, NP);
  constexpr int NE = spec_entries(A);
  __shared__ typename Env::Model sm;
  // step-tree slots: {n0, n1, obs key lo, obs key hi | done << 31} and the reward
  __shared__ uint4 sp_e[NP > 0 ? kSpecSlots * NE : 1];
  __shared__ double sp_r[NP > 0 ? kSpecSlots * NE : 1];
  // per slot: simulation + 1, model / other counters, -, the simulation's particle {t, v0, v1}, -
  __shared__ int sp_hdr[kSpecSlots * 8];
  __shared__ int sp_ctl[8];
  __shared__ uint4 pool[C * 8 * A];
  __shared__ uint4 path[(kMaxPath + 1) * 3];
  __shared__ double dpw[kLdsDpow];
  __shared__ uint4 bel[kLdsBelief];
  // the node of LDS block b: nl_n[b] = N of its next arrival (its visits + 1),
  // nl_v[b] = math.log(N) (pomcp_device.h node line bytes 20..31)
  __shared__ double nl_v[C];
  __shared__ int32_t nl_n[C];
  stage_model(p.model, sm);
  const int tree = (int)blockIdx.x;   // grid = B workgroups: the search wave + NP producers
  const int lane = lane_id();
  const int wv = (int)(threadIdx.x >> 6);   // 0: the search wave
  const int al = lane >> 3 < A ? lane >> 3 : A - 1;   // this lane's action group
  const int ql = lane & 7;                             // part of the action's line
  char* const an = reinterpret_cast<char*>(p.an + tree_base_lines(tree, p.Nb, blk_lines(A)));
  const int64_t blk_bytes = blk_stride_lines(blk_lines(A)) * 128;
  auto hblk = [&](int b) -> uint4* { return reinterpret_cast<uint4*>(an + (int64_t)b * blk_bytes); };
  // part q of action a's LDS line <-> the HBM block (pomcp_device.h)
  auto hld = [&](int b, int a, int q) -> uint4 {
    uint4* const x = hblk(b);
    if (q >= 2) return x[part_slot(a, q - 2)];
    const uint4 vt = x[part_vt(a)];
    return q == 0 ? make_uint4(reinterpret_cast<const uint32_t*>(x)[a], 0u, vt.x, vt.y)
                  : make_uint4(vt.z, vt.w, 0u, 0u);
  };
  auto hst = [&](int b, int a, int q, uint4 v) {
    uint4* const x = hblk(b);
    if (q >= 2) {
      x[part_slot(a, q - 2)] = v;
    } else if (q == 0) {
      reinterpret_cast<uint32_t*>(x)[a] = v.x;
      reinterpret_cast<uint2*>(x + part_vt(a))[0] = make_uint2(v.z, v.w);
    } else {
      reinterpret_cast<uint2*>(x + part_vt(a))[1] = make_uint2(v.x, v.y);
    }
  };
  auto hnode_st = [&](int b, int n, double lg) {   // the node's {visits, log(visits + 1)}
    uint32_t* const w = reinterpret_cast<uint32_t*>(hblk(b));
    w[kNodeVisByte / 4] = (uint32_t)n;
    reinterpret_cast<double*>(w)[kNodeLogByte / 8] = lg;
  };
  auto lpart = [&](int b, int a, int q) -> uint4* { return &pool[(b * A + a) * 8 + q]; };
  // b is wave-uniform: the LDS / HBM choice is a scalar branch
  auto ldp = [&](int b, int a, int q) -> uint4 { return b < C ? *lpart(b, a, q) : hld(b, a, q); };
  auto stp = [&](int b, int a, int q, uint4 v) {   // call from one lane
    if (b < C) *lpart(b, a, q) = v;
    else hst(b, a, q, v);
  };

  const TreeHdr* const h = p.hdr + tree;
  // the root belief: particle i at rbel[bdir * i] (pomcp_device.h bel_at)
  const int bdir = uni(h->belief_sel) ? -1 : 1;
  const uint4* const rbel = p.belief + (int64_t)tree * p.Nr + (uni(h->belief_sel) ? p.Nr - 1 : 0);
  int root_blk = uni(h->root_blk), root_visits = uni(h->root_visits);
  int n_blocks = uni(h->n_blocks), n_log = uni(h->n_log), n_nodes = uni(h->n_nodes);
  const int bsize = uni(h->belief_size), epoch = uni(h->epoch), root_abs = uni(h->root_abs);
  const int root_t = uni(h->root_t);
  int err = uni(h->error);
  double mm_min = uni_d(h->mm_min), mm_max = uni_d(h->mm_max);
  const uint64_t seed = uni64(h->seed);
  const uint32_t tkey = uniu(h->tree_key);
  VStream sb{0u, uniu(h->ctr[0]) - 64u, uniu(h->ctr[0])};   // belief
  VStream ss{0u, uniu(h->ctr[1]) - 64u, uniu(h->ctr[1])};   // select
  VStream sd{0u, uniu(h->ctr[2]) - 64u, uniu(h->ctr[2])};   // model
  VStream s0s{0u, uniu(h->ctr[3]) - 64u, uniu(h->ctr[3])};  // agent 0's actions
  VStream s1s{0u, uniu(h->ctr[4]) - 64u, uniu(h->ctr[4])};  // agent 1's actions
  auto d_belief = [&](uint32_t n) { return uniform_int(vs_next(sb, seed, tkey, S_BELIEF), n); };
  auto d_select = [&](uint32_t n) { return uniform_int(vs_next(ss, seed, tkey, S_SELECT), n); };
  auto d_model = [&](uint32_t n) {
    return Env::kStepDraws ? uniform_int(vs_next(sd, seed, tkey, S_MODEL), n) : 0u;
  };
  auto d_act = [&](int agent, uint32_t n) {
    return agent == 0 ? uniform_int(vs_next(s0s, seed, tkey, S_ACT_BASE), n)
                      : uniform_int(vs_next(s1s, seed, tkey, S_ACT_BASE + 1), n);
  };
  const int log0 = n_log, blocks0 = n_blocks, nodes0 = n_nodes;
  int c_rollout = 0, c_probes = 0;
#ifdef POMCP_PHASE_TIMING
  uint64_t pt[16];   // tools/phase_timing.py --kernel wave: sections of tree 0's simulations
  for (int i = 0; i < 16; ++i) pt[i] = 0;
  uint64_t pt_last = __builtin_amdgcn_s_memtime();
#endif
  LogRec* const scr = p.lscr + (int64_t)tree * p.Np;   // this launch's records, in order
  const uint32_t ltag = (uint32_t)(tree & (kWave - 1)) << kIdBits;
  OvfSlot* const ovf = p.ovf + (int64_t)tree * p.H;
  const int islots = p.islots;

  // ---- the blocks into LDS (part q of action a's line <- its HBM part)
  const int nstage = n_blocks < C ? n_blocks : C;
  if (wv == 0 && lane < 8 * A) {
    const int a = lane >> 3, q = lane & 7;
    int b = 0;
    for (; b + 4 <= nstage; b += 4) {
      const uint4 x0 = hld(b, a, q), x1 = hld(b + 1, a, q), x2 = hld(b + 2, a, q),
                  x3 = hld(b + 3, a, q);
      *lpart(b, a, q) = x0;
      *lpart(b + 1, a, q) = x1;
      *lpart(b + 2, a, q) = x2;
      *lpart(b + 3, a, q) = x3;
    }
    for (; b < nstage; ++b) *lpart(b, a, q) = hld(b, a, q);
  }
  for (int b = lane; wv == 0 && b < nstage; b += kWave) {
    const uint4 x = hblk(b)[1];
    nl_n[b] = (int)x.y + 1;
    nl_v[b] = hilo_d(x.z, x.w);
  }
  const int ndp = p.dpow_n < kLdsDpow ? p.dpow_n : kLdsDpow;
  for (int i = (int)threadIdx.x; i < ndp; i += (int)blockDim.x) dpw[i] = p.dpow[i];
  const bool bel_lds = bsize <= kLdsBelief;
  if (bel_lds)
    for (int i = (int)threadIdx.x; i < bsize; i += (int)blockDim.x) bel[i] = rbel[bdir * i];
  // the step streams are simulation-aligned (oracle/rng.py SIM_STREAMS): every
  // simulation starts the model's and both agents' action streams at a Philox
  // block boundary (counters rounded up to a multiple of 4)
  auto al4 = [](uint32_t c) { return (c + 3u) & ~3u; };
  // the step tree's prediction: simulation k of this launch draws the model and
  // the other agent's words from sync_m / sync_o + (k - sync_k) * stride, a
  // simulation that does not terminate consuming depth_limit + 1 words from an
  // aligned start (stride: that rounded up to a multiple of 4)
  const int d1 = (int)al4((uint32_t)(p.depth_limit + 1));
  const int dm = Env::kStepDraws ? d1 : 0;
  int syn_k = 0, syn_m = (int)al4(sd.ctr), syn_o = (int)al4(p.other == 0 ? s0s.ctr : s1s.ctr);
  const uint32_t bctr0 = sb.ctr;
  if (NP > 0 && threadIdx.x == 0) {
    sp_ctl[SP_NEXT] = 0;
    sp_ctl[SP_CONSUMED] = 0;
    sp_ctl[SP_STOP] = 0;
    sp_ctl[SP_SYNC_K] = syn_k;
    sp_ctl[SP_SYNC_M] = syn_m;
    sp_ctl[SP_SYNC_O] = syn_o;
    for (int i = 0; i < kSpecSlots; ++i) sp_hdr[8 * i] = 0;
  }
  __syncthreads();
  auto dpow = [&](int k) { return k < kLdsDpow ? dpw[k] : p.dpow[k]; };
  auto logtab = [&](int n) { return p.logtab[n < p.logtab_n ? n : 0]; };
  // math.log(n) from the host table, waited for (volatile: not speculated)
  auto logtab_now = [&](int n) {
    return *reinterpret_cast<const volatile double*>(p.logtab + (n < p.logtab_n ? n : 0));
  };
  auto particle = [&](uint32_t i) { return bel_lds ? bel[i] : rbel[bdir * (int)i]; };
  // the root's math.log(n): block b's entry when it holds n (the previous
  // simulation left it there), else the host table
  auto root_log = [&](int b, int n) {
    const int bc = b < C ? b : 0;
    double x = nl_v[bc];
    if (!(b < C && nl_n[bc] == n)) x = logtab_now(n);
    return x;
  };

  // ObsNode.add_child for every action (mcts.py:279-281, 318-321): a zeroed block
  auto alloc_block = [&]() -> int {
    if (n_blocks >= p.Nb) {
      err = POMCP_E_ARENA;
      return -1;
    }
    const int b = n_blocks++;
    if (b < C) {
      if (lane < 8 * A) *lpart(b, lane >> 3, lane & 7) = make_uint4(0, 0, 0, 0);
      if (lane == 0) {   // a node with no visits: N = 1, log(1) = 0
        nl_n[b] = 1;
        nl_v[b] = 0.0;
      }
    } else if (lane < blk_parts(blk_lines(A))) {
      reinterpret_cast<uint4*>(an + (int64_t)b * blk_bytes)[lane] = make_uint4(0, 0, 0, 0);
    }
    return b;
  };

  // ---- producer waves: the step tree of every coming simulation, in order
  if (NP > 0 && wv > 0) {
    const uint32_t oth_sid = (uint32_t)(S_ACT_BASE + p.other);
    for (;;) {
      // claim the next simulation (lane 0 adds 1, the other lanes 0)
      const int j = uni(__hip_atomic_fetch_add(&sp_ctl[SP_NEXT], lane == 0 ? 1 : 0, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP));
      if (j >= num_sims) break;
      // slot j % kSpecSlots is free once the search wave is done with simulation
      // j - kSpecSlots.  The search wave releases SP_STOP when it ends (or stops
      // waiting for the producers, below), so this wait always ends; the large
      // bound is a last resort only (a producer that leaves early makes the
      // search wave fall back to computing its simulations, never an error)
      bool stop = false;
      int spins = 0;
      while (lds_acquire(&sp_ctl[SP_CONSUMED]) < j - kSpecSlots + 1) {
        if (lds_acquire(&sp_ctl[SP_STOP]) != 0 || ++spins > 16 * kSpinMax) {
#ifdef POMCP_SPIN_DEBUG
          if (spins > kSpinMax && lane == 0)
            printf("producer %d: j %d consumed %d stop %d\n", wv, j, sp_ctl[SP_CONSUMED], sp_ctl[SP_STOP]);
#endif
          stop = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (stop || lds_acquire(&sp_ctl[SP_STOP]) != 0) break;
#ifdef POMCP_SPIN_DEBUG
      if (lane == 0 && j < 8) printf("producer %d: claimed %d\n", wv, j);
#endif
      const int sk = uni(lds_acquire(&sp_ctl[SP_SYNC_K]));
      const uint32_t cm = (uint32_t)uni(lds_acquire(&sp_ctl[SP_SYNC_M])) + (uint32_t)((j - sk) * dm);
      const uint32_t co = (uint32_t)uni(lds_acquire(&sp_ctl[SP_SYNC_O])) + (uint32_t)((j - sk) * d1);
      // the simulation's draws, one lane each: 0 its particle (belief.py:55),
      // 1..3 the model's shuffle draw of level 0..2, 4..6 the other agent's action
      uint32_t sid = S_BELIEF, ctr = bctr0 + (uint32_t)j;
      if (lane >= 1 && lane <= 3) {
        sid = S_MODEL;
        ctr = cm + (uint32_t)(lane - 1);
      } else if (lane >= 4) {
        sid = oth_sid;
        ctr = co + (uint32_t)(lane - 4);
      }
      const uint32_t w = philox_word(seed, tkey, sid, ctr);
      const uint4 pr = particle(uniform_int(rlu(w, 0), (uint32_t)bsize));
      uint32_t jm[kSpecLevels], ao[kSpecLevels];
#pragma unroll
      for (int l = 0; l < kSpecLevels; ++l) {
        jm[l] = Env::kStepDraws ? uniform_int(rlu(w, 1 + l), 2u) : 0u;
        ao[l] = uniform_int(rlu(w, 4 + l), (uint32_t)A);
      }
      const int slot = j % kSpecSlots;
      uint4* const E = sp_e + slot * NE;
      double* const ER = sp_r + slot * NE;
      auto put = [&](int e, uint32_t n0, uint32_t n1, double r, int dn) {
        const uint64_t ok = Env::obs_key(sm, p.ego, n0, n1);
        E[e] = make_uint4(n0, n1, (uint32_t)ok, (uint32_t)(ok >> 32) | ((uint32_t)dn << 31));
        ER[e] = r;
      };
      // levels 0 and 1: lane a0 * A + a1
      uint32_t q0 = 0u, q1 = 0u;
      if (lane < A * A) {
        const uint32_t a0 = (uint32_t)lane / A, a1 = (uint32_t)lane % A;
        uint32_t m0, m1;
        double r;
        int dn;
        Env::step(sm, p.ego, pr.y, pr.z, a0, ao[0], jm[0], &m0, &m1, &r, &dn);
        if (a1 == 0u) put((int)a0, m0, m1, r, dn);
        Env::step(sm, p.ego, m0, m1, a1, ao[1], jm[1], &q0, &q1, &r, &dn);
        put(A + lane, q0, q1, r, dn);
      }
      // level 2: entries lane and lane + 64, from level-1 state e / A
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = lane + kWave * h;
        const int pfx = e / A < A * A ? e / A : 0;
        const uint32_t x0 = (uint32_t)__shfl((int)q0, pfx), x1 = (uint32_t)__shfl((int)q1, pfx);
        if (e < A * A * A) {
          uint32_t m0, m1;
          double r;
          int dn;
          Env::step(sm, p.ego, x0, x1, (uint32_t)(e % A), ao[2], jm[2], &m0, &m1, &r, &dn);
          put(A + A * A + e, m0, m1, r, dn);
        }
      }
#ifdef POMCP_SPIN_DEBUG
      if (lane == 0 && j < 8) printf("producer %d: publish %d slot %d\n", wv, j, slot);
#endif
      if (lane == 0) {
        sp_hdr[8 * slot + 1] = (int)cm;
        sp_hdr[8 * slot + 2] = (int)co;
        sp_hdr[8 * slot + 4] = (int)pr.x;
        sp_hdr[8 * slot + 5] = (int)pr.y;
        sp_hdr[8 * slot + 6] = (int)pr.z;
        lds_release(&sp_hdr[8 * slot], j + 1);   // after every lane's entries
      }
    }
  }

  bool run = wv == 0 && err == 0 && !root_abs;   // mcts.py:270-272
  if (run && root_t == 0) {
    err = POMCP_E_STATE;
    run = false;
  }
  if (run) {
    if (root_blk < 0) root_blk = alloc_block();   // mcts.py:279-281
    if (root_blk < 0 || bsize <= 0) {
      if (err == 0) err = POMCP_E_STATE;
      run = false;
    }
  }
  if (num_sims <= 0) run = false;
  uint4 pf = make_uint4(0, 0, 0, 0);
  // the first simulation's particle (with producers: theirs, from its slot)
  if (run) {
    if (NP > 0) ++sb.ctr;
    else pf = particle(d_belief((uint32_t)bsize));
  }
  // the pending node update of the previous level's node, or of the leaf just
  // expanded: N of its next arrival and math.log(N), stored one level later,
  // when the log load has landed
  int pend_b = -1, pend_n = 0;
  double pend_v = 0.0;
  auto pend_flush = [&]() {
    if (pend_b >= 0 && lane == 0) {
      if (pend_b < C) {
        nl_v[pend_b] = pend_v;
        nl_n[pend_b] = pend_n;
      } else {
        hnode_st(pend_b, pend_n - 1, pend_v);
      }
    }
    pend_b = -1;
  };
  // the N of a node's arrival and math.log(N) (wave-uniform block)
  auto node_n = [&](int b, int* n, double* lg) {
    if (b < C) {
      *n = nl_n[b];
      *lg = nl_v[b];
    } else {
      const uint4 x = hblk(b)[1];
      *n = (int)x.y + 1;
      *lg = hilo_d(x.z, x.w);
    }
  };

  // Overflow children (beyond the inline slots) of action node ani: wave-uniform.
  struct OvfChild {
    uint32_t cid;
    int cblk, cvis;
    int32_t* cptr;
  };
  auto ovf_child = [&](uint32_t ani, uint64_t okey, int done, int cblk, int cvis) -> OvfChild {
    OvfChild o{0u, cblk, cvis, nullptr};
    const uint64_t key = okey | ((uint64_t)epoch << kEpochShift);
    uint32_t b = ovf_hash(ani, okey) & p.bucket_mask;
    bool found = false;
    for (uint32_t probe = 0; probe <= p.bucket_mask && !found; ++probe) {
      ++c_probes;
      for (int e = 0; e < kBucket; ++e) {
        OvfSlot* ep = ovf + (int64_t)b * kBucket + e;
        const uint4 w0 = reinterpret_cast<const uint4*>(ep)[0];
        const uint64_t skey = (uint64_t)w0.x | ((uint64_t)w0.y << 32);
        const bool live = (uint32_t)(skey >> kEpochShift) == (uint32_t)epoch;
        if (!live || (skey == key && w0.z == ani)) {
          if (live) {
            const uint4 w1 = reinterpret_cast<const uint4*>(ep)[1];
            o.cblk = (int)w1.x;
            o.cvis = (int)w1.y + 1;
          } else {
            ++n_nodes;
          }
          if (lane == 0) {
            reinterpret_cast<uint4*>(ep)[0] =
                make_uint4((uint32_t)key, (uint32_t)(key >> 32), ani, (uint32_t)done);
            reinterpret_cast<uint4*>(ep)[1] = make_uint4((uint32_t)o.cblk, (uint32_t)o.cvis, 0u, 0u);
          }
          o.cid = p.ovf_base + b * kBucket + (uint32_t)e;
          o.cptr = &ep->block;
          found = true;
          break;
        }
      }
      b = (b + 1) & p.bucket_mask;
    }
    if (!found) err = POMCP_E_ARENA;
    return o;
  };

  // particle-log records of this launch, buffered in VGPRs (lane i: record i
  // of the batch) and flushed to the scratch log 64 at a time: no global store
  // inside a simulation (a wait for any load would also wait for every older
  // store to be acknowledged)
  uint32_t rb_id = 0u, rb_v0 = 0u, rb_v1 = 0u;
  int rb_n = 0, rb_base = 0;
  auto flush_log = [&]() {
    if (lane < rb_n) {
      LogRec* const rp = scr + rb_base + lane;
      rp->id = rb_id;
      rp->v0 = rb_v0;
      rp->v1 = rb_v1;
    }
    rb_base += rb_n;
    rb_n = 0;
  };
  int sims = 0, max_depth = 0;
  // polls of a late hand-off before the search wave stops the producers (tests
  // shrink it: pomcp_debug_set_spin_limit)
  const int spin_max = p.spin_max > 0 ? p.spin_max : kSpinMax;
  bool sp_off = false;   // the producers were stopped (a late hand-off): compute every step
  for (int it = 0; it < num_sims && run; ++it) {
    // ------------------------------------------------ start (mcts.py:286-287)
    sd.ctr = al4(sd.ctr);   // the simulation's step streams start at a block
    s0s.ctr = al4(s0s.ctr);
    s1s.ctr = al4(s1s.ctr);
    uint4 pr = pf;                                         // belief.py:55
    if (sims + 1 < num_sims) {
      if (NP > 0) ++sb.ctr;
      else pf = particle(d_belief((uint32_t)bsize));
    }
    int depth = 0, plen = 0;
    // the step tree of this simulation (NP > 0): usable when the producers'
    // counters are this simulation's
    bool spv = false;
    int sp_base = 0, pidx = 0;
    if (NP > 0 && !sp_off) {
      const int slot = it % kSpecSlots;
      int spins = 0;
      while (lds_acquire(&sp_hdr[8 * slot]) != it + 1) {
        if (++spins > spin_max) {
          // the hand-off is late (a slow producer): stop the producers and run
          // the rest of the launch without them -- a slower search, the same
          // results (no slot is read after this)
#ifdef POMCP_SPIN_DEBUG
          if (lane == 0)
            printf("search wave: sim %d slot %d seq %d next %d consumed %d\n", it, slot,
                   sp_hdr[8 * slot], sp_ctl[SP_NEXT], sp_ctl[SP_CONSUMED]);
#endif
          if (lane == 0) lds_release(&sp_ctl[SP_STOP], 1);
          sp_off = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!sp_off) {
        const uint32_t oc = p.other == 0 ? s0s.ctr : s1s.ctr;
        spv = uniu((uint32_t)sp_hdr[8 * slot + 1]) == sd.ctr && uniu((uint32_t)sp_hdr[8 * slot + 2]) == oc;
        sp_base = slot * NE;
        pr = make_uint4((uint32_t)sp_hdr[8 * slot + 4], (uint32_t)sp_hdr[8 * slot + 5],
                        (uint32_t)sp_hdr[8 * slot + 6], 0u);   // the producer's draw of it
      }
    }
    if (NP > 0 && sp_off)   // the particle the producer would have drawn (belief.py:55)
      pr = particle(uniform_int(philox_word(seed, tkey, S_BELIEF, bctr0 + (uint32_t)it), (uint32_t)bsize));
    int t = (int)pr.x;
    uint32_t s0 = pr.y, s1 = pr.z;
    int blk = root_blk, nv = root_visits;
    double lg = root_log(root_blk, root_visits);   // math.log(nv), mcts.py:534
    double ret = 0.0;
    int phase = (0 > p.depth_limit || t > p.step_limit) ? TP_BACKUP : TP_LEVEL;   // mcts.py:315
    PT_MARK(0);
    // leaf: where its block index goes (inline slot of block lb, or an overflow entry)
    int lb = -1, la = 0, lk = 0;
    int32_t* lptr = nullptr;
    int k = 0, rdepth = 0;
    // -------------------------------------------------- the tree levels
    while (phase == TP_LEVEL) {
      const double log_n = lg;
      // every action's generative step at once (mcts.py:331-352): lane group a's
      // results for action a, from the step tree or computed here
      uint32_t n0, n1;
      double r;
      int done;
      uint64_t okey;
      uint4 v;                                             // part ql of action al's line
      if (NP > 0 && spv && depth < kSpecLevels) {
        const int e = sp_base + (depth == 0 ? 0 : (depth == 1 ? A : A + A * A)) + pidx * A + al;
        const uint4 x = sp_e[e];
        r = sp_r[e];
        v = ldp(blk, al, ql);
        PT_MARK(2);
        n0 = x.x;
        n1 = x.y;
        okey = (uint64_t)x.z | ((uint64_t)(x.w & 0x7FFFFFFFu) << 32);
        done = (int)(x.w >> 31);
        if (Env::kStepDraws) ++sd.ctr;   // the words the step tree used
        if (p.other == 0) {
          ++s0s.ctr;
        } else {
          ++s1s.ctr;
        }
      } else {
        const uint32_t j = d_model(2);                     // drawn before the selection:
        const uint32_t ao = d_act(p.other, (uint32_t)A);     // independent streams
        PT_MARK(1);
        v = ldp(blk, al, ql);
        PT_MARK(2);
        Env::step(sm, p.ego, s0, s1, (uint32_t)al, ao, j, &n0, &n1, &r, &done);
        okey = Env::obs_key(sm, p.ego, n0, n1);
      }
      PT_MARK(3);
      // _search_action_selection (mcts.py:492-563) on lanes 8a
      PT_MARK(4);
      int a = 0;
      if (SEL == POMCP_SEL_PUCB && nv == 0) {              // random.choices, uniform prior
        const double w = 1.0 / (double)A;
        double total = w;
        for (int q = 1; q < A; ++q) total = total + w;
        const double x = uniform_float(vs_next(ss, seed, tkey, S_SELECT)) * (total + 0.0);
        double acc = w;
        a = A - 1;
        for (int q = 0; q < A - 1; ++q) {
          if (x < acc) {
            a = q;
            break;
          }
          acc = acc + w;
        }
      } else if (nv == 0) {
        a = (int)d_select((uint32_t)A);
      } else if (SEL == POMCP_SEL_UNIFORM) {               // min_visit_action_selection
        int min_n = nv + 1;
#pragma unroll
        for (int q = 0; q < A; ++q) {
          const int vq = (int)rlu(v.x, 8 * q);
          if (vq < min_n) {
            min_n = vq;
            a = q;
          }
        }
      } else {
        const bool nz = mm_max > mm_min;                   // utils.py:34-39
        const double range = mm_max - mm_min;
        const int n = (int)v.x;
        const double val = hilo_d(v.z, v.w);
#ifdef PB_ABL_NOSEL
        const double nvq = val + (nz ? range : 0.0);
#else
        const double nvq = nz ? (val - mm_min) / range : val;
#endif
        double sc;
        if (SEL == POMCP_SEL_UCB) {                        // mcts.py:529-546
          if (nv >= p.logtab_n) err = POMCP_E_ARENA;
#ifdef PB_ABL_NOSEL   // ablation (results wrong, measurement only): no FP64 UCB arithmetic
          sc = nvq - (double)n;
#else
          sc = nvq + p.c * sqrt(log_n / (double)(n > 0 ? n : 1));
#endif
        } else {                                           // PUCB, mcts.py:502-527
          const double noise = 1.0 / (double)A;
          const double prior = (1.0 / (double)A) * (1.0 - p.pucb_f) + p.pucb_f * noise;
          const double sqrt_n = sqrt((double)nv);
          sc = (n > 0 ? nvq : 0.0) + p.c * prior * (sqrt_n / (double)(1 + n));
        }
        double best = rl_d(sc, 0);
#pragma unroll
        for (int q = 1; q < A; ++q) {
          const double sq = rl_d(sc, 8 * q);
          if (sq > best) {
            best = sq;
            a = q;
          }
        }
        if (SEL == POMCP_SEL_UCB) {                        // mcts.py:539-540: first unvisited
          const uint64_t unv = __ballot(ql == 0 && lane < 8 * A && v.x == 0u);
          if (unv != 0ull) a = (__ffsll((long long)unv) - 1) >> 3;
        }
      }
      PT_MARK(5);
      // ActionNode.children[obs] among the inline slots (mcts.py:356-370), every action
      const uint64_t sk = (uint64_t)v.x | ((uint64_t)v.y << 32);
      const bool slot_lane = ql >= 2 && ql - 2 < islots;
      const bool vb = (sk & kValidBit) != 0;
      const uint64_t hm = __ballot(slot_lane && (!vb || (sk & kObsMask) == okey));
      const uint64_t vm = __ballot(slot_lane && vb);
      // this node's next arrival (visits nv + 1): its log(N) into the cache
      pend_flush();
      pend_v = logtab(nv + 1);
      pend_b = blk;
      pend_n = nv + 1;
      // the chosen action's results, out of its lane group (lane g: action a's
      // step and statistics, g + 1 its total, g + 2 + k its child slot k)
      a = uni(a);   // wave-uniform (selects of uniform values end up in VGPRs)
      const int g = 8 * a;
      const uint32_t c0 = rlu(n0, g), c1 = rlu(n1, g);
      const int dn = rl(done, g);
      const uint32_t gh = (uint32_t)((hm >> (g + 2)) & 0x3Fu);
      const int ks = uni(gh != 0u ? __ffs((int)gh) - 1 : -1);
      const int sl = g + 2 + ks;
      const uint32_t ani = (uint32_t)(blk * A + a);
      uint32_t cid = 0;
      int cblk = -1, cvis = 1;
      uint4 nsl = make_uint4(0, 0, 0, 0);   // lane sl: the child slot as written
      lptr = nullptr;
      lb = -1;
      if (ks >= 0) {
        const bool match = ((vm >> sl) & 1ull) != 0ull;   // an existing child
        if (match) {
          cblk = (int)rlu(v.z, sl);
          cvis = (int)rlu(v.w, sl) + 1;
        } else {
          ++n_nodes;
        }
        const uint64_t nk = okey | kValidBit | ((uint64_t)done << 63);
        nsl = make_uint4((uint32_t)nk, (uint32_t)(nk >> 32), match ? v.z : 0xFFFFFFFFu,
                         match ? v.w + 1u : 1u);
        if (lane == sl) stp(blk, a, 2 + ks, nsl);
        cid = ani * kSlots + (uint32_t)ks + 1u;
        lb = blk;
        la = a;
        lk = ks;
      } else {
        const uint64_t ok =
            (uint64_t)rlu((uint32_t)okey, g) | ((uint64_t)rlu((uint32_t)(okey >> 32), g) << 32);
        const OvfChild o = ovf_child(ani, ok, dn, cblk, cvis);
        cid = o.cid;
        cblk = o.cblk;
        cvis = o.cvis;
        lptr = o.cptr;
      }
      if (cblk >= 0 && dn && lane == 0) {   // a done arrival at a child with a block (rare)
        if (cblk < C) {
          const int n2 = nl_n[cblk] + 1;
          nl_n[cblk] = n2;
          nl_v[cblk] = logtab_now(n2);
        } else {
          const uint4 x = hblk(cblk)[1];
          hnode_st(cblk, (int)x.y + 1, logtab_now((int)x.y + 2));
        }
      }
      PT_MARK(6);
      if (err != 0 || n_log >= p.Np || plen > kMaxPath) {
        if (err == 0) err = POMCP_E_ARENA;
        run = false;
        break;
      }
#ifdef PB_ABL_NOLOG   // ablation (results wrong, measurement only): no particle-log records
      rb_n = 0;
#endif
      if (rb_n == kWave) flush_log();
      {
        const bool mine = lane == rb_n;                      // mcts.py:371
        rb_id = mine ? (cid | ltag) : rb_id;
        rb_v0 = mine ? c0 : rb_v0;
        rb_v1 = mine ? c1 : rb_v1;
      }
      ++rb_n;
      // the path entry, written by the lanes that hold it: {visits, -, value}
      // and {total, -} of action a as they were, {block << 3 | a | done << 31, r}
      if (lane == g || lane == g + 1) {
        path[3 * plen + (lane - g)] = v;
        if (lane == g)
          path[3 * plen + 2] = make_uint4(((uint32_t)blk << 3) | (uint32_t)a | ((uint32_t)done << 31),
                                          (uint32_t)__double2loint(r), (uint32_t)__double2hiint(r), 0u);
      }
      ++n_log;
      ++plen;
      // descend (mcts.py:371-376): arrival at the child (mcts.py:315-328)
      if (dn) {
        ret = 0.0;
        phase = TP_BACKUP;
        break;
      }
      s0 = c0;
      s1 = c1;
      ++t;
      ++depth;
      if (depth > p.depth_limit || t > p.step_limit) {
        ret = 0.0;
        phase = TP_BACKUP;
      } else if (cblk < 0) {                               // mcts.py:318-328
        const int b = alloc_block();
        if (b < 0) {
          run = false;
          break;
        }
        if (lb >= 0) {
          if (lane == 8 * la + 2 + lk) stp(lb, la, 2 + lk, make_uint4(nsl.x, nsl.y, (uint32_t)b, nsl.w));
        } else if (lane == 0) {
          *lptr = b;
        }
        pend_flush();   // the leaf's own visits (cvis) and log(cvis + 1)
        pend_v = logtab(cvis + 1);
        pend_b = b;
        pend_n = cvis + 1;
        k = 0;
        rdepth = depth;   // the rollout's own depth counter (mcts.py:449)
        phase = TP_ROLL;
      } else {
        blk = cblk;   // the next level
        pidx = pidx * A + a;
        node_n(cblk, &nv, &lg);
      }
      PT_MARK(7);
      __builtin_amdgcn_wave_barrier();   // keep lane 0's LDS stores before the next reads
    }
    if (!run) break;
    // ------------------------------------------------------ the rollout
    while (phase == TP_ROLL) {                             // mcts.py:414-450
      if (!(rdepth <= p.depth_limit && t <= p.step_limit)) {
        phase = TP_BACKUP;
        break;
      }
      const uint32_t ae = d_act(p.ego, (uint32_t)A);       // search_policy.py:177
      const uint32_t j = d_model(2);
      const uint32_t ao = d_act(p.other, (uint32_t)A);     // other_policy.py:151
      uint32_t n0, n1;
      double r;
      int dn;
      Env::step(sm, p.ego, s0, s1, ae, ao, j, &n0, &n1, &r, &dn);
      if (k >= p.dpow_n) {
        err = POMCP_E_ARENA;
        run = false;
        break;
      }
      ret += dpow(k) * r;   // mcts.py:420-422
      ++c_rollout;
      if (dn) {
        phase = TP_BACKUP;
      } else {
        s0 = n0;
        s1 = n1;
        ++t;
        ++rdepth;
        ++k;
      }
    }
    if (!run) break;
    PT_MARK(8);
    // ------------------------------------------------------ backup (mcts.py:374-381)
    __builtin_amdgcn_wave_barrier();
    if (plen <= kWave) {
      // lane l < plen backs up level l: its return is the reference's chain from
      // the leaf (gr = r + discount * gr, level by level) stopped at l, then its
      // Welford update; the levels' records are distinct (a node appears once
      // per path), so all levels are written at once
      const bool mine = lane < plen;
      const int lv = mine ? lane : 0;
      // {visits, -, value} and {total, -} before, {block << 3 | a | done << 31, r}
      const uint4 e0 = path[3 * lv], e1 = path[3 * lv + 1], e2 = path[3 * lv + 2];
      const double rl = hilo_d(e2.y, e2.z);
      const uint32_t dl = e2.x >> 31;
      double gr = ret;
      for (int l = plen - 1; l >= 0; --l) {
        const double r = rl_d(rl, l);
        const double g2 = rlu(dl, l) ? r : r + p.discount * gr;
        gr = l >= lane ? g2 : gr;
      }
      const int n = (int)e0.x + 1;
      const double value0 = hilo_d(e0.z, e0.w);
      const double total = hilo_d(e1.x, e1.y) + gr;
      const double delta = gr - value0;
      const double value = value0 + delta / (double)n;
      const uint32_t ba = e2.x & 0x7FFFFFFFu;
      if (mine) {
        stp((int)(ba >> 3), (int)(ba & 7u), 0,
            make_uint4((uint32_t)n, 0u, (uint32_t)__double2loint(value), (uint32_t)__double2hiint(value)));
        stp((int)(ba >> 3), (int)(ba & 7u), 1,
            make_uint4((uint32_t)__double2loint(total), (uint32_t)__double2hiint(total), 0u, 0u));
      }
      for (int l = 0; l < plen; ++l) {   // utils.py:29-32 (min / max: any order)
        const double x = rl_d(value, l);
        if (x > mm_max) mm_max = x;
        if (x < mm_min) mm_min = x;
      }
    } else {   // a path longer than a wave (kMaxPath + 1 levels): level by level
      double gr = ret;
      for (int l = plen - 1; l >= 0; --l) {
        const uint4 e0 = path[3 * l], e1 = path[3 * l + 1], e2 = path[3 * l + 2];
        const double r = hilo_d(e2.y, e2.z);
        gr = (e2.x >> 31) ? r : r + p.discount * gr;
        const int n = (int)e0.x + 1;
        const double value0 = hilo_d(e0.z, e0.w);
        const double total = hilo_d(e1.x, e1.y) + gr;
        const double delta = gr - value0;
        const double value = value0 + delta / (double)n;
        const uint32_t ba = e2.x & 0x7FFFFFFFu;
        if (lane == 0) {
          stp((int)(ba >> 3), (int)(ba & 7u), 0,
              make_uint4((uint32_t)n, 0u, (uint32_t)__double2loint(value), (uint32_t)__double2hiint(value)));
          stp((int)(ba >> 3), (int)(ba & 7u), 1,
              make_uint4((uint32_t)__double2loint(total), (uint32_t)__double2hiint(total), 0u, 0u));
        }
        if (value > mm_max) mm_max = value;
        if (value < mm_min) mm_min = value;
      }
    }
    pend_flush();
    ++root_visits;                                          // mcts.py:288
    max_depth = depth > max_depth ? depth : max_depth;
    ++sims;
    if (NP > 0 && !sp_off) {
      // the next simulation's counters off the prediction (this one terminated
      // early): re-base the producers -- before the slot is released, so the
      // producer it frees builds its slot from the new prediction
      const uint32_t oc = al4(p.other == 0 ? s0s.ctr : s1s.ctr);   // the next one's aligned starts
      const uint32_t mc = al4(sd.ctr);
      if (mc != (uint32_t)(syn_m + (it + 1 - syn_k) * dm) ||
          oc != (uint32_t)(syn_o + (it + 1 - syn_k) * d1)) {
        syn_k = it + 1;
        syn_m = (int)mc;
        syn_o = (int)oc;
        if (lane == 0) {
          sp_ctl[SP_SYNC_M] = syn_m;
          sp_ctl[SP_SYNC_O] = syn_o;
          lds_release(&sp_ctl[SP_SYNC_K], syn_k);
        }
      }
      if (lane == 0) lds_release(&sp_ctl[SP_CONSUMED], it + 1);   // the slot is free
    }
    PT_MARK(9);
    __builtin_amdgcn_wave_barrier();
  }
#ifdef POMCP_PHASE_TIMING
  if (p.timing != nullptr && tree == 0 && wv == 0 && lane == 0)
    for (int i = 0; i < 16; ++i) p.timing[i] = pt[i];
#endif
  if (NP > 0 && wv == 0 && lane == 0) lds_release(&sp_ctl[SP_STOP], 1);   // the producers exit
  flush_log();
  __syncthreads();
  if (wv > 0) return;

  // ------------------------------------------------------------------ results
  const bool have = err == 0 && !root_abs && root_blk >= 0;
  uint4 st_l = make_uint4(0, 0, 0, 0), s1_l = st_l;
  if (have) {
    st_l = ldp(root_blk, al, 0);
    s1_l = ldp(root_blk, al, 1);
  }
  // the blocks back to HBM
  {
    const int nback = n_blocks < C ? n_blocks : C;
    if (lane < 8 * A) {
      const int a = lane >> 3, q = lane & 7;
      for (int b = 0; b < nback; ++b) hst(b, a, q, *lpart(b, a, q));
    }
    for (int b = lane; b < nback; b += kWave) hnode_st(b, nl_n[b] - 1, nl_v[b]);
  }
  // _final_action_selection (mcts.py:565-600) ends get_action; a search split
  // over several launches (final_sel = 0 for all but the last) draws it once
  // an absorbing root is not searched and get_action returns action_space[0]
  // (mcts.py:270-272); -1 = no action (an error, or not the final launch)
  int action = err == 0 && root_abs && final_sel ? 0 : -1;
  if (have && final_sel) {
    action = 0;
    uint32_t ties = 0;
    int nt = 0;
    bool direct = false;
    if (SEL == POMCP_SEL_PUCB) {
      if (root_visits == 0) {
        action = (int)d_select((uint32_t)A);
        direct = true;
      } else {
        int mx = 0;
        for (int a = 0; a < A; ++a) {
          const int na = (int)rlu(st_l.x, 8 * a);
          if (na == mx) {
            ties |= 1u << a;
            ++nt;
          } else if (na > mx) {
            mx = na;
            ties = 1u << a;
            nt = 1;
          }
        }
      }
    } else {
      double mx = -__builtin_inf();
      for (int a = 0; a < A; ++a) {
        const double va = hilo_d(rlu(st_l.z, 8 * a), rlu(st_l.w, 8 * a));
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
    if (!direct) action = kth_bit(ties, d_select((uint32_t)nt));
  }
  if (lane == 0) {
    TreeHdr* const hw = p.hdr + tree;
    hw->n_blocks = n_blocks;
    hw->n_log = n_log;
    hw->n_nodes = n_nodes;
    hw->error = err;
    hw->root_blk = root_blk;
    hw->root_visits = root_visits;
    hw->mm_min = mm_min;
    hw->mm_max = mm_max;
    hw->ctr[0] = sb.ctr;
    hw->ctr[1] = ss.ctr;
    hw->ctr[2] = sd.ctr;
    hw->ctr[3] = s0s.ctr;
    hw->ctr[4] = s1s.ctr;
  }
  pomcp_root_stats* const so = p.stats + tree;
  double* const xr = p.merge + (int64_t)tree * POMCP_XREC(A);   // exchange record (pomcp.h)
  if (lane < 8 * A && ql == 0) {   // lane 8a: action a's root child
    const int a = lane >> 3;
    const double va = hilo_d(st_l.z, st_l.w), tot = hilo_d(s1_l.x, s1_l.y);
    so->child_visits[a] = (int)st_l.x;
    so->child_values[a] = va;
    so->child_totals[a] = tot;
    xr[2 * a] = (double)st_l.x;
    xr[2 * a + 1] = tot;
  }
  if (lane == 0) {
    xr[2 * A + 0] = (double)sims;
    xr[2 * A + 1] = (double)root_visits;
    xr[2 * A + 2] = (double)max_depth;
    xr[2 * A + 3] = (double)err;
    xr[2 * A + 4] = mm_min;
    xr[2 * A + 5] = mm_max;
    so->action = action;
    so->num_sims = sims;
    so->search_depth = max_depth;
    so->root_visits = root_visits;
    so->root_absorbing = root_abs;
    so->belief_size = bsize;
    so->error = err;
    so->num_children = have ? A : 0;
    so->min_value = mm_min;
    so->max_value = mm_max;
    so->n_levels = n_log - log0;
    so->n_expansions = n_blocks - blocks0;
    so->n_new_nodes = n_nodes - nodes0;
    so->n_rollout_steps = c_rollout;
    so->n_probes = c_probes;
    so->n_obs_nodes = n_nodes;
    so->n_blocks = n_blocks;
    so->n_log = n_log;
    so->n_deferred = 0;
    so->n_cutoff = 0;          // (not counted by this kernel)
    so->n_exact_selects = 0;   // (this kernel's scores are always the exact ones)
  }
}

// After k_search_lds: append every tree's scratch records of the launch
// (stats.n_levels of them, in insertion order) to its search wave's shared
// log, trees in lane order.  A tree's records keep their order; the re-root
// (k_compact_log) separates the trees by lane tag.  One workgroup per (tree lane,
// search wave) -- grid (min(B, 64), search waves) -- copies one tree's records
// to its range (the prefix of the lower lanes' counts), so the trees of a
// batch are copied in parallel (one wave copied them in turn: 64 trees x 65,536
// simulations took ~0.1 s); k_log_merge_end then moves each log's end.
__global__ __launch_bounds__(256) void k_log_merge(DevParams p) {
  const int l = (int)blockIdx.x, sw = (int)blockIdx.y;
  __shared__ uint32_t s_off, s_n;
  if (threadIdx.x < kWave) {
    const int lane = (int)threadIdx.x;
    const int tree = sw * kWave + lane;
    const uint32_t cnt = tree < p.B ? (uint32_t)p.stats[tree].n_levels : 0u;
    uint32_t incl = cnt;   // inclusive prefix over the lanes
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
      if (lane >= o) incl += y;
    }
    const uint32_t base = uniu(p.wlog[sw]);
    if (lane == l) {
      s_off = base + incl - cnt;
      s_n = cnt;
    }
  }
  __syncthreads();
  const uint32_t n = s_n, off = s_off;
  const WaveLog wl(p.plog, p.Np, sw);
  const LogRec* const src = p.lscr + (int64_t)(sw * kWave + l) * p.Np;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) wl.store(off + i, src[i]);
}

// The end of every search wave's log after k_log_merge (a lane per search wave).
__global__ void k_log_merge_end(DevParams p, int nsw) {
  const int sw = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (sw >= nsw) return;
  uint32_t total = 0u;
  for (int l = 0; l < kWave; ++l) {
    const int tree = sw * kWave + l;
    if (tree < p.B) total += (uint32_t)p.stats[tree].n_levels;
  }
  p.wlog[sw] += total;
}

#define PB_SEARCH_LDS_INST(E, NA, NP)                                             \
  template __global__ void k_search_lds<E, POMCP_SEL_PUCB, NA, NP>(DevParams, int, int);  \
  template __global__ void k_search_lds<E, POMCP_SEL_UCB, NA, NP>(DevParams, int, int);   \
  template __global__ void k_search_lds<E, POMCP_SEL_UNIFORM, NA, NP>(DevParams, int, int);
PB_SEARCH_LDS_INST(EnvDriving, 5, 0)
PB_SEARCH_LDS_INST(EnvPursuitEvasion, 4, 0)
PB_SEARCH_LDS_INST(EnvDriving, 5, kSpecProducers)
PB_SEARCH_LDS_INST(EnvPursuitEvasion, 4, kSpecProducers)
#undef PB_SEARCH_LDS_INST

}  // namespace pb
