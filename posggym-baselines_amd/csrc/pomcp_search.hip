// k_search: the POMCP simulation loop with ONE tree per lane.
//
// Replaces posggym_baselines/planning/mcts.py:269-452 (get_action, _simulate,
// _rollout, the three selection rules, the final action choice) and the
// search-side parts of node.py / belief.py / utils.py:15-42.
//
// Why one tree per lane: the per-simulation work of a tree is a serial chain
// (select -> step -> observe -> descend -> back up) with almost no data
// parallelism inside one tree (A = 5 children).  Spreading one tree over 16
// lanes (an earlier design) made every instruction of the chain do the same
// group-uniform work 16 times; here each lane runs its own tree and every
// VALU instruction advances 64 trees.
//
// What bounds it: a wave waits for the slowest of its 64 lanes at every
// dependent memory access, so the cost of an iteration of the phase loop is
// the number of memory waits in it, whatever the lanes' phases are.  Hence:
//   * the ROOT's action statistics and inline child slots live in LDS for the
//     whole launch (35 x 16 B per tree, lane-interleaved: conflict-free), its
//     action totals in registers, so the root level of every simulation costs
//     no HBM round trip;
//   * the belief particle of the NEXT simulation is prefetched when a
//     simulation starts (belief.py:55: its index only depends on the belief
//     stream's counter);
//   * one loop iteration = one level below the root + a whole rollout + the
//     backup + the start of the next simulation with its root level (LDS);
//     whenever a lane descends into an expanded node, the node line (its
//     action statistics, its own visit count and log(N)) is loaded right away
//     and consumed by the NEXT iteration, so its latency hides behind the rest
//     of this iteration; only the chosen action's child line is waited for.
//     A depth-2 simulation takes two iterations.
//   * a level's backup writes the node line only: the chosen action's visits
//     and {value, total}, the node's visits and the log(N) of its next
//     arrival (loaded during the level).  A child slot is written only when it
//     changes beyond its visit count: a new child, its block at expansion, an
//     absorbing flag flip, and the visits of a child that has no block yet and
//     lies within the depth / step limits (the next arrival there expands it
//     and needs them); a cut-off arrival writes nothing (pomcp_device.h).
//     Against the (A + 1)-line layout with {total, agg} in the action's slot
//     line (round 2) this is 2 written sectors in one line per level instead
//     of 3 in two: -11% wave memory-wait cycles and -10% L2 misses (PMC), 0 to
//     +10% simulations/s depending on the box.
// The root block is written back to HBM at the end of the launch.
//
// Block layout: pomcp_device.h ((A + 1) x 128 B lines).
// The path of the running simulation (PathEntry: the level's statistics are
// captured on the way down -- a node appears once per path and only this lane
// writes this tree -- so the backup reads no tree memory) is held in registers
// for the root and the next kRegPath levels and in p.path below them.
#pragma clang fp contract(off)

namespace pb {

constexpr int kMaxA = 5;     // LDS root cache: A <= 5 (Driving-v1 5, PursuitEvasion-v1 4)
constexpr int kTPB = 256;    // lanes per workgroup of a full launch (one workgroup per CU)
// Small launches (root-parallel trees of one planner, few batched roots) use
// one-wave workgroups so their waves spread over the CUs instead of filling
// a few of them (pomcp_capi.hip search_tpb).
constexpr int kTPBSmall = 64;
// Root cache layout: the root's {visits, -, value} of action a (always) and,
// when kRootSlotsInLds, its inline child slots[a][k].  Without the slots a tree
// needs 80 B of LDS, which leaves room for more than one workgroup per CU.
#ifndef POMCP_ROOT_SLOTS_LDS
#define POMCP_ROOT_SLOTS_LDS 1
#endif
#ifndef POMCP_WAVES_PER_EU
#define POMCP_WAVES_PER_EU 1
#endif
constexpr bool kRootSlotsInLds = POMCP_ROOT_SLOTS_LDS != 0;
constexpr int kRootParts = kMaxA * (kRootSlotsInLds ? 1 + kSlots : 1);
__host__ __device__ constexpr int rc_stats(int a) { return a; }
__host__ __device__ constexpr int rc_slot(int a, int k) { return kMaxA + a * kSlots + k; }

constexpr int kRegPath = 3;  // levels 1..kRegPath held in registers (deeper ones in p.path)
#ifndef PB_BQ_LEVELS
#define PB_BQ_LEVELS 3
#endif
constexpr int kBq = PB_BQ_LEVELS;   // levels 1..kBq: backup stores queued (pomcp_search.hip q_flush)
static_assert(kBq >= 1 && kBq <= kRegPath, "only register-path levels are queued (level() passes ql = -1 below)");
constexpr int kPre = 2 + kMaxA;   // node line parts read by a level: visits, node, {value, total}

// One level (depth >= 1) of the running simulation's path: {block << 3 |
// action | done << 31, the action's visits before, r}, {value before, total
// before}, {node line bytes 16..31 as the backup writes them: visits of action
// 4, the node's visits (this arrival counted), log(visits + 1)}.
struct PathEntry {
  uint4 e0, e1, e2;
};

// Action a's visits out of node line parts 0 and 1 (a compile-time index).
__device__ __forceinline__ uint32_t line_visits(const uint4& p0, const uint4& p1, int a) {
  return a == 0 ? p0.x : a == 1 ? p0.y : a == 2 ? p0.z : a == 3 ? p0.w : p1.x;
}

// Phase timing (diagnostics build, -DPOMCP_PHASE_TIMING): per-wave s_memtime
// deltas per loop section into p.timing[wave][16]; each mark first drains every
// outstanding memory operation, so a section is charged the waits it issued.
#ifdef POMCP_PHASE_TIMING
#define PT_MARK(slot)                                          \
  do {                                                         \
    __builtin_amdgcn_s_waitcnt(0);                             \
    const uint64_t pt_now_ = __builtin_amdgcn_s_memtime();     \
    pt[slot] += pt_now_ - pt_last;                             \
    pt_last = pt_now_;                                         \
  } while (0)
#elif defined(POMCP_ASM_MARKS)   // analysis builds (-S): section markers in the assembly
#define PT_MARK(slot) asm volatile(";@@MARK " #slot)
#else
#define PT_MARK(slot) \
  do {                \
  } while (0)
#endif

enum : int { TP_LEVEL = 0, TP_ROLL = 1, TP_BACKUP = 2, TP_START = 3, TP_DONE = 4 };

// TM = 1: the type-based search of POTMMCP (potmmcp.py:164-301) with
// fixed-distribution policies (pomcp_device.h TmTables): per simulation an ego
// policy drawn from the meta-policy row of the particle's other-agent policy
// (sample_policy, potmmcp.py:381-389); the other agent acts by its particle's
// policy, rollouts by the drawn ego policy; PUCB's prior is the node's
// action_probs (a prior line per block), moved towards the drawn policy's
// distribution on every arrival at an existing child (potmmcp.py:255-264).
template <class Env, int SEL, int NA, int TPB, int TM>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(POMCP_WAVES_PER_EU, POMCP_WAVES_PER_EU))) void k_search(DevParams p, int num_sims, int final_sel) {
  static_assert(NA >= 2 && NA <= kMaxA, "action count");
  __shared__ typename Env::Model sm;
  __shared__ uint4 rc[kRootParts][TPB];   // the root block of every lane's tree
  stage_model(p.model, sm);
  const int lid = (int)threadIdx.x;
  const int lane = lid & (kWave - 1);
#ifdef PB_XCD_REMAP   // measurement builds: workgroups of one XCD (dispatched round-robin) on one contiguous eighth of the trees
  const int nwg = (int)gridDim.x;
  const int bx = nwg % 8 == 0 ? (int)((blockIdx.x & 7u) * (unsigned)(nwg / 8) + (blockIdx.x >> 3)) : (int)blockIdx.x;
#else
  const int bx = (int)blockIdx.x;
#endif
  const int wave = bx * (TPB / kWave) + (int)(threadIdx.x >> 6);
  const int tree = wave * kWave + lane;
  const bool valid = tree < p.B;
  const int tt = valid ? tree : 0;
  constexpr int A = NA;   // == p.A (host dispatch)
  constexpr int L = blk_lines(NA, TM);   // == p.lines
  // this tree's blocks: interleaved with the wave's other trees (pomcp_device.h)
  char* const an = reinterpret_cast<char*>(p.an + tree_base_lines(tt, p.Nb, L));
  const int64_t blk_bytes = blk_stride_lines(L) * 128;   // block b at an + b * blk_bytes
  // the wave's shared particle log (pomcp_device.h LogRec), appended at the
  // per-wave LDS counter wcnt (below)
  const WaveLog wl(p.plog, p.Np, wave, TM);
  // TM: the policy tables staged in LDS (every draw and prior reads them)
  __shared__ __attribute__((aligned(16))) char tm_lds[TM != 0 ? sizeof(TmTables) : 16];
  if constexpr (TM != 0) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(p.tmt);
    uint32_t* dst = reinterpret_cast<uint32_t*>(tm_lds);
    for (int i = (int)threadIdx.x; i < (int)(sizeof(TmTables) / 4); i += TPB) dst[i] = src[i];
    __syncthreads();
  }
  const TmTables* const tmt = reinterpret_cast<const TmTables*>(tm_lds);
  uint32_t pid = 0;   // TM: the running simulation's other-agent policy (its particle's)
  int epol = 0;       // TM: the ego policy drawn for it
  const int islots = p.islots;   // kSlots (fewer: overflow-map tests)
  const uint32_t wpos0 = p.wlog[wave];
  bool app = false;          // this lane has a record to append
  LogRec rec = {0u, 0u, 0u};
  // A lane's particle-log record (mcts.py:371) waits in `rec` and is stored
  // inside the NEXT level, after that level's child-line loads: vmcnt
  // completes in order on gfx950, so a store issued before a load makes the
  // wait for that load also wait for the store's acknowledgement (appended
  // right after a level, the record delayed the next child-line wait: +5%
  // simulations/s).  The level code is divergent, so positions
  // come from a per-wave LDS counter (one ds_add per active set, lanes in
  // lane order); each lane's records stay in its insertion order.
  __shared__ uint32_t wcnt[TPB / kWave];
  if (lane == 0) wcnt[threadIdx.x >> 6] = wpos0;
  __builtin_amdgcn_wave_barrier();
  auto append = [&]() {
    if (app) {
#ifndef POMCP_ABLATE_LOG   // ablation build only: no particle-log stores
      const uint32_t at = atomicAdd(&wcnt[threadIdx.x >> 6], 1u);
      wl.store(at, rec);
      if constexpr (TM != 0) wl.aux[at] = pid;
#endif
      app = false;
    }
  };
  OvfSlot* const ovf = p.ovf + (int64_t)tt * p.H;
  PathEntry* const path = reinterpret_cast<PathEntry*>(p.path) + (int64_t)tt * kMaxPath;
  const TreeHdr* const h = p.hdr + tt;
  // the root belief: particle i at rbel[bdir * i] (pomcp_device.h bel_at)
  const int bdir = h->belief_sel ? -1 : 1;
  const uint4* const rbel = p.belief + (int64_t)tt * p.Nr + (h->belief_sel ? p.Nr - 1 : 0);
  int root_blk = h->root_blk, root_visits = h->root_visits;
  int n_blocks = h->n_blocks, n_log = h->n_log, n_nodes = h->n_nodes;
  const int bsize = h->belief_size, epoch = h->epoch, root_abs = h->root_abs;
  int err = h->error;
  double mm_min = h->mm_min, mm_max = h->mm_max;
  // every tree of a context has the same seed (pomcp_create / pomcp_rekey): as a
  // wave-uniform value the Philox key word k0 and its schedule live in SGPRs
  const uint64_t seed = uni64(h->seed);
  const uint32_t tkey = h->tree_key;
  uint32_t c_bel = h->ctr[0], c_sel = h->ctr[1], c_mod = h->ctr[2], c_a0 = h->ctr[3],
           c_a1 = h->ctr[4];
  const int log0 = n_log, blocks0 = n_blocks, nodes0 = n_nodes;
  int c_rollout = 0, c_probes = 0, c_cut = 0, c_exact = 0;
#ifdef POMCP_PHASE_TIMING
  uint64_t pt[16];
  for (int i = 0; i < 16; ++i) pt[i] = 0;
  uint64_t pt_last = __builtin_amdgcn_s_memtime();
#endif

  // ---- RNG streams (philox.h): one stateless Philox block per draw
  auto d_belief = [&](uint32_t n) { return uniform_int(philox_word(seed, tkey, S_BELIEF, c_bel++), n); };
  auto d_select = [&](uint32_t n) { return uniform_int(philox_word(seed, tkey, S_SELECT, c_sel++), n); };
  // (counters updated by selects: increments in the branches of a condition
  // become a store through a selected pointer, i.e. scratch memory)
  auto d_act_word = [&](int agent) {
    const bool a0 = agent == 0;
    const uint32_t j = a0 ? c_a0 : c_a1;
    c_a0 += a0 ? 1u : 0u;
    c_a1 += a0 ? 0u : 1u;
    return philox_word(seed, tkey, (uint32_t)S_ACT_BASE + (a0 ? 0u : 1u), j);
  };
  // The step streams (the model's shuffle draw, the other agent's action) are
  // simulation-aligned (oracle/rng.py SIM_STREAMS): every simulation starts
  // them at a Philox block boundary, so the words of its first four steps come
  // from ONE block per stream -- one block per stream and simulation instead of
  // one per draw (DESIGN.md §4 "Simulation-aligned streams").  The next
  // simulation's blocks are computed speculatively while the first level's
  // node line is in flight (spec_blocks, after the root level: a simulation
  // that draws 1..4 words of a stream starts the next one block further on);
  // the simulation's words live in LDS (rw, [stream][word][lane]: registers
  // spilled to AGPRs cost more, A/B DESIGN.md §6 r5e).  A simulation that drew 0
  // or more than 4 words of a stream recomputes at the next start (divergent,
  // rare), and a fifth step of a simulation draws its word on its own.  The
  // belief stream keeps its one-draw lookahead, computed while a level's loads
  // are in flight (la_bel); the stored counter excludes that word.
  __shared__ uint32_t rw[2][4][TPB];   // this simulation's words: [model, other agent][k][lane]
  uint32_t m_base = 0u, o_base = 0u;   // the aligned counters at this simulation's start
  uint32_t w_bel = 0u;
  int pend_b = 0;   // a belief lookahead word is held
  uint32_t nm0 = 0u, nm1 = 0u, nm2 = 0u, nm3 = 0u, no0 = 0u, no1 = 0u, no2 = 0u, no3 = 0u;
  uint32_t nm_base = 0xFFFFFFFFu, no_base = 0xFFFFFFFFu;   // the speculated blocks' counters
  auto spec_blocks = [&]() {   // the next simulation's, assuming this one draws 1..4 words
    const uint32_t cm = m_base + 4u, co = o_base + 4u;
    uint32_t bo[4] = {co >> 2, 0u, (uint32_t)(S_ACT_BASE + p.other), (uint32_t)(seed >> 32)};
    philox4x32(bo, (uint32_t)seed, tkey);
    no0 = bo[0];
    no1 = bo[1];
    no2 = bo[2];
    no3 = bo[3];
    no_base = co;
    if constexpr (Env::kStepDraws) {
      uint32_t bm[4] = {cm >> 2, 0u, (uint32_t)S_MODEL, (uint32_t)(seed >> 32)};
      philox4x32(bm, (uint32_t)seed, tkey);
      nm0 = bm[0];
      nm1 = bm[1];
      nm2 = bm[2];
      nm3 = bm[3];
      nm_base = cm;
    }
  };
  auto sim_blocks = [&]() {   // a simulation starts: align, take (or compute) its blocks
    c_mod = (c_mod + 3u) & ~3u;
    c_a0 = (c_a0 + 3u) & ~3u;
    c_a1 = (c_a1 + 3u) & ~3u;
    const uint32_t co = p.other == 0 ? c_a0 : c_a1;
    const bool hit = co == no_base && (!Env::kStepDraws || c_mod == nm_base);
    if (!hit) {   // (divergent: the first simulation, or one that drew 0 or > 4 words)
      uint32_t bo[4] = {co >> 2, 0u, (uint32_t)(S_ACT_BASE + p.other), (uint32_t)(seed >> 32)};
      philox4x32(bo, (uint32_t)seed, tkey);
      no0 = bo[0];
      no1 = bo[1];
      no2 = bo[2];
      no3 = bo[3];
      if constexpr (Env::kStepDraws) {
        uint32_t bm[4] = {c_mod >> 2, 0u, (uint32_t)S_MODEL, (uint32_t)(seed >> 32)};
        philox4x32(bm, (uint32_t)seed, tkey);
        nm0 = bm[0];
        nm1 = bm[1];
        nm2 = bm[2];
        nm3 = bm[3];
      }
    }
    o_base = co;
    m_base = c_mod;
    rw[0][0][lid] = nm0;
    rw[0][1][lid] = nm1;
    rw[0][2][lid] = nm2;
    rw[0][3][lid] = nm3;
    rw[1][0][lid] = no0;
    rw[1][1][lid] = no1;
    rw[1][2][lid] = no2;
    rw[1][3][lid] = no3;
  };
  // word k of this simulation's block of stream q (0 model, 1 the other
  // agent's), else (k >= 4) a block of its own
  auto blk_word = [&](int q, uint32_t k, uint32_t sid, uint32_t j) -> uint32_t {
    uint32_t x = rw[q][k & 3u][lid];
    if (k >= 4u) x = philox_word(seed, tkey, sid, j);
    return x;
  };
  auto la_bel = [&]() {
    if (!pend_b) {
      w_bel = philox_word(seed, tkey, S_BELIEF, c_bel++);
      pend_b = 1;
    }
  };
  // the other agent's action (mcts.py:602-615): uniform (RandomOtherAgentPolicy)
  // or, TM, by its particle's policy (OtherAgentMixturePolicy.sample_action)
  auto take_oth = [&]() -> uint32_t {
    const bool o0 = p.other == 0;
    const uint32_t j = o0 ? c_a0 : c_a1;
    const uint32_t w = blk_word(1, j - o_base, (uint32_t)S_ACT_BASE + (o0 ? 0u : 1u), j);
    c_a0 += o0 ? 1u : 0u;
    c_a1 += o0 ? 0u : 1u;
    if constexpr (TM != 0) {
      if (tmt->other_uniform) return uniform_int(w, (uint32_t)A);
      return (uint32_t)tm_choice(tmt->oth_cum[pid], tmt->oth_tot[pid], A, w);
    } else {
      return uniform_int(w, (uint32_t)A);
    }
  };
  auto take_mod = [&](uint32_t n) -> uint32_t {
    if constexpr (Env::kStepDraws) {
      const uint32_t w = blk_word(0, c_mod - m_base, (uint32_t)S_MODEL, c_mod);
      ++c_mod;
      return uniform_int(w, n);
    } else {
      return 0u;
    }
  };
  // ObsNode.add_child for every action (mcts.py:279-281, 318-321): zeroed block
  // (TM: its prior line = the action_probs of prior code `code`)
  auto alloc_block = [&](int code) -> int {
    if (n_blocks >= p.Nb) {
      err = POMCP_E_ARENA;
      return -1;
    }
    const int b = n_blocks++;
    uint4* d = reinterpret_cast<uint4*>(an + (int64_t)b * blk_bytes);
    for (int q = 0; q < blk_parts(A + 1); ++q) d[q] = make_uint4(0, 0, 0, 0);
    if constexpr (TM != 0) {
      double* const pr = reinterpret_cast<double*>(d + part_prior(A));
      for (int q = 0; q < A; ++q) pr[q] = tmt->prior[code][q];
    }
    return b;
  };

  // _search_action_selection (mcts.py:492-563) over the statistics st[] of a
  // node with nv visits; log_n = math.log(nv) (host table, prefetched).  The
  // children's scores are computed branch-free (independent chains the wave
  // issues back to back); the strict '>' scan in action order is kept.
  // ap: the node's action_probs (TM; the uniform prior otherwise).
  auto select_action = [&](const uint4 (&st)[kMaxA], int nv, double log_n,
                           const double (&ap)[kMaxA]) -> int {
    int a = 0;
    if (SEL == POMCP_SEL_PUCB && nv == 0) {   // random.choices over the node's prior
      double cum[kMaxA], acc = 0.0;
#pragma unroll
      for (int q = 0; q < kMaxA; ++q) {
        const double w = TM != 0 ? ap[q] : 1.0 / (double)A;
        acc = q == 0 ? w : acc + w;
        cum[q] = acc;
      }
      const double x = uniform_float(philox_word(seed, tkey, S_SELECT, c_sel++)) * (cum[A - 1] + 0.0);
      a = A - 1;
      for (int q = 0; q < A - 1; ++q) {
        if (x < cum[q]) {
          a = q;
          break;
        }
      }
    } else if (nv == 0) {
      a = (int)d_select((uint32_t)A);
    } else if (SEL == POMCP_SEL_UNIFORM) {   // min_visit_action_selection
      int min_n = nv + 1;
#pragma unroll
      for (int q = 0; q < A; ++q) {
        if ((int)st[q].x < min_n) {
          min_n = (int)st[q].x;
          a = q;
        }
      }
    } else {
      const bool nz = mm_max > mm_min;   // utils.py:34-39
      const double range = mm_max - mm_min;
      double sc[A];
      bool exact = true;   // sc[] holds the reference's scores (else a is decided)
      if (SEL == POMCP_SEL_UCB) {          // mcts.py:529-546
        if (nv >= p.logtab_n) err = POMCP_E_ARENA;
#ifdef POMCP_ABLATE_SELECT   // ablation build only (tools/ablate.sh): no FP64 div / sqrt, breaks parity
#pragma unroll
        for (int q = 0; q < A; ++q)
          sc[q] = hilo_d(st[q].z, st[q].w) + p.c * log_n * (double)(int)st[q].x;
#else
        // Fast scores: (v - min) * rcp(range) + c sqrt(log N) rsq(n), each
        // within a few ulp of the reference's (v - min) / range + c
        // sqrt(log N / n) (rcp_nr / rsq_nr: |fast - exact| < ~1e-14 (|q| + e)).
        // When the leader beats every action with different statistics by
        // more than 1e-12 of their magnitudes, the reference's strict '>'
        // scan picks the same action; otherwise (~6e-4 of selections, mostly
        // exact ties of different statistics) the exact scores decide.
        // Actions with equal statistics have equal scores either way (the
        // first of them wins in both).
        {
          const double rr = nz ? rcp_nr(range) : 1.0;
          const double csl = p.c * sqrt_fast(log_n);
          double sf[A], mg[A];
#pragma unroll
          for (int q = 0; q < A; ++q) {
            const double v = hilo_d(st[q].z, st[q].w);
            const int n = (int)st[q].x > 0 ? (int)st[q].x : 1;
            const double qf = nz ? (v - mm_min) * rr : v;
            const double ef = csl * rsq_nr((double)n);
            sf[q] = qf + ef;
            mg[q] = __builtin_fabs(qf) + ef;
          }
          int af = 0;
          double bf = sf[0], bm = mg[0];
          uint4 sb = st[0];
#pragma unroll
          for (int q = 1; q < A; ++q) {
            if (sf[q] > bf) {
              bf = sf[q];
              bm = mg[q];
              af = q;
            }
          }
#pragma unroll
          for (int q = 1; q < A; ++q) sb = sel4(q == af, st[q], sb);
          bool amb = false;
#pragma unroll
          for (int q = 0; q < A; ++q) {
            const bool same = st[q].x == sb.x && st[q].z == sb.z && st[q].w == sb.w;
            amb |= q != af && !same && !(bf - sf[q] > p.sel_margin * (mg[q] + bm));
          }
          a = af;
          exact = amb;
#ifdef POMCP_EXACT_SELECT   // measurement builds only (A/B): the exact scores always
          exact = true;
#endif
        }
        if (exact) {
#pragma unroll
          for (int q = 0; q < A; ++q) {
            const double v = hilo_d(st[q].z, st[q].w);
            const double nvq = nz ? (v - mm_min) / range : v;
            const int n = (int)st[q].x > 0 ? (int)st[q].x : 1;
            sc[q] = nvq + p.c * sqrt(log_n / (double)n);
          }
        }
#endif
      } else {                             // PUCB, mcts.py:502-527
        const double noise = 1.0 / (double)A;
        const double sqrt_n = sqrt((double)nv);
        double cp[A];   // c * prior (exact: the same operations as the reference)
#pragma unroll
        for (int q = 0; q < A; ++q)
          cp[q] = p.c * ((TM != 0 ? ap[q] : 1.0 / (double)A) * (1.0 - p.pucb_f) + p.pucb_f * noise);
#ifndef POMCP_EXACT_SELECT
        {   // fast scores, the exact ones for near-ties (as UCB above); equal
            // statistics here include the prior (type-based priors differ)
          const double rr = nz ? rcp_nr(range) : 1.0;
          double sf[A], mg[A];
#pragma unroll
          for (int q = 0; q < A; ++q) {
            const int n = (int)st[q].x;
            const double v = hilo_d(st[q].z, st[q].w);
            const double qf = n > 0 ? (nz ? (v - mm_min) * rr : v) : 0.0;
            const double ef = cp[q] * (sqrt_n * rcp_nr((double)(1 + n)));
            sf[q] = qf + ef;
            mg[q] = __builtin_fabs(qf) + __builtin_fabs(ef);
          }
          int af = 0;
          double bf = sf[0], bm = mg[0], bp = cp[0];
          uint4 sb = st[0];
#pragma unroll
          for (int q = 1; q < A; ++q) {
            if (sf[q] > bf) {
              bf = sf[q];
              bm = mg[q];
              af = q;
            }
          }
#pragma unroll
          for (int q = 1; q < A; ++q) {
            sb = sel4(q == af, st[q], sb);
            bp = q == af ? cp[q] : bp;
          }
          bool amb = false;
#pragma unroll
          for (int q = 0; q < A; ++q) {
            const bool same = st[q].x == sb.x && st[q].z == sb.z && st[q].w == sb.w && cp[q] == bp;
            amb |= q != af && !same && !(bf - sf[q] > p.sel_margin * (mg[q] + bm));
          }
          a = af;
          exact = amb;
        }
#endif
        if (exact) {
#pragma unroll
          for (int q = 0; q < A; ++q) {
            const int n = (int)st[q].x;
            const double v = hilo_d(st[q].z, st[q].w);
            const double nvq = nz ? (v - mm_min) / range : v;
            sc[q] = (n > 0 ? nvq : 0.0) + cp[q] * (sqrt_n / (double)(1 + n));
          }
        }
      }
      if (exact) {
        ++c_exact;   // (the stats' n_exact_selects: tests force and count this path)
        a = 0;
        double best = sc[0];
#pragma unroll
        for (int q = 1; q < A; ++q) {
          if (sc[q] > best) {
            best = sc[q];
            a = q;
          }
        }
      }
      if (SEL == POMCP_SEL_UCB) {   // mcts.py:539-540: the first unvisited child wins
        int unv = -1;
#pragma unroll
        for (int q = A - 1; q >= 0; --q)
          if (st[q].x == 0u) unv = q;
        if (unv >= 0) a = unv;
      }
    }
    return a;
  };

  int phase = TP_START, sims = 0, max_depth = 0;
  int t = 0, depth = 0, plen = 0, blk = 0, nvis = 0, k = 0, rdepth = 0;
  uint32_t s0 = 0, s1 = 0;
  int32_t* leaf_ptr = nullptr;   // where a leaf child's block index goes (HBM) ...
  int leaf_rc = -1;              // ... or its root-cache slot part (LDS)
  double ret = 0.0;
  uint4 pf = make_uint4(0, 0, 0, 0);   // belief particle of the next simulation
  // the root level of the running simulation: {a | done << 31, visits before},
  // r, value before, total before
  int r0_on = 0;
  uint32_t r0_a = 0, r0_vis = 0;
  double r0_r = 0.0, r0_val = 0.0, r0_tot = 0.0;
  // the root's action totals: in registers for the whole launch (only the
  // backup reads or writes them), written back at the end -- a root level then
  // touches no HBM line at all
  double rt[kMaxA];
#pragma unroll
  for (int q = 0; q < kMaxA; ++q) rt[q] = 0.0;
  // TM: the root's action_probs (registers for the launch, written back at the
  // end) and the prior line of the next LEVEL pass's node (prefetched with it)
  double rap[kMaxA];
#pragma unroll
  for (int q = 0; q < kMaxA; ++q) rap[q] = 0.0;
  uint4 ppr[3] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  PathEntry rpath[kRegPath];     // levels 1..kRegPath
  uint4 pre[kPre];               // node line of the next LEVEL pass's node (parts 0 .. A + 1)
#pragma unroll
  for (int q = 0; q < kPre; ++q) pre[q] = make_uint4(0, 0, 0, 0);
  // the leaf expanded by the running simulation: its node line's bytes 16..31
  // ({0, visits, log(visits + 1)}) are written by the backup, when the log(N)
  // load issued at the expansion has long landed
  int lf_b = -1;
  uint32_t lf_nv = 0;
  double lf_ln = 0.0;
  // A simulation's backup writes of its register-path levels (node line bytes
  // 0..31 and the action's {value, total}) wait in registers and are stored
  // right after the NEXT simulation's first node-line load is issued: vmcnt
  // completes in order on gfx950, so stores issued before that load made its
  // wait also wait for their acknowledgements (as the particle-log record,
  // DESIGN.md §4 "Deferred backup stores").  That load may read the level-1
  // node the queue writes (a node is at one depth: only queue entry 0, the
  // level-1 node, can be it): its line is patched from the entry (fw_*) when
  // the level pass consumes it.  Queue entry l = path level l + 1.
  int q_n = 0;                      // queued levels (0..kBq)
  int q_b[kBq];                     // block
  uint32_t q_a[kBq];                // action
  uint4 q_s1[kBq], q_vt[kBq];       // node line part 1 as written, {value, total}
  uint32_t q_v[kBq];                // action a's visits (node line word a, a < 4)
  bool fw_on = false;               // the next level pass is depth 1: patch its line if fw_b
  int fw_b = -1;
  uint32_t fw_a = 0, fw_v = 0;
  uint4 fw_s1 = make_uint4(0, 0, 0, 0), fw_vt = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int l = 0; l < kBq; ++l) {
    q_b[l] = -1;
    q_a[l] = 0u;
    q_v[l] = 0u;
    q_s1[l] = make_uint4(0, 0, 0, 0);
    q_vt[l] = make_uint4(0, 0, 0, 0);
  }
  auto q_flush = [&]() {
#pragma unroll
    for (int l = 0; l < kBq; ++l) {
      if (l < q_n) {
        char* const lp = an + (int64_t)q_b[l] * blk_bytes;   // the node line
        if (q_a[l] < 4u) reinterpret_cast<uint32_t*>(lp)[q_a[l]] = q_v[l];
        reinterpret_cast<uint4*>(lp)[1] = q_s1[l];
        reinterpret_cast<uint4*>(lp)[part_vt((int)q_a[l])] = q_vt[l];
      }
    }
    q_n = 0;
  };
  auto logtab = [&](int n) { return p.logtab[n < p.logtab_n ? n : 0]; };

  if (!valid || err != 0 || root_abs) phase = TP_DONE;   // mcts.py:270-272
  if (phase != TP_DONE && h->root_t == 0) {
    err = POMCP_E_STATE;
    phase = TP_DONE;
  }
  if (phase != TP_DONE) {
    if (root_blk < 0) root_blk = alloc_block(h->root_code);   // mcts.py:279-281
    if (root_blk < 0 || bsize <= 0) {
      if (err == 0) err = POMCP_E_STATE;
      phase = TP_DONE;
    }
  }
  if (num_sims <= 0) phase = TP_DONE;
  const bool cached = phase != TP_DONE;   // this lane's root block is in rc[][lid]
  double root_logn = logtab(root_visits); // math.log(root visits) of the next simulation
  const uint4* const rb = reinterpret_cast<const uint4*>(an + (int64_t)(cached ? root_blk : 0) * blk_bytes);
  if (cached) {
    const uint4 p0 = rb[0], p1 = rb[1];
#pragma unroll
    for (int a = 0; a < kMaxA; ++a) {
      if (a < A) {
        const uint4 vt = rb[part_vt(a)];
        rc[rc_stats(a)][lid] = make_uint4(line_visits(p0, p1, a), 0u, vt.x, vt.y);
        if (kRootSlotsInLds) {
#pragma unroll
          for (int q = 0; q < kSlots; ++q) rc[rc_slot(a, q)][lid] = rb[part_slot(a, q)];
        }
        rt[a] = hilo_d(vt.z, vt.w);
        if constexpr (TM != 0) rap[a] = reinterpret_cast<const double*>(rb + part_prior(A))[a];
      }
    }
    pf = rbel[bdir * (int)d_belief((uint32_t)bsize)];   // the first simulation's particle
    la_bel();
  }

  // Overflow children (beyond the kSlots inline ones) of action node ani.
  // Returns its results by value: out-parameters would keep the caller's
  // locals in scratch memory.
  // TM: ncode = the prior code of a child created here; o.code = the child's.
  struct OvfChild {
    uint32_t cid;
    int cblk, cvis, code, existed;
    int32_t* cptr;
  };
  auto ovf_child = [&](uint32_t ani, uint64_t okey, int done, int cblk, int cvis,
                       int ncode) -> OvfChild {
    OvfChild o{0u, cblk, cvis, ncode, 0, nullptr};
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
            o.code = (int)((w0.w >> 1) & 15u);
            o.existed = 1;
          } else {
            ++n_nodes;
          }
          reinterpret_cast<uint4*>(ep)[0] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), ani,
                                                       (uint32_t)done | ((uint32_t)o.code << 1));
          reinterpret_cast<uint4*>(ep)[1] = make_uint4((uint32_t)o.cblk, (uint32_t)o.cvis, 0u, 0u);
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

  // The generative step of one tree level (mcts.py:331-352) for ego action a.
  // ao: the other agent's action (mcts.py:331), j: the model's exec-order
  // shuffle draw; both are drawn before the selection (their streams are
  // independent of it) so that they overlap the statistics load.
  // need_key = false: a deferred level (no child lookup, the record names the
  // action node): the observation key is not computed -- the re-root derives
  // it from the record's state (Env::obs_key in k_compact_log)
  auto tree_step = [&](int a, uint32_t ao, uint32_t j, uint32_t* n0, uint32_t* n1, double* r,
                       int* done, uint64_t* okey, bool need_key) {
    PT_MARK(15);
    Env::step(sm, p.ego, s0, s1, (uint32_t)a, ao, j, n0, n1, r, done);
    PT_MARK(9);
    *okey = 0ull;
#ifdef PB_NO_CUTKEY_SKIP   // A/B builds: the key computed at deferred levels too
    need_key = true;
#endif
    if (need_key) *okey = Env::obs_key(sm, p.ego, *n0, *n1);
    PT_MARK(11);
  };

  // ActionNode.children[obs] among the inline slots (mcts.py:356-370): filled
  // in order, so the first invalid slot is the insertion point.  -1: all taken.
  auto find_slot = [&](const uint4 (&sl)[kSlots], uint64_t okey, bool* match) -> int {
    int ks = -1;
    *match = false;
#pragma unroll
    for (int q = kSlots - 1; q >= 0; --q) {
      const uint64_t sk = (uint64_t)sl[q].x | ((uint64_t)sl[q].y << 32);
      const bool vb = (sk & kValidBit) != 0;
      if (q < islots && (!vb || (sk & kObsMask) == okey)) {
        ks = q;
        *match = vb;
      }
    }
    return ks;
  };

  // Descend into the child (mcts.py:371-376): arrival at an obs node (start of
  // _simulate, mcts.py:315-328): depth/step cutoff -> back up 0; unexpanded ->
  // expand and roll out; else select there (next LEVEL).  cvis: the child's
  // visits with this arrival when it has no block (its slot's count); code:
  // its prior code (TM: the prior line of a block allocated for it).
  auto descend = [&](int done, int cblk, int cvis, uint32_t n0, uint32_t n1, int code) {
    if (done) {
      ret = 0.0;
      phase = TP_BACKUP;
      return;
    }
    blk = cblk;
    s0 = n0;
    s1 = n1;
    ++t;
    ++depth;
    if (depth > p.depth_limit || t > p.step_limit) {   // mcts.py:315
      ret = 0.0;
      phase = TP_BACKUP;
    } else if (blk < 0) {                               // mcts.py:318-328
      const int b = alloc_block(code);
      if (b < 0) {
        phase = TP_DONE;
      } else {
        if (leaf_rc >= 0) rc[leaf_rc][lid].z = (uint32_t)b;
        else *leaf_ptr = b;
        lf_b = b;
        lf_nv = (uint32_t)cvis;
        lf_ln = logtab(cvis + 1);
        ret = 0.0;
        k = 0;
        rdepth = depth;   // the rollout's own depth counter (mcts.py:449)
        phase = TP_ROLL;
      }
    } else {   // next LEVEL pass: issue its node line now (no wait)
      phase = TP_LEVEL;
      const uint4* const cp = reinterpret_cast<const uint4*>(an + (int64_t)blk * blk_bytes);
#pragma unroll
      for (int q = 0; q < kPre; ++q) pre[q] = q < 2 + A ? cp[q] : make_uint4(0, 0, 0, 0);
      if constexpr (TM != 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q) ppr[q] = cp[part_prior(A) + q];
      }
    }
  };
  // TM: action_probs of a node += (the drawn policy's pi - them) / its visits
  // (potmmcp.py:259-264), on an arrival at an existing child
  auto prior_ema = [&](double (&ap)[kMaxA], int nv) {
#pragma unroll
    for (int q = 0; q < kMaxA; ++q)
      if (q < A) ap[q] = ap[q] + (tmt->prior[epol + 1][q] - ap[q]) / (double)nv;
  };
  // A done arrival at a child that has a block (rare: it was expanded by an
  // earlier, non-terminal arrival): ObsNode.visits += 1 in its node line.
  auto bump_node = [&](int cb) {
    q_flush();   // (rare) its line may be queued
    uint4* const c1 = reinterpret_cast<uint4*>(an + (int64_t)cb * blk_bytes) + 1;
    const uint4 x = *c1;
    const double ln = logtab((int)x.y + 2);
    *c1 = make_uint4(x.x, x.y + 1u, (uint32_t)__double2loint(ln), (uint32_t)__double2hiint(ln));
  };
  auto push_path = [&](PathEntry pe) {
    if (plen < kRegPath) {
#pragma unroll
      for (int l = 0; l < kRegPath; ++l)
        if (plen == l) rpath[l] = pe;
    } else {
      path[plen] = pe;
    }
    ++plen;
  };

  // One iteration of this uniform loop = one simulation of every lane's tree,
  // lanes in lockstep: the start and root level, then the levels below it
  // (one pass per depth while any lane still descends), the rollouts, the
  // backup.  A lane that has failed (or has no search) idles, masked.
  for (int it = 0; it < num_sims; ++it) {
    PT_MARK(7);
    // ------------------------------------- start a simulation + the root level
    if (phase == TP_START) {
      {
        const uint4 pr = pf;                                     // belief.py:55
        if (sims + 1 < num_sims) {
#ifdef POMCP_ABLATE_BELIEF   // ablation build only (tools/ablate.sh): no belief line per simulation
          pf.w += uniform_int(w_bel, (uint32_t)bsize) & 1u;
#else
          pf = rbel[bdir * (int)uniform_int(w_bel, (uint32_t)bsize)];
#endif
          pend_b = 0;
        }
        t = (int)pr.x;
        s0 = pr.y;
        s1 = pr.z;
        depth = 0;
        plen = 0;
        r0_on = 0;
        sim_blocks();   // the step streams of this simulation (oracle/rng.py SIM_STREAMS)
        if constexpr (TM != 0) {   // sample_policy (potmmcp.py:381-389), select stream
          pid = pr.w;
          if (!tmt->no_meta_draw) {   // (the base planner: one search policy, no draw)
            const int i = tm_choice(tmt->meta_cum[pid], tmt->meta_tot[pid], tmt->meta_len[pid],
                                    philox_word(seed, tkey, S_SELECT, c_sel++));
            epol = tmt->meta_idx[pid][i];
          }
        }
        if (0 > p.depth_limit || t > p.step_limit) {            // mcts.py:315
          ret = 0.0;
          phase = TP_BACKUP;
        } else {
          const uint32_t j = take_mod(2);
          const uint32_t ao = take_oth();
          uint4 st[kMaxA];
#pragma unroll
          for (int q = 0; q < kMaxA; ++q) st[q] = q < A ? rc[rc_stats(q)][lid] : make_uint4(0, 0, 0, 0);
          const int a = select_action(st, root_visits, root_logn, rap);
          uint4 sa = st[0];
          uint4 sl[kSlots];
#pragma unroll
          for (int q = 1; q < kMaxA; ++q)
            sa = sel4(q == a, st[q], sa);
#pragma unroll
          for (int q = 0; q < kSlots; ++q)
            sl[q] = kRootSlotsInLds ? rc[rc_slot(a, q)][lid] : rb[part_slot(a, q)];
          r0_tot = rt[0];
#pragma unroll
          for (int q = 1; q < kMaxA; ++q) r0_tot = q == a ? rt[q] : r0_tot;   // (selects: registers)
          uint32_t n0, n1;
          double r;
          int done;
          uint64_t okey;
#ifdef POMCP_ABLATE_ROOTSTEP   // ablation build only (measurement): no root-level model step
          n0 = s0;
          n1 = s1;
          r = 0.0;
          done = 0;
          okey = (uint64_t)ao;
#else
          tree_step(a, ao, j, &n0, &n1, &r, &done, &okey, true);
#endif
          bool match;
          const int ks = find_slot(sl, okey, &match);
          const uint32_t ani = (uint32_t)(root_blk * A + a);
          uint32_t cid = 0;
          int cblk = -1, cvis = 1, ccode = epol + 1, existed = 0;
          if (ks >= 0) {
            uint4 sk = sl[0];
#pragma unroll
            for (int q = 1; q < kSlots; ++q)
              sk = sel4(q == ks, sl[q], sk);
            // selects, not if / else: stores to different locals in the two
            // branches get merged into one store through a pointer
            cblk = match ? (int)sk.z : cblk;
            cvis = match ? (int)sk.w + 1 : cvis;
            n_nodes += match ? 0 : 1;
            existed = match ? 1 : 0;
            if (match && cblk >= 0 && done) bump_node(cblk);
            // (LDS: the slot is rewritten on every arrival; its visits are
            // meaningful while the child has no block)
            uint64_t nk = okey | kValidBit | ((uint64_t)done << 63);
            if constexpr (TM != 0) {
              ccode = match ? (int)((sk.y >> (kCodeShift - 32)) & 15u) : ccode;
              nk |= (uint64_t)ccode << kCodeShift;
            }
            const uint4 nsl = make_uint4((uint32_t)nk, (uint32_t)(nk >> 32), (uint32_t)cblk, (uint32_t)cvis);
            cid = ani * kSlots + (uint32_t)ks + 1u;
            if (kRootSlotsInLds) {
              rc[rc_slot(a, ks)][lid] = nsl;
              leaf_rc = rc_slot(a, ks);
            } else {
              uint4* slot = const_cast<uint4*>(rb) + part_slot(a, ks);
              *slot = nsl;
              leaf_ptr = reinterpret_cast<int32_t*>(slot) + 2;
              leaf_rc = -1;
            }
          } else {
            const OvfChild o = ovf_child(ani, okey, done, cblk, cvis, ccode);
            cid = o.cid;
            cblk = o.cblk;
            cvis = o.cvis;
            ccode = o.code;
            existed = o.existed;
            leaf_ptr = o.cptr;
            leaf_rc = -1;
            if (cblk >= 0 && done) bump_node(cblk);
          }
          if constexpr (TM != 0) {
            if (existed) prior_ema(rap, root_visits);
          }
          if (err != 0 || n_log >= p.Np) {
            if (err == 0) err = POMCP_E_ARENA;
            phase = TP_DONE;
          } else {
            rec = LogRec{cid | ((uint32_t)lane << kIdBits), n0, n1};   // mcts.py:371
            app = true;
            ++n_log;
            r0_on = 1;
            r0_a = (uint32_t)a | ((uint32_t)done << 31);
            r0_vis = sa.x;
            r0_r = r;
            r0_val = hilo_d(sa.z, sa.w);
            descend(done, cblk, cvis, n0, n1, ccode);
          }
        }
      }
      root_logn = logtab(root_visits + 1);   // the next simulation's (no wait)
      // the previous simulation's backup stores, after this one's first
      // node-line load (descend); entry 0 forwards to it
      fw_on = q_n > 0 && phase == TP_LEVEL;
      fw_b = q_b[0];
      fw_a = q_a[0];
      fw_v = q_v[0];
      fw_s1 = q_s1[0];
      fw_vt = q_vt[0];
      q_flush();
      PT_MARK(0);
    }
    // refill the lookahead words the root level consumed while the first level's
    // statistics line (issued by descend) is in flight
    if (phase != TP_DONE) {   // while the first level's node line is in flight
      la_bel();
      spec_blocks();
    }
    // ------------------------------------------------- the levels below the root
    while (__ballot(phase == TP_LEVEL) != 0ull) {
      if (phase == TP_LEVEL) {
        const uint4* const ap = reinterpret_cast<const uint4*>(an + (int64_t)blk * blk_bytes);
        const uint32_t j = take_mod(2);
        const uint32_t ao = take_oth();
        PT_MARK(8);
        // the node line, prefetched by descend(): this arrival's N (its visits
        // + 1) and math.log(N) are in it
        if (fw_on) {   // the line loaded before the previous backup's stores (q_flush)
          fw_on = false;
          if (blk == fw_b) {
            const uint32_t a4 = fw_a;
            pre[0] = make_uint4(a4 == 0u ? fw_v : pre[0].x, a4 == 1u ? fw_v : pre[0].y,
                                a4 == 2u ? fw_v : pre[0].z, a4 == 3u ? fw_v : pre[0].w);
            pre[1] = fw_s1;
#pragma unroll
            for (int q = 2; q < kPre; ++q) pre[q] = sel4(q == part_vt((int)a4), fw_vt, pre[q]);
          }
        }
        nvis = (int)pre[1].y + 1;
        const double log_n = hilo_d(pre[1].z, pre[1].w);
        const double lnx = logtab(nvis + 1);   // written back by the backup (no wait here)
        uint4 st[kMaxA];   // {visits, -, value} per action, as select_action reads them
  #pragma unroll
        for (int q = 0; q < kMaxA; ++q)
          st[q] = q < A ? make_uint4(line_visits(pre[0], pre[1], q), 0u, pre[part_vt(q)].x,
                                     pre[part_vt(q)].y)
                        : make_uint4(0, 0, 0, 0);
        double lap[kMaxA];   // TM: the node's action_probs (its prior line)
#pragma unroll
        for (int q = 0; q < kMaxA; ++q)
          lap[q] = TM != 0 ? hilo_d(q & 1 ? ppr[q >> 1].z : ppr[q >> 1].x, q & 1 ? ppr[q >> 1].w : ppr[q >> 1].y)
                           : 0.0;
        PT_MARK(1);
        const int a = select_action(st, nvis, log_n, lap);
        PT_MARK(2);
        uint4 sa = st[0], va = pre[part_vt(0)];
  #pragma unroll
        for (int q = 1; q < kMaxA; ++q) {
          sa = sel4(q == a, st[q], sa);
          va = sel4(q == a, pre[part_vt(q < A ? q : 0)], va);
        }
        // the chosen action's child slots (second round trip) -- except for a
        // child beyond the depth / step limits (mcts.py:315): the simulation
        // stops there whatever its slot holds, so its record is deferred
        // (pomcp_device.h: no slot read or write; the re-root materialises the
        // children that survive it).  TM looks it up: the node's prior moves
        // on arrivals at existing children (potmmcp.py:255-264).
        // (p.defer = 0, pomcp_set_defer_cutoff: the eager lookup -- cheaper re-roots)
        const bool cutc = depth + 1 > p.depth_limit || t + 1 > p.step_limit;   // mcts.py:315
        c_cut += cutc ? 1 : 0;   // (stats: n_cutoff, and n_deferred when deferring)
        const bool skipc = TM == 0 && p.defer && cutc;
        uint4 sl[kSlots];
  #pragma unroll
        for (int q = 0; q < kSlots; ++q) sl[q] = make_uint4(0, 0, 0, 0);
        if (!skipc) {
  #pragma unroll
          for (int q = 0; q < kSlots; ++q) sl[q] = ap[part_slot(a, q)];
        }
        PT_MARK(3);
        append();   // the previous level's record, after this level's loads
        uint32_t n0, n1;
        double r;
        int done;
        uint64_t okey;
        tree_step(a, ao, j, &n0, &n1, &r, &done, &okey, !skipc);
        bool match = false;
        int ks = 0;
        if (!skipc) ks = find_slot(sl, okey, &match);
        PT_MARK(12);
        const uint32_t ani = (uint32_t)(blk * A + a);
        uint32_t cid = 0;
        int cblk = -1, cvis = 1, ccode = epol + 1, existed = 0;
        leaf_rc = -1;
        if (skipc) {
          cid = p.cut_base + ani;
        } else if (ks >= 0) {
          uint4 sk = sl[0];
  #pragma unroll
          for (int q = 1; q < kSlots; ++q)
            sk = sel4(q == ks, sl[q], sk);
          cblk = match ? (int)sk.z : cblk;   // (selects, as at the root level)
          cvis = match ? (int)sk.w + 1 : cvis;
          n_nodes += match ? 0 : 1;
          existed = match ? 1 : 0;
          uint64_t nk = okey | kValidBit | ((uint64_t)done << 63);
          if constexpr (TM != 0) {
            ccode = match ? (int)((sk.y >> (kCodeShift - 32)) & 15u) : ccode;
            nk |= (uint64_t)ccode << kCodeShift;
          }
          uint4* slot = const_cast<uint4*>(ap) + part_slot(a, ks);
          // the slot changes beyond its visit count, or its count is needed
          // (no block yet, within the limits): pomcp_device.h
          const bool flip = (sk.y >> 31) != (uint32_t)done;
          if (!match || flip || (cblk < 0 && (done || !cutc)))
            *slot = make_uint4((uint32_t)nk, (uint32_t)(nk >> 32), (uint32_t)cblk, (uint32_t)cvis);
          if (match && cblk >= 0 && done) bump_node(cblk);
          cid = ani * kSlots + (uint32_t)ks + 1u;
          leaf_ptr = reinterpret_cast<int32_t*>(slot) + 2;
        } else {
          const OvfChild o = ovf_child(ani, okey, done, cblk, cvis, ccode);
          cid = o.cid;
          cblk = o.cblk;
          cvis = o.cvis;
          ccode = o.code;
          existed = o.existed;
          leaf_ptr = o.cptr;
          if (cblk >= 0 && done) bump_node(cblk);
        }
        if constexpr (TM != 0) {
          if (existed) {   // this node's action_probs move (potmmcp.py:255-264)
            prior_ema(lap, nvis);
            double* const pl = reinterpret_cast<double*>(const_cast<uint4*>(ap) + part_prior(A));
#pragma unroll
            for (int q = 0; q < kMaxA; ++q)
              if (q < A) pl[q] = lap[q];
          }
        }
        PT_MARK(13);
        if (err != 0 || n_log >= p.Np || plen >= kMaxPath) {
          if (err == 0) err = POMCP_E_ARENA;
          phase = TP_DONE;
        } else {
          rec = LogRec{cid | ((uint32_t)lane << kIdBits), n0, n1};   // mcts.py:371
          app = true;
          ++n_log;
          const uint32_t ba = ((uint32_t)blk << 3) | (uint32_t)a;   // blk < 2^26 / 30
          push_path(PathEntry{
              make_uint4(ba | ((uint32_t)done << 31), sa.x, (uint32_t)__double2loint(r),
                         (uint32_t)__double2hiint(r)),
              va,
              make_uint4(pre[1].x, (uint32_t)nvis, (uint32_t)__double2loint(lnx),
                         (uint32_t)__double2hiint(lnx))});
          PT_MARK(14);
          descend(done, cblk, cvis, n0, n1, ccode);
        }
        PT_MARK(4);
      }
    }
    append();   // the last level's record
    // ------------------------------------------------------ the rollout
    while (phase == TP_ROLL) {                               // mcts.py:414-450
      if (!(rdepth <= p.depth_limit && t <= p.step_limit)) {
        phase = TP_BACKUP;
      } else {
        // the ego's rollout action: RandomSearchPolicy (search_policy.py:177) or,
        // TM, the simulation's drawn policy (potmmcp.py:221-229)
        const uint32_t aw = d_act_word(p.ego);
        uint32_t ae;
        if constexpr (TM != 0)
          ae = tmt->ego_uniform ? uniform_int(aw, (uint32_t)A)
                                : (uint32_t)tm_choice(tmt->ego_cum[epol], tmt->ego_tot[epol], A, aw);
        else ae = uniform_int(aw, (uint32_t)A);
        const uint32_t j = take_mod(2);
        const uint32_t ao = take_oth();                       // other_policy.py:151
        uint32_t n0, n1;
        double r;
        int dn;
        Env::step(sm, p.ego, s0, s1, ae, ao, j, &n0, &n1, &r, &dn);
        if (k >= p.dpow_n) {
          err = POMCP_E_ARENA;
          phase = TP_DONE;
        } else {
          ret += p.dpow[k] * r;   // mcts.py:420-422
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
      }
      PT_MARK(5);
    }
    // ------------------------------------------------------ backup
    if (phase == TP_BACKUP) {                                // mcts.py:374-381
      double gr = ret;
      // ql >= 0: a register-path level, its stores queued as entry ql
      auto level = [&](const PathEntry& pe, int ql) {
        const uint4 e0 = pe.e0, e1 = pe.e1, e2 = pe.e2;
        const double r = hilo_d(e0.z, e0.w);
        gr = (e0.x >> 31) ? r : r + p.discount * gr;
        const int n = (int)e0.y + 1;
        const double value0 = hilo_d(e1.x, e1.y);
        const double total = hilo_d(e1.z, e1.w) + gr;
        const double delta = gr - value0;
        const double value = value0 + delta / (double)n;
        const uint32_t ba = e0.x & 0x7FFFFFFFu;
        const uint32_t a = ba & 7u;
        const uint4 s1w = make_uint4(a == 4u ? (uint32_t)n : e2.x, e2.y, e2.z, e2.w);
        const uint4 vtw = make_uint4((uint32_t)__double2loint(value), (uint32_t)__double2hiint(value),
                                     (uint32_t)__double2loint(total), (uint32_t)__double2hiint(total));
        if (ql < 0 || ql >= kBq) {
          char* const lp = an + (int64_t)(ba >> 3) * blk_bytes;   // the node line
          if (a < 4u) reinterpret_cast<uint32_t*>(lp)[a] = (uint32_t)n;
          reinterpret_cast<uint4*>(lp)[1] = s1w;
          reinterpret_cast<uint4*>(lp)[part_vt((int)a)] = vtw;
        } else {
#pragma unroll
          for (int l = 0; l < kBq; ++l) {
            if (l == ql) {
              q_b[l] = (int)(ba >> 3);
              q_a[l] = a;
              q_v[l] = (uint32_t)n;
              q_s1[l] = s1w;
              q_vt[l] = vtw;
            }
          }
        }
        if (value > mm_max) mm_max = value;   // utils.py:29-32
        if (value < mm_min) mm_min = value;
      };
      for (int l = plen - 1; l >= kRegPath; --l) level(path[l], -1);
      q_flush();   // (nothing queued: the START after the previous backup flushed)
#pragma unroll
      for (int l = kRegPath - 1; l >= 0; --l)
        if (l < plen) level(rpath[l], l);
      q_n = plen < kBq ? plen : kBq;
      if (lf_b >= 0) {   // the expanded leaf's own visits and log(N)
        reinterpret_cast<uint4*>(an + (int64_t)lf_b * blk_bytes)[1] =
            make_uint4(0u, lf_nv, (uint32_t)__double2loint(lf_ln), (uint32_t)__double2hiint(lf_ln));
        lf_b = -1;
      }
      if (r0_on) {   // the root level: statistics in LDS, totals in registers
        const int a = (int)(r0_a & 0x7FFFFFFFu);
        gr = (r0_a >> 31) ? r0_r : r0_r + p.discount * gr;
        const int n = (int)r0_vis + 1;
        const double total = r0_tot + gr;
        const double delta = gr - r0_val;
        const double value = r0_val + delta / (double)n;
        rc[rc_stats(a)][lid] = make_uint4((uint32_t)n, 0u, (uint32_t)__double2loint(value),
                                          (uint32_t)__double2hiint(value));
#pragma unroll
        for (int q = 0; q < kMaxA; ++q) rt[q] = q == a ? total : rt[q];
        if (value > mm_max) mm_max = value;
        if (value < mm_min) mm_min = value;
      }
      ++root_visits;                                          // mcts.py:288
      max_depth = depth > max_depth ? depth : max_depth;
      ++sims;
      phase = TP_START;
      PT_MARK(6);
    }
  }
#ifdef POMCP_PHASE_TIMING
  if (p.timing != nullptr && (threadIdx.x & (kWave - 1)) == 0 && wave * kWave < p.B) {
    for (int i = 0; i < 16; ++i) p.timing[wave * 16 + i] = pt[i];
  }
#endif

  q_flush();   // the last simulation's backup stores
  // ------------------------------------------------------------------ results
  {   // the wave's log length: every lane's appends of this launch
    uint32_t mine = valid ? (uint32_t)(n_log - log0) : 0u;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mine += (uint32_t)__shfl_xor((int)mine, o);
    if (lane == 0) p.wlog[wave] = wpos0 + mine;
  }
  if (!valid) return;
  if (cached) {   // write the root block back (its node line's bytes 16..31 are unused)
    uint4* const wb = const_cast<uint4*>(rb);
    uint32_t vw[kMaxA];
#pragma unroll
    for (int a = 0; a < kMaxA; ++a) {
      vw[a] = 0u;
      if (a < A) {
        const uint4 s = rc[rc_stats(a)][lid];
        vw[a] = s.x;
        wb[part_vt(a)] = make_uint4(s.z, s.w, (uint32_t)__double2loint(rt[a]), (uint32_t)__double2hiint(rt[a]));
        if (kRootSlotsInLds) {
#pragma unroll
          for (int q = 0; q < kSlots; ++q) wb[part_slot(a, q)] = rc[rc_slot(a, q)][lid];
        }
      }
    }
    wb[0] = make_uint4(vw[0], vw[1], vw[2], vw[3]);
    reinterpret_cast<uint32_t*>(wb)[4] = vw[4];
    if constexpr (TM != 0) {
#pragma unroll
      for (int a = 0; a < kMaxA; ++a)
        if (a < A) reinterpret_cast<double*>(wb + part_prior(A))[a] = rap[a];
    }
  }
  const bool have = err == 0 && !root_abs && root_blk >= 0;
  uint4 st[kMaxA];   // {visits, -, value}
  double tot[kMaxA];
  {
    const uint4* const hb = reinterpret_cast<const uint4*>(an + (int64_t)(have ? root_blk : 0) * blk_bytes);
    uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0;
    if (have && !cached) {
      p0 = hb[0];
      p1 = hb[1];
    }
#pragma unroll
    for (int a = 0; a < kMaxA; ++a) {
      st[a] = make_uint4(0, 0, 0, 0);
      tot[a] = 0.0;
      if (have && a < A) {
        if (cached) {
          st[a] = rc[rc_stats(a)][lid];
          tot[a] = rt[a];
        } else {
          const uint4 vt = hb[part_vt(a)];
          st[a] = make_uint4(line_visits(p0, p1, a), 0u, vt.x, vt.y);
          tot[a] = hilo_d(vt.z, vt.w);
        }
      }
    }
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
#pragma unroll
        for (int a = 0; a < kMaxA; ++a) {
          if (a >= A) continue;
          const int na = (int)st[a].x;
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
#pragma unroll
      for (int a = 0; a < kMaxA; ++a) {
        if (a >= A) continue;
        const double va = hilo_d(st[a].z, st[a].w);
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
  TreeHdr* const hw = p.hdr + tree;
  hw->n_blocks = n_blocks;
  hw->n_log = n_log;
  hw->n_nodes = n_nodes;
  hw->error = err;
  hw->root_blk = root_blk;
  hw->root_visits = root_visits;
  hw->mm_min = mm_min;
  hw->mm_max = mm_max;
  hw->ctr[0] = c_bel - (uint32_t)pend_b;   // draws consumed, not looked ahead
  hw->ctr[1] = c_sel;
  hw->ctr[2] = c_mod;
  hw->ctr[3] = c_a0;
  hw->ctr[4] = c_a1;
  pomcp_root_stats* const so = p.stats + tree;
  double* const xr = p.merge + (int64_t)tree * POMCP_XREC(A);   // exchange record (pomcp.h)
#pragma unroll
  for (int a = 0; a < kMaxA; ++a) {
    if (a >= A) continue;
    const double va = hilo_d(st[a].z, st[a].w);
    so->child_visits[a] = (int)st[a].x;
    so->child_values[a] = va;
    so->child_totals[a] = tot[a];
    xr[2 * a] = (double)st[a].x;
    xr[2 * a + 1] = tot[a];
  }
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
  so->n_deferred = TM == 0 && p.defer ? c_cut : 0;
  so->n_cutoff = c_cut;
  so->n_exact_selects = c_exact;
}

// Instantiated only in pomcp_search_tu.hip, the translation unit of its own
// that k_search is compiled in (its scheduler flag, build.py); the C-ABI's
// launcher takes the kernels from pb_search_kernel below.
#ifdef PB_SEARCH_TU
#define PB_SEARCH_INST(E, NA, T, TM)                                                 \
  template __global__ void k_search<E, POMCP_SEL_PUCB, NA, T, TM>(DevParams, int, int);  \
  template __global__ void k_search<E, POMCP_SEL_UCB, NA, T, TM>(DevParams, int, int);   \
  template __global__ void k_search<E, POMCP_SEL_UNIFORM, NA, T, TM>(DevParams, int, int);
PB_SEARCH_INST(EnvDriving, 5, kTPB, 0)
PB_SEARCH_INST(EnvPursuitEvasion, 4, kTPB, 0)
PB_SEARCH_INST(EnvDriving, 5, kTPBSmall, 0)
PB_SEARCH_INST(EnvPursuitEvasion, 4, kTPBSmall, 0)
PB_SEARCH_INST(EnvDriving, 5, kTPB, 1)
PB_SEARCH_INST(EnvPursuitEvasion, 4, kTPB, 1)
PB_SEARCH_INST(EnvDriving, 5, kTPBSmall, 1)
PB_SEARCH_INST(EnvPursuitEvasion, 4, kTPBSmall, 1)
#undef PB_SEARCH_INST

#endif  // PB_SEARCH_TU

}  // namespace pb

#ifdef PB_SEARCH_TU
// The k_search instantiation launched for (row = 2 * TM + small workgroups,
// environment, selection rule): pomcp_capi.hip launch_search.
__attribute__((visibility("hidden"))) const void* pb_search_kernel(int row, int e, int sel) {
  using namespace pb;
  using KFn = void (*)(DevParams, int, int);
#define PB_SEARCH_ROW(T, TM)                                                                      \
  {{k_search<EnvDriving, POMCP_SEL_PUCB, 5, T, TM>, k_search<EnvDriving, POMCP_SEL_UCB, 5, T, TM>, \
    k_search<EnvDriving, POMCP_SEL_UNIFORM, 5, T, TM>},                                           \
   {k_search<EnvPursuitEvasion, POMCP_SEL_PUCB, 4, T, TM>,                                        \
    k_search<EnvPursuitEvasion, POMCP_SEL_UCB, 4, T, TM>,                                         \
    k_search<EnvPursuitEvasion, POMCP_SEL_UNIFORM, 4, T, TM>}}
  static const KFn table[4][2][3] = {PB_SEARCH_ROW(kTPB, 0), PB_SEARCH_ROW(kTPBSmall, 0),
                                     PB_SEARCH_ROW(kTPB, 1), PB_SEARCH_ROW(kTPBSmall, 1)};
#undef PB_SEARCH_ROW
  return reinterpret_cast<const void*>(table[row][e][sel]);
}
#endif  // PB_SEARCH_TU
