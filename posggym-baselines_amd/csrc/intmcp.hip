// I-NTMCP, nesting level 1, two agents: the ego's level-1 tree and the other
// agent's level-0 tree, ONE planner pair per lane.  Nesting level 0
// (ImParams::nest0): the planner's own level-0 tree alone, held as tree 1 --
// the tree a level-1 pair keeps for its other agent -- with the planner as
// that tree's agent (p.other) and one support entry, the root belief.
//
// Replaces posggym_baselines/planning/intmcp.py:198-517, 547-593, 634-862 as
// built by INTMCP.initialize(model, ego, config, 1, None) (random search
// policies at both levels).  Restates oracle/intmcp.py, which the real
// reference pins (tests/golden/intmcp_*.json); the representation is the
// oracle's (DESIGN.md "I-NTMCP"):
//   * obs nodes are keyed by the agent's history; a node records its parent
//     edge (node, action) -- the None action of the initial observation is
//     action A -- and which of its actions are registered as children, in
//     registration order (what ObsNode.get_child_nodes() iterates);
//   * a particle of the level-1 tree carries the other agent's history as its
//     node id in the level-0 tree: created with the particle, registered on the
//     path only when the reference traverses (INTMCP.traverse, intmcp.py:797);
//   * beliefs: an append-only particle log per tree (the node a particle
//     entered), materialised at every update into the level-1 root belief and
//     the beliefs of the level-0 nodes the root belief's histories name (the
//     "support"), both ping-ponged (the previous ones are the parents of the
//     reinvigoration).
// Serial per planner pair; many pairs per launch (config 5: nested trees as a
// batched launch).  No atomics: a pair is touched by one lane.
#pragma clang fp contract(off)

namespace pb {

constexpr int kImPath = 128;          // tree levels per simulation
// Default widening factor of the bounded FP32 fast path of the other agent's
// softmax (ImPair::sample_action, ImParams::fast_slack): 1 = the proven
// bound; any value >= 1 keeps results exact, and tests widen it at run time
// (intmcp_debug_set_softmax_slack) so that the exact fallbacks run often.
#ifndef IM_FAST_SLACK
#define IM_FAST_SLACK 1.0f
#endif
constexpr int kImMaxA = 6;            // registration order: 6 x 3 bits (INode.info)
constexpr int kImRegPath = 3;         // path levels held in registers (deeper ones in p.path)
// A node: its line (128 B) = the INode {parent, info, visits, t} (16 B), the
// head {visits u32, value f64} of each action's statistics (12 B each, from
// byte 16) and, at byte 80, the cold fields (ICold: obs key, statistics
// index, support slot: never read by a simulation); and one 32 B action record per
// action (the None action A included): the action's total (ActionNode
// total_value; agg is not kept) and kImInline obs-child slots
// {obs key, child id} (id 0: empty -- a tree's node 0 is never a child).
// A node view (selection, the other agent's softmax) is its line; the chosen
// action's record is loaded right after selection, so the obs child is found
// in registers once the step has produced the observation (no probe round
// trip); a (node, action) with more than kImInline children keeps the rest in
// the per-tree hash map (IHash), probed only when the inline slots are full.
// Blocks start zeroed (the arena is cleared at create and reset; nodes are
// never reused within an episode), so statistics need no initialising writes.
constexpr int kImInline = 2;
constexpr int64_t kImLine = 128;
constexpr int64_t kImRec = 32;                              // {total f64, 2 x {okey u64, child i32}}
constexpr int64_t kImRecs = 6 * kImRec;                     // records of actions 0..5 (kImMaxA)
constexpr int64_t kImBlock = kImLine + kImRecs;             // 320 B per node (packed extraction ABI)
// Nodes are interleaved by wavefront: per wave [2 trees][Nn] slabs of W nodes
// (W = 64, fewer in a last partial wave; nt trees: [nt trees][Nn] at nesting
// level 2), each slab = the W node lines then
// the W nodes' records ([W][128 B] [W][192 B]), so the pairs of a wave keep
// node n of their trees side by side (a view load is W whole lines) and a
// wave's loads spread over the slabs in use, not over 64 separate per-pair
// arenas (fewer pages per load instruction to translate).  B x 2 x Nn x
// kImBlock bytes in all.
__host__ __device__ __forceinline__ int im_wave_width(int B, int b) {
  const int w0 = b - b % kWave;
  return B - w0 < kWave ? B - w0 : kWave;
}
__host__ __device__ __forceinline__ int64_t im_node_stride(int B, int b) {   // node n -> n + 1
  return (int64_t)im_wave_width(B, b) * kImBlock;
}
// node n's line (tree k of pair b)
__host__ __device__ __forceinline__ int64_t im_node_off(int64_t Nn, int B, int b, int k, int64_t n,
                                                       int nt) {
  const int64_t w0 = b - b % kWave;
  return w0 * nt * Nn * kImBlock + ((int64_t)k * Nn + n) * im_node_stride(B, b) + (b - w0) * kImLine;
}
// a node's action records, relative to its line
__host__ __device__ __forceinline__ int64_t im_rec_delta(int B, int b) {
  const int64_t j = b - (b - b % kWave);
  return (im_wave_width(B, b) - j) * kImLine + j * kImRecs;
}
constexpr uint32_t kImNoSupport = 0xFFFFFFFFu;
constexpr int32_t kImSkip = -2;       // intmcp_update action: leave the pair untouched
constexpr int kWave64 = 64;           // lanes of a wave (k_im_update's wave mode)
constexpr int kImLogLds = 2048;       // math.log(N) entries staged in LDS by k_im_search
constexpr int kImDpowLds = 64;        // discount powers staged in LDS by k_im_search
constexpr int kImRootWords = 7;       // the level-1 root's view (INode + <= 6 heads) in LDS, uint4s

struct INode {          // 16 B, line bytes 0-15
  int32_t parent;
  uint32_t info;        // paction:3 | absorbing:1 | path_ok:1 | nreg:3 | order 6 x 3 bits
                        // | statistics allocated:1 (bit 26)
  int32_t visits;
  int32_t t;
};
struct ICold {          // 16 B, line bytes 80-95
  uint64_t okey;
  int32_t stats;        // first of A IStat entries (-1: none registered yet)
  uint32_t support;     // support slot while materialising beliefs (level-0 tree)
};
constexpr int64_t kImHeads = 16;      // line byte of action 0's head (12 B each)
constexpr int64_t kImCold = 80;       // line byte of the ICold
constexpr uint32_t kImStatsBit = 1u << 26;
struct IStat {          // 32 B: ActionNode visits / value / total_value / agg
  int32_t visits, pad;
  double value, total, agg;
};
struct IHash {          // 16 B: (parent, action, obs key) -> child
  uint64_t okey;
  uint32_t na;          // parent << 3 | action
  int32_t child;        // -1: empty
};
struct IRec {           // particle log record: the particle (v0, v1[, other's node]) entered `node`
  uint32_t node, v0, v1, nested;
};
struct ISup {           // a materialised level-0 belief
  int32_t node, off, size, cap;
};

// Trees of a pair: nesting level L >= 1 keeps L + 1 trees, tree k the level-
// (L - k) planner's -- tree 0 the planner's own, the last (nt - 1) the level-0
// one; nesting level 1: tree 0 (the planner's level-1 tree) and tree 1 (the
// other agent's level-0 tree); level 2 (ImParams::nt = 3) adds a middle tree
// (tree 1, level 1, the other agent), level 3 two (trees 1 and 2, levels 2
// and 1), ... level L >= 2 L - 1 (trees 1 .. L - 1, levels L - 1 .. 1; built up
// to nesting level 5).  Tree k models agent ego if k is even.  The bottom
// tree's beliefs are the "support" (sup / supp); middle tree k's are
// msup[k - 1] / msupp[k - 1].
constexpr int kImMaxT = INTMCP_MAX_TREES;   // nesting levels 0 .. kImMaxT - 1
constexpr int kImMaxMid = kImMaxT - 2;      // middle trees (nesting level 5: trees 1 .. 4)
struct ImSims {                             // simulations per level of one k_im_searchN launch
  int32_t s[kImMaxT];
};
struct IHdr {
  int32_t n_nodes[kImMaxT], n_stats[kImMaxT], n_log[kImMaxT];
  int32_t cur, root_sel, root_size, sup_sel, n_sup, sup_used, err, last_action;
  int32_t num_sims, search_depth, sims_done, pad;
  // middle tree k = m + 1's beliefs: table select, entries, particles used, and
  // the previous table's entry count during an update
  int32_t msel[kImMaxMid], n_msup[kImMaxMid], msup_used[kImMaxMid], mpad[kImMaxMid];
  double mm_min[kImMaxT], mm_max[kImMaxT];
  uint64_t seed;
  uint32_t tree_key;
  uint32_t ctr[6 + kImMaxMid];   // belief (top), select, model, act0, act1, belief (level 0),
                                 // belief (middle trees 1 .. kImMaxMid)
};

struct ImParams {
  int32_t B, A, ego, other, sel, depth_limit, step_limit, n_target, extra, has_kb,
      state_belief_only,
      nest0,            // nesting level 0: only tree 1, whose agent (p.other) is the planner
      nt;               // trees per pair in the arenas: 2 (nesting levels 0, 1), else level + 1
  double discount, c, limit_factor, kb_min, kb_max;
  int64_t Nn, Ns, Nl, H, Nr, Nsp;   // per tree: nodes, stat entries, log records, hash slots;
                                    // per pair: root belief, support particles
  IHdr* hdr;
  char* nodes;          // node lines + action records (kImBlock B a node), wave-interleaved:
                        // im_node_off, im_rec_delta
  int64_t nstride;      // kImBlock (the packed block size of the extraction ABI)
  IHash* hash;          // [B][nt][H] obs children beyond a record's inline slots
  IRec* log;            // [B][nt][Nl]
  uint4* root;          // [B][2][Nr] {v0, v1, nested, support slot}
  ISup* sup;            // [B][2][Nr] the bottom (level-0) tree's beliefs
  uint2* supp;          // [B][2][Nsp]
  ISup* msup[kImMaxMid];     // [B][2][Nr] middle tree m + 1's beliefs ...
  uint4* msupp[kImMaxMid];   // [B][2][Nsp] ... {v0, v1, next tree's node, its table slot}
  double* mprob[kImMaxMid];  // [B][Nr] middle tree m + 1's history distribution
  int4* path;           // [B][kImPath][3] path of the running simulation (deep levels)
  double* prob;         // [B][Nr] support probabilities (update scratch)
  const double* logtab;
  int64_t logtab_n;
  const double* dpow;
  int32_t dpow_n;
  const void* model;
  const int32_t* in_actions;
  const uint64_t* in_obs;
  int32_t* out;         // [B][2] {root absorbing, error}
  uint64_t* out_obs;    // [B] synthetic roots
  uint64_t* timing;     // [B][kImPhases] (diagnostics build, -DPOMCP_PHASE_TIMING)
  // the other agent's softmax (sample_action): the fast path's bound is widened
  // by fast_slack (1 = the product's bound; tests widen it so the exact FP64
  // path runs on most draws, intmcp_debug_set_softmax_slack), and the exact-path
  // draws are counted when exact_draws is set (tests only)
  float fast_slack;
  // search policies (INTMCP search_policies, intmcp.py:956-971) of tree k's
  // planner for agent i: sp_fixed[k][i] = 0 RandomSearchPolicy
  // (Discrete.sample()), 1 a fixed distribution drawn as random.choices
  // (sp_cum / sp_tot, pomcp_device.h tm_choice) on the agent's action stream;
  // sp_any: some table is fixed (else the draws stay the plain uniform ones)
  int32_t sp_any;
  unsigned long long* exact_draws;
  int32_t sp_fixed[kImMaxT][2];
  double sp_cum[kImMaxT][2][kImMaxA];
  double sp_tot[kImMaxT][2];
};

// Phase timing (diagnostics build, -DPOMCP_PHASE_TIMING): per-lane s_memtime
// deltas per section of k_im_search; each mark first drains every outstanding
// memory operation, so a section is charged the waits of the loads it issued.
constexpr int kImPhases = 12;
enum : int { IP_START = 0, IP_SELECT, IP_OTHER, IP_STEP, IP_CHILD, IP_DESCEND, IP_EXPAND,
             IP_ROLLOUT, IP_BACKUP, IP_SIMEND };
#ifdef POMCP_PHASE_TIMING
#define IM_MARK(slot)                                        \
  do {                                                       \
    __builtin_amdgcn_s_waitcnt(0);                           \
    const uint64_t im_now_ = __builtin_amdgcn_s_memtime();   \
    pt[slot] += im_now_ - pt_last;                           \
    pt_last = im_now_;                                       \
  } while (0)
#define IM_MARK_P(slot)                                      \
  do {                                                       \
    __builtin_amdgcn_s_waitcnt(0);                           \
    const uint64_t im_now_ = __builtin_amdgcn_s_memtime();   \
    P.pt[slot] += im_now_ - P.pt_last;                       \
    P.pt_last = im_now_;                                     \
  } while (0)
#elif defined(POMCP_ASM_MARKS)   // analysis builds (-S): section markers in the assembly
#define IM_MARK(slot) asm volatile(";@@IMARK " #slot)
#define IM_MARK_P(slot) IM_MARK(slot)
#else
#define IM_MARK(slot) \
  do {                \
  } while (0)
#define IM_MARK_P(slot) IM_MARK(slot)
#endif

__device__ __forceinline__ uint32_t im_paction(uint32_t info) { return info & 7u; }
__host__ __device__ __forceinline__ bool im_absorbing(uint32_t info) { return (info >> 3) & 1u; }
__device__ __forceinline__ bool im_path_ok(uint32_t info) { return (info >> 4) & 1u; }
__host__ __device__ __forceinline__ int im_nreg(uint32_t info) { return (int)((info >> 5) & 7u); }
__host__ __device__ __forceinline__ int im_order(uint32_t info, int k) { return (int)((info >> (8 + 3 * k)) & 7u); }
__device__ __forceinline__ bool im_has_stats(uint32_t info) { return (info & kImStatsBit) != 0u; }

// One planner pair (lane): pointers, counters, RNG.  NT: trees per pair
// (== ImParams::nt: 2, else the nesting level + 1).
template <class Env, int NT = 2>
struct ImPair {
  using Model = typename Env::Model;
  static constexpr int kNA = Env::kA;   // == p.A (intmcp_create checks num_actions)
  static constexpr int kBot = NT - 1;   // the level-0 tree
  const ImParams& p;
  const Model& m;
  int pair;
  char* nb[NT];    // node blocks of tree k (0: the planner's)
  int64_t ns;      // node n -> n + 1 (im_node_stride)
  int64_t ro;      // node line -> its action records (im_rec_delta)
  IHash* hs[NT];
  IRec* lg[NT];
  uint4* rootb;   // [2][Nr]
  ISup* sup;      // [2][Nr] the level-0 tree's beliefs
  uint2* supp;    // [2][Nsp]
  ISup* msup[kImMaxMid];     // [2][Nr] middle tree m + 1's beliefs
  uint4* msupp[kImMaxMid];   // [2][Nsp]
  double* mprob[kImMaxMid];  // [Nr]
  int4* path;
  double* prob;   // [Nr]
  IHdr h;
  // k_im_search only: math.log(N) for N < lt_n staged in LDS, and the level-1
  // root's view (this lane's column of an [kImRootWords][64] uint4 array),
  // which only this lane's backups at the root change during a search
  const double* lt_lds = nullptr;
  int lt_n = 0;
  uint4* rv = nullptr;
  int rv_root = -1;
  // the rollout's discount powers and the exp table of the other agent's
  // softmax (k_im_search: staged in LDS)
  const double* dp = nullptr;
  const uint64_t* exp_tab = kHostExpTab;
  // k_im_search only: one-word lookahead per RNG stream.  la_fill computes the
  // next word of every stream whose last word was consumed, at points where the
  // wave waits on a load anyway; draw() consumes it.  Each stream is consumed
  // in order, so results are unchanged; stored counters exclude a computed but
  // unconsumed word (la_pend).
  uint32_t la_w[6 + kImMaxMid];
  uint32_t la_pend = 0u;
#ifdef POMCP_PHASE_TIMING
  uint64_t pt[kImPhases] = {};
  uint64_t pt_last = 0;
#endif

  __device__ ImPair(const ImParams& pp, const Model& mm, int b) : p(pp), m(mm), pair(b) {
    for (int k = 0; k < NT; ++k) {
      nb[k] = p.nodes + im_node_off(p.Nn, p.B, b, k, 0, NT);
      hs[k] = p.hash + ((int64_t)b * NT + k) * p.H;
      lg[k] = p.log + ((int64_t)b * NT + k) * p.Nl;
    }
    ns = im_node_stride(p.B, b);
    ro = im_rec_delta(p.B, b);
    rootb = p.root + (int64_t)b * 2 * p.Nr;
    sup = p.sup + (int64_t)b * 2 * p.Nr;
    supp = p.supp + (int64_t)b * 2 * p.Nsp;
#pragma unroll
    for (int m = 0; m < kImMaxMid; ++m) {
      const bool on = m < NT - 2;
      msup[m] = on ? p.msup[m] + (int64_t)b * 2 * p.Nr : nullptr;
      msupp[m] = on ? p.msupp[m] + (int64_t)b * 2 * p.Nsp : nullptr;
      mprob[m] = on ? p.mprob[m] + (int64_t)b * p.Nr : nullptr;
    }
    path = p.path + (int64_t)b * kImPath * 3;
    prob = p.prob + (int64_t)b * p.Nr;
    h = p.hdr[b];
    dp = p.dpow;
  }
  static constexpr int kCtrs = NT > 2 ? 4 + NT : 6;   // RNG streams in use (slot 5 + k: middle tree k)
  static_assert(kCtrs <= 6 + kImMaxMid, "IHdr::ctr holds every stream's counter");
  __device__ __forceinline__ uint32_t ctr_stored(int q) const { return h.ctr[q] - ((la_pend >> q) & 1u); }
  // intmcp.py:326-330 (_prune_traverse's clear_belief at every update): the
  // particles of nodes more than two steps behind the current one are dropped
  // -- nothing reads them again (a search starts at the current root, a
  // reinvigoration reads the previous step's beliefs) -- so both trees' logs
  // keep only the records of nodes with t >= cur_t - 2, in insertion order.
  // The reference clears only nodes that have children; the other old nodes'
  // beliefs are as unreachable, so they go too.  The trees stay.
  template <bool kWave>
  __device__ void clear_old_beliefs(int cur_t);
  __device__ void store() {
    IHdr o = h;
#pragma unroll
    for (int q = 0; q < kCtrs; ++q) o.ctr[q] = ctr_stored(q);
    p.hdr[pair] = o;
  }
  // what a search changes (k_im_search): the other fields need not stay live
  // in registers for the launch
  __device__ void store_search() {
    IHdr& o = p.hdr[pair];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      o.n_nodes[k] = h.n_nodes[k];
      o.n_stats[k] = h.n_stats[k];
      o.n_log[k] = h.n_log[k];
      o.mm_min[k] = h.mm_min[k];
      o.mm_max[k] = h.mm_max[k];
    }
#pragma unroll
    for (int q = 0; q < kCtrs; ++q) o.ctr[q] = ctr_stored(q);
    o.err = h.err;
    o.last_action = h.last_action;
    o.num_sims = h.num_sims;
    o.search_depth = h.search_depth;
  }

  // A node's line: the INode with the heads of its actions' statistics
  // (node.py:120-178), so a node and its statistics arrive together (they
  // used to be an index apart: two dependent loads).
  __device__ __forceinline__ INode& N(int k, int n) const {
    return *reinterpret_cast<INode*>(nb[k] + (int64_t)n * ns);
  }
  __device__ __forceinline__ ICold& C(int k, int n) const {
    return *reinterpret_cast<ICold*>(nb[k] + (int64_t)n * ns + kImCold);
  }
  __device__ __forceinline__ uint32_t* H(int k, int n, int a) const {   // {visits, value} of action a
    return reinterpret_cast<uint32_t*>(nb[k] + (int64_t)n * ns + kImHeads + 12 * (int64_t)a);
  }
  // action a's record: words 0-1 total, slot i = words 2+3i (okey lo, hi), 4+3i (child)
  __device__ __forceinline__ uint32_t* R(int k, int n, int a) const {
    return reinterpret_cast<uint32_t*>(nb[k] + (int64_t)n * ns + ro + (int64_t)a * kImRec);
  }
  struct Rec {
    uint4 w[2];
  };
  __device__ __forceinline__ Rec rec(int k, int n, int a) const {
    const uint4* r = reinterpret_cast<const uint4*>(R(k, n, a));
    Rec v;
    v.w[0] = r[0];
    v.w[1] = r[1];
    return v;
  }
  __device__ __forceinline__ void set_total(int k, int n, int a, double total) const {
    *reinterpret_cast<uint2*>(R(k, n, a)) =
        make_uint2((uint32_t)__double2loint(total), (uint32_t)__double2hiint(total));
  }
  // the node and the head of every action's statistics as {visits, -,
  // value} (entries of unregistered actions are never used): the line's
  // first 16 + 12 A bytes, ceil((16 + 12 A) / 16) loads
  struct View {
    INode x;
    uint4 sh[kNA];
  };
  static constexpr int kViewLoads = (int)((kImHeads + 12 * kNA + 15) / 16);
  __device__ __forceinline__ View view(int k, int n) const {
    const uint4* l = reinterpret_cast<const uint4*>(nb[k] + (int64_t)n * ns);
    uint32_t w[4 * kViewLoads];
#pragma unroll
    for (int i = 0; i < kViewLoads; ++i) {
      const uint4 u = l[i];
      w[4 * i] = u.x;
      w[4 * i + 1] = u.y;
      w[4 * i + 2] = u.z;
      w[4 * i + 3] = u.w;
    }
    View v;
    v.x.parent = (int32_t)w[0];
    v.x.info = w[1];
    v.x.visits = (int32_t)w[2];
    v.x.t = (int32_t)w[3];
#pragma unroll
    for (int q = 0; q < kNA; ++q) v.sh[q] = make_uint4(w[4 + 3 * q], 0u, w[5 + 3 * q], w[6 + 3 * q]);
    return v;
  }
  // the node alone (one load): a child at which the descent stops -- its
  // statistics heads would only serve a next level's selection
  __device__ __forceinline__ View view_node(int k, int n) const {
    const uint4 u = *reinterpret_cast<const uint4*>(nb[k] + (int64_t)n * ns);
    View v;
    v.x.parent = (int32_t)u.x;
    v.x.info = u.y;
    v.x.visits = (int32_t)u.z;
    v.x.t = (int32_t)u.w;
#pragma unroll
    for (int q = 0; q < kNA; ++q) v.sh[q] = make_uint4(0, 0, 0, 0);
    return v;
  }
  // a node just created (INode x, zero statistics): its view without a load
  __device__ __forceinline__ static View fresh_view(const INode& x) {
    View v;
    v.x = x;
#pragma unroll
    for (int q = 0; q < kNA; ++q) v.sh[q] = make_uint4(0, 0, 0, 0);
    return v;
  }
  __device__ void rv_put(const View& v) {
    rv[0] = make_uint4((uint32_t)v.x.parent, v.x.info, (uint32_t)v.x.visits, (uint32_t)v.x.t);
#pragma unroll
    for (int q = 0; q < kNA; ++q) rv[(1 + q) * kWave] = v.sh[q];
  }
  __device__ View rv_get() const {
    View v;
    const uint4 w = rv[0];
    v.x.parent = (int32_t)w.x;
    v.x.info = w.y;
    v.x.visits = (int32_t)w.z;
    v.x.t = (int32_t)w.w;
#pragma unroll
    for (int q = 0; q < kNA; ++q) v.sh[q] = rv[(1 + q) * kWave];
    return v;
  }
  __device__ void fail(int code) {
    if (h.err == 0) h.err = code;
  }

  // ------------------------------------------------------------------ RNG
  __device__ __forceinline__ uint32_t draw(int slot, uint32_t stream) {
    if ((la_pend >> slot) & 1u) {
      la_pend &= ~(1u << slot);
      return la_w[slot];
    }
    return philox_word(h.seed, h.tree_key, stream, h.ctr[slot]++);
  }
  // the stream of counter slot q: slot 5 + k is middle tree k's planner's,
  // whose level is NT - 1 - k (philox.h belief_mid_stream, oracle/intmcp.py
  // belief_stream)
  static __device__ __forceinline__ constexpr uint32_t slot_stream(int q) {
    return q == 0 ? (uint32_t)S_BELIEF : q == 1 ? (uint32_t)S_SELECT : q == 2 ? (uint32_t)S_MODEL
           : q == 3 ? (uint32_t)S_ACT_BASE : q == 4 ? (uint32_t)S_ACT_BASE + 1u
           : q == 5 ? (uint32_t)S_BELIEF_NESTED : belief_mid_stream(NT + 4 - q);
  }
  __device__ __forceinline__ void la_fill() {
#pragma unroll
    for (int q = 0; q < kCtrs; ++q) {
      if (q == 2 && !Env::kStepDraws) continue;
      if (!((la_pend >> q) & 1u)) {
        la_w[q] = philox_word(h.seed, h.tree_key, slot_stream(q), h.ctr[q]++);
        la_pend |= 1u << q;
      }
    }
  }
  // tree k's planner's random.Random(seed): the top planner's S_BELIEF, the
  // level-0 planner's S_BELIEF_NESTED, a middle tree's S_BELIEF_MID + its
  // level - 1 (the oracle's streams, oracle/intmcp.py OracleINTMCP)
  __device__ __forceinline__ uint32_t d_bel(int k, uint32_t n) {
    if (k == kBot) return uniform_int(draw(5, S_BELIEF_NESTED), n);
    if (k == 0) return uniform_int(draw(0, S_BELIEF), n);
    return uniform_int(draw(5 + k, slot_stream(5 + k)), n);   // middle tree k
  }
  __device__ __forceinline__ uint32_t d_sel(uint32_t n) { return uniform_int(draw(1, S_SELECT), n); }
  __device__ __forceinline__ double d_sel_float() { return uniform_float(draw(1, S_SELECT)); }
  __device__ __forceinline__ uint32_t d_model(uint32_t n) { return uniform_int(draw(2, S_MODEL), n); }
  __device__ __forceinline__ uint32_t d_act(int agent, uint32_t n) {   // model.action_spaces[agent].sample()
    return agent == 0 ? uniform_int(draw(3, S_ACT_BASE), n) : uniform_int(draw(4, S_ACT_BASE + 1), n);
  }
  // search_policies[agent].sample_action of tree k's planner
  __device__ __forceinline__ uint32_t d_pol(int k, int agent) {
    if (!p.sp_any || !p.sp_fixed[k][agent]) return d_act(agent, (uint32_t)p.A);
    const uint32_t w = agent == 0 ? draw(3, S_ACT_BASE) : draw(4, S_ACT_BASE + 1);
    return (uint32_t)tm_choice(p.sp_cum[k][agent], p.sp_tot[k][agent], p.A, w);
  }

  // ---------------------------------------------------------------- trees
  // k = 0: the level-1 (ego) tree, k = 1: the level-0 (other agent) tree
  __device__ uint32_t hkey(uint32_t na, uint64_t okey) const {
    return ovf_hash(na, okey) & (uint32_t)(p.H - 1);
  }
  // a new obs node, child (n, a, okey) (visits 0); -1 if the arena is full.
  // hot = false: the caller writes the INode itself (*xo)
  __device__ int new_node(int k, int n, int a, uint64_t okey, int parent_t, INode* xo = nullptr,
                          bool hot = true) {
    if (h.n_nodes[k] >= p.Nn) {
      fail(POMCP_E_ARENA);
      return -1;
    }
    const int c = h.n_nodes[k]++;
    INode x;
    x.parent = n;
    x.info = (uint32_t)a;
    x.visits = 0;
    x.t = (parent_t >= 0 ? parent_t : N(k, n).t) + 1;
    if (hot) N(k, c) = x;
    ICold o;
    o.okey = okey;
    o.stats = -1;
    o.support = kImNoSupport;
    C(k, c) = o;
    if (xo) *xo = x;
    return c;
  }
  // The obs child (n, a, okey); created (visits 0) if missing (INTMCP.traverse /
  // history extension, intmcp.py:797-809, 466).
  // created (optional): whether it was missing; parent_t >= 0: node n's t,
  // known to the caller (saves reloading the parent).
  __device__ int child(int k, int n, int a, uint64_t okey, bool* created = nullptr,
                       int parent_t = -1) {
    return child_rec(k, n, a, okey, rec(k, n, a), created, parent_t);
  }
  // child(), with (n, a)'s record r already loaded: the inline slots, then
  // (both full, neither matching) the hash map.  A (node, action)'s children
  // fill its inline slots in creation order before any goes to the map, so
  // a miss with a free slot means the child is missing.
  // xo / hot: as new_node's, for a created child
  __device__ int child_rec(int k, int n, int a, uint64_t okey, const Rec& r, bool* created,
                           int parent_t, INode* xo = nullptr, bool hot = true) {
    const uint32_t lo = (uint32_t)okey, hi = (uint32_t)(okey >> 32);
    if (created) *created = false;
    const int c0 = (int)r.w[1].x, c1 = (int)r.w[1].w;
    if (c0 != 0 && r.w[0].z == lo && r.w[0].w == hi) return c0;
    if (c1 != 0 && r.w[1].y == lo && r.w[1].z == hi) return c1;
    if (c1 == 0) {   // a free inline slot: create the child there
      if (created) *created = true;
      const int c = new_node(k, n, a, okey, parent_t, xo, hot);
      if (c < 0) return -1;
      uint32_t* w = R(k, n, a);
      *reinterpret_cast<uint3*>(w + (c0 == 0 ? 2 : 5)) = make_uint3(lo, hi, (uint32_t)c);
      return c;
    }
    const uint32_t na = ((uint32_t)n << 3) | (uint32_t)a;
    uint32_t s = hkey(na, okey);
    for (int64_t probe = 0; probe < p.H; ++probe) {
      const IHash e = hs[k][s];
      if (e.child >= 0 && e.na == na && e.okey == okey) return e.child;
      if (e.child < 0) {
        if (created) *created = true;
        const int c = new_node(k, n, a, okey, parent_t, xo, hot);
        if (c < 0) return -1;
        IHash ne;
        ne.okey = okey;
        ne.na = na;
        ne.child = c;
        hs[k][s] = ne;
        return c;
      }
      s = (s + 1) & (uint32_t)(p.H - 1);
    }
    fail(POMCP_E_ARENA);
    return -1;
  }
  // ObsNode.add_child(a) (node.py:68-80) if not a child yet
  __device__ void reg(int k, int n, int a) {
    INode& x = N(k, n);
    const int nr = im_nreg(x.info);
    for (int i = 0; i < nr; ++i)
      if (im_order(x.info, i) == a) return;
    if (nr >= 6) {
      fail(POMCP_E_INVALID);
      return;
    }
    x.info = (x.info & ~(7u << 5)) | ((uint32_t)(nr + 1) << 5) | ((uint32_t)a << (8 + 3 * nr));
    if (a < p.A && !im_has_stats(x.info)) {   // the statistics: zero since the arena was cleared
      if (h.n_stats[k] + p.A > p.Ns) {
        fail(POMCP_E_ARENA);
        return;
      }
      x.info |= kImStatsBit;
      C(k, n).stats = h.n_stats[k];
      h.n_stats[k] += p.A;
    }
  }
  // reg() of node n whose INode the caller holds current (x, updated): no reads
  __device__ void reg_known(int k, int n, int a, INode& x) {
    const int nr = im_nreg(x.info);
    for (int i = 0; i < nr; ++i)
      if (im_order(x.info, i) == a) return;
    if (nr >= 6) {
      fail(POMCP_E_INVALID);
      return;
    }
    x.info = (x.info & ~(7u << 5)) | ((uint32_t)(nr + 1) << 5) | ((uint32_t)a << (8 + 3 * nr));
    if (a < p.A && !im_has_stats(x.info)) {
      if (h.n_stats[k] + p.A > p.Ns) {
        fail(POMCP_E_ARENA);
        return;
      }
      x.info |= kImStatsBit;
      C(k, n).stats = h.n_stats[k];
      h.n_stats[k] += p.A;
    }
    N(k, n).info = x.info;
  }
  __device__ void traverse(int k, int n) {   // intmcp.py:797-809
    while (n > 0 && !im_path_ok(N(k, n).info)) {
      const int par = N(k, n).parent;
      reg(k, par, (int)im_paction(N(k, n).info));
      N(k, n).info |= 1u << 4;
      n = par;
    }
  }
  __device__ void expand(int k, int n) {
    for (int a = 0; a < p.A; ++a) reg(k, n, a);
  }
  // expand() of node n whose INode the caller holds current (x, updated):
  // the same registrations in action order, no reads -- reg() re-reads the
  // node for every action, a dependent round trip each
  __device__ void expand_known(int k, int n, INode& x) {
    uint32_t info = x.info;
    int nr = im_nreg(info);
    bool alloc = false;
    for (int a = 0; a < p.A; ++a) {
      bool have = false;
      for (int i = 0; i < nr; ++i) have |= im_order(info, i) == a;
      if (have) continue;
      if (nr >= 6) {
        fail(POMCP_E_INVALID);
        break;
      }
      info = (info & ~(7u << 5)) | ((uint32_t)(nr + 1) << 5) | ((uint32_t)a << (8 + 3 * nr));
      ++nr;
      alloc |= !im_has_stats(info);
    }
    if (alloc) {
      if (h.n_stats[k] + p.A > p.Ns) {
        fail(POMCP_E_ARENA);
        return;
      }
      info |= kImStatsBit;
      C(k, n).stats = h.n_stats[k];
      h.n_stats[k] += p.A;
    }
    x.info = info;
    N(k, n).info = info;
  }

  __device__ void mm_update(int k, double v) {
    if (v > h.mm_max[k]) h.mm_max[k] = v;
    if (v < h.mm_min[k]) h.mm_min[k] = v;
  }
  __device__ double normalize(int k, double v) const {
    return h.mm_max[k] > h.mm_min[k] ? (v - h.mm_min[k]) / (h.mm_max[k] - h.mm_min[k]) : v;
  }
  __device__ double logn(int n) {
    if (n < lt_n) return lt_lds[n];
    if (n >= p.logtab_n) {
      fail(POMCP_E_ARENA);
      return 0.0;
    }
    return p.logtab[n];
  }

  // ------------------------------------------------------------- selection
  // the agent of tree k: k = 0 the ego, k = 1 the other agent
  __device__ int agent(int k) const { return (k & 1) == 0 ? p.ego : p.other; }
  // the planner's own tree: 0 (nesting level 1), 1 (nesting level 0)
  __device__ int top() const { return p.nest0 ? 1 : 0; }

  // {visits, -, value} of the registered children of node x, in registration
  // order, from the node's view
  __device__ void child_stats(const View& v, int nr, uint4 (&q)[kImMaxA]) const {
#pragma unroll
    for (int i = 0; i < kImMaxA; ++i) {
      const int a = im_order(v.x.info, i);
      uint4 r = make_uint4(0, 0, 0, 0);   // (the None action: no statistics)
#pragma unroll
      for (int j = 0; j < kNA; ++j)
        r = sel4(j == a, v.sh[j], r);
      q[i] = i < nr ? r : make_uint4(0, 0, 0, 0);
    }
  }

  __device__ int select(int k, const View& v) {   // intmcp.py:670-701
    const INode& x = v.x;
    if (x.visits == 0) return (int)d_sel((uint32_t)p.A);
    const int nr = im_nreg(x.info);
    uint4 q[kImMaxA];
    child_stats(v, nr, q);
    if (p.sel == POMCP_SEL_UCB) {
      // the first unvisited child in registration order, if any
      int zero = -1;
#pragma unroll
      for (int i = kImMaxA - 1; i >= 0; --i)
        if (i < nr && q[i].x == 0u) zero = i;
      if (zero >= 0) return im_order(x.info, zero);
      const double log_n = logn(x.visits);
#if !defined(IM_ABLATE_SELECT) && !defined(POMCP_EXACT_SELECT)
      // Fast scores first, the exact ones only for near-ties of different
      // statistics: as k_search's select_action (pomcp_search.hip), in
      // registration order
      {
        const double lo = h.mm_min[k], hi = h.mm_max[k];
        const bool nz = hi > lo;
        const double rr = nz ? rcp_nr(hi - lo) : 1.0;
        const double csl = p.c * sqrt_fast(log_n);
        double sf[kImMaxA], mg[kImMaxA];
        int bi = 0;
        double bf = -__builtin_inf(), bm = 0.0;
        uint4 sb = q[0];
#pragma unroll
        for (int i = 0; i < kImMaxA; ++i) {
          const double v = hilo_d(q[i].z, q[i].w);
          const double qf = nz ? (v - lo) * rr : v;
          const double ef = csl * rsq_nr((double)((int)q[i].x > 0 ? (int)q[i].x : 1));
          sf[i] = qf + ef;
          mg[i] = __builtin_fabs(qf) + ef;
          if (i < nr && sf[i] > bf) {
            bf = sf[i];
            bm = mg[i];
            bi = i;
          }
        }
#pragma unroll
        for (int i = 1; i < kImMaxA; ++i) sb = sel4(i == bi, q[i], sb);
        bool amb = false;
#pragma unroll
        for (int i = 0; i < kImMaxA; ++i) {
          const bool same = q[i].x == sb.x && q[i].z == sb.z && q[i].w == sb.w;
          amb |= i < nr && i != bi && !same && !(bf - sf[i] > 1e-12 * (mg[i] + bm));
        }
        if (!amb && nr > 0) return im_order(x.info, bi);
      }
#endif
      double best = -__builtin_inf();
      int ba = 0;
      // unrolled with a bound check: the arrays stay in registers (a loop to
      // nr indexes them dynamically, which puts them in scratch memory)
#pragma unroll
      for (int i = 0; i < kImMaxA; ++i) {
        if (i >= nr) break;
        const int a = im_order(x.info, i);
        const int sv = (int)q[i].x;
#ifdef IM_ABLATE_SELECT   // ablation build only (measurement): no FP64 div / sqrt
        const double v = hilo_d(q[i].z, q[i].w) + p.c * log_n * (double)sv;
#else
        const double v = normalize(k, hilo_d(q[i].z, q[i].w)) + p.c * sqrt(log_n / (double)sv);
#endif
        if (v > best) {
          best = v;
          ba = a;
        }
      }
      return ba;
    }
    int min_n = x.visits + 1, nxt = 0;            // min_visit_action_selection
#pragma unroll
    for (int i = 0; i < kImMaxA; ++i) {
      if (i >= nr) break;
      const int a = im_order(x.info, i);
      const int v = (int)q[i].x;
      if (v < min_n) {
        min_n = v;
        nxt = a;
      }
    }
    return nxt;
  }

  // INTMCP.sample_action (intmcp.py:763-791) of tree j's planner (the level
  // below its caller's, tree j - 1) at node n
  __device__ int sample_action(int j, int n) {
    View v = view(j, n);                // node + statistics: one round trip
    return sample_action(j, n, v, -1, nullptr);
  }
  // pn / pnx: a node the caller holds current (the previous level's history
  // node: usually n's parent), so the traverse of a fresh history node
  // registers it at its parent without reading either
  __device__ int sample_action(int j, int n, View& v, int pn = -1, INode* pnx = nullptr) {
    if (n > 0 && !im_path_ok(v.x.info)) {
      if (pnx != nullptr && v.x.parent == pn) {   // traverse(j, n), first step known
        reg_known(j, pn, (int)im_paction(v.x.info), *pnx);
        N(j, n).info = v.x.info | (1u << 4);
        if (pn > 0 && !im_path_ok(pnx->info)) traverse(j, pn);
      } else {
        traverse(j, n);         // registers n's path at its ancestors; n itself
      }
      v.x.info |= 1u << 4;      // only gains the path_ok bit (no reload)
    }
    const INode& x = v.x;
    const int nr = im_nreg(x.info);
    if (x.visits == 0 || nr == 0) return (int)d_pol(j - 1, agent(j));   // the caller's policy
    uint4 q[kImMaxA];
    child_stats(v, nr, q);
    const double d = d_sel_float();   // random.choices' random() (the stream's only draw here)
#ifndef IM_EXACT_SOFTMAX
    // The choice from bounded FP32 weights: p_i = 2^(x_i log2 e), x_i =
    // visits_i / sqrt(N), relative error < x 2.4e-7 + 1.2e-7 (1-ulp rsq / exp2,
    // FP32 rounding); the cumulative weights c_i are then within
    // E/2 = 4.8e-7 x_max + 1.2e-6 of the exact FP64 ones (c <= 1), u = random()
    // within 6e-8.  When u is farther than E from every c_i the bisection's
    // answer is the exact one; otherwise (~1e-3 of draws) the exact FP64
    // softmax below decides.  (IM_EXACT_SOFTMAX: the exact path only.)
    {
      const float rs = __builtin_amdgcn_rsqf((float)x.visits);
      float pf[kImMaxA];
      float tot = 0.0f, xmax = 0.0f;
#pragma unroll
      for (int i = 0; i < kImMaxA; ++i) {
        const float t = (float)q[i].x * rs;
        pf[i] = i < nr ? __builtin_amdgcn_exp2f(t * 1.44269504f) : 0.0f;
        if (i < nr) xmax = __builtin_fmaxf(xmax, t);
        tot += pf[i];
      }
      const float rt = __builtin_amdgcn_rcpf(tot);
      const float E = p.fast_slack * (1e-6f * xmax + 2.4e-6f);
      const float uf = (float)d;
      bool amb = !(xmax <= 80.0f);
      int lo = nr - 1;
      float acc = 0.0f;
#pragma unroll
      for (int i = 0; i < kImMaxA - 1; ++i) {
        if (i < nr - 1) {
          acc += pf[i] * rt;
          amb |= __builtin_fabsf(uf - acc) <= E;
          if (lo == nr - 1 && uf < acc) lo = i;
        }
      }
      if (!amb) return im_order(x.info, lo);
    }
#endif
    if (p.exact_draws != nullptr) atomicAdd(p.exact_draws, 1ull);   // tests: fallbacks fired
    const double sq = sqrt((double)x.visits);
    double pr[kImMaxA];
    double total = 0.0;
#pragma unroll
    for (int i = 0; i < kImMaxA; ++i) {
      if (i >= nr) break;
#ifdef IM_ABLATE_SOFTMAX   // ablation build only (measurement): no exp / division
      pr[i] = (double)(int)q[i].x + 1.0;
#else
      pr[i] = host_exp_tab((double)(int)q[i].x / sq, exp_tab);   // == math.exp (host_exp.h)
#endif
      total = i == 0 ? pr[i] : total + pr[i];
    }
    // random.choices(children, weights=p / sum): cum weights, x = random() * total
    double cum[kImMaxA];
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < kImMaxA; ++i) {
      if (i >= nr) break;
#ifdef IM_ABLATE_SOFTMAX
      const double w = pr[i];
#else
      const double w = pr[i] / total;
#endif
      acc = i == 0 ? w : acc + w;
      cum[i] = acc;
    }
    double last = cum[0];
#pragma unroll
    for (int i = 1; i < kImMaxA; ++i)
      if (i == nr - 1) last = cum[i];
    const double u = d * (last + 0.0);
    // bisect_right(cum, u, 0, nr - 1) over the non-decreasing cum: the first
    // i < nr - 1 with u < cum[i], else nr - 1 (a scan keeps cum in registers)
    int lo = nr - 1;
#pragma unroll
    for (int i = kImMaxA - 2; i >= 0; --i)
      if (i < nr - 1 && u < cum[i]) lo = i;
    return im_order(x.info, lo);
  }

  // the other agent's action from a particle of tree k (intmcp.py:602-615)
  __device__ int other_action(int k, uint32_t nested) {
    if (k == kBot || p.state_belief_only) return (int)d_bel(k, (uint32_t)p.A);
    return sample_action(k + 1, (int)nested);
  }

  // joint step for tree k's agent; the next particle's other-agent node
  __device__ void step(int k, uint32_t s0, uint32_t s1, uint32_t nested, int a_self,
                       int a_other, uint32_t* n0, uint32_t* n1, double* r, int* done,
                       uint64_t* okey, uint32_t* nested_out) {
    const int me = agent(k);
    const uint32_t j = Env::kStepDraws ? d_model(2) : 0u;
    Env::step(m, me, s0, s1, (uint32_t)a_self, (uint32_t)a_other, j, n0, n1, r, done);
    *okey = Env::obs_key(m, me, *n0, *n1);
    *nested_out = 0;
    if (k < kBot) {   // the other agent's history extension in tree k + 1
      const uint64_t ok = Env::obs_key(m, agent(k + 1), *n0, *n1);
      const int c = child(k + 1, (int)nested, a_other, ok);
      *nested_out = c < 0 ? 0u : (uint32_t)c;
    }
  }

  __device__ void log_add(int k, int node, uint32_t v0, uint32_t v1, uint32_t nested) {
    if (h.n_log[k] >= p.Nl) {
      fail(POMCP_E_ARENA);
      return;
    }
#ifdef IM_ABLATE_LOG   // ablation build only (measurement): no particle log stores
    if (node >= 0) return;
#endif
    IRec r;
    r.node = (uint32_t)node;
    r.v0 = v0;
    r.v1 = v1;
    r.nested = nested;
    lg[k][h.n_log[k]++] = r;
  }

  // ------------------------------------------------------------ rollout
  __device__ double rollout(int k, uint32_t s0, uint32_t s1, int t, int depth) {   // intmcp.py:547-593
#ifdef IM_ABLATE_ROLLOUT   // ablation build only (measurement): no rollout
    return 0.0;
#endif
    double ret = 0.0;
    int kk = 0;
    const int me = agent(k);
    while (depth <= p.depth_limit && t <= p.step_limit) {
      const uint32_t a0 = d_pol(k, 0);
      const uint32_t a1 = d_pol(k, 1);
      const uint32_t j = Env::kStepDraws ? d_model(2) : 0u;
      uint32_t n0, n1;
      double r;
      int done;
      Env::step(m, me, s0, s1, me == 0 ? a0 : a1, me == 0 ? a1 : a0, j, &n0, &n1, &r, &done);
      if (kk >= p.dpow_n) {
        fail(POMCP_E_ARENA);
        return ret;
      }
      ret += dp[kk] * r;
      if (done) break;
      s0 = n0;
      s1 = n1;
      ++t;
      ++depth;
      ++kk;
    }
    return ret;
  }

  // ----------------------------------------------------------- simulate
  // INTMCP._simulate (intmcp.py:444-517) from node n of tree k; returns the
  // search depth.  Each level loads the child's line (node + statistics
  // heads) once: it updates the child's visits / flags and is the next
  // level's view; and the chosen action's record (total, obs children).  The
  // path keeps each level's statistics as they were before (visits, value,
  // total), so the backup writes without reading; the first kImRegPath levels
  // stay in registers.
  __device__ int simulate(int k, uint32_t s0, uint32_t s1, uint32_t nested, int n, View v) {
    int depth = 0, plen = 0;
    double leaf = 0.0;
    uint4 rp[kImRegPath][3];   // {n, a, done, visits0}, {r, value0}, {total0, -}
    View nv;                   // the other agent's history node (level 1), prefetched
    bool have_nv = false;
    INode pnx;                 // the previous level's history node, as it is now
    int pn = -1;
    int roll_t = -1;           // >= 0: the descent ended at a leaf of this t
    if (k < kBot && !p.state_belief_only) {   // the first level's history view, in flight
      nv = view(k + 1, (int)nested);          // while the root selection runs
      have_nv = true;
      la_fill();                            // (the RNG words, while it is in flight)
    }
    for (;;) {
      const INode& x = v.x;
      if (depth > p.depth_limit || x.t + depth > p.step_limit) break;
      if (im_nreg(x.info) < p.A) {                 // leaf: add the missing children
        INode xe = x;
        expand_known(k, n, xe);
        IM_MARK(IP_EXPAND);
        roll_t = x.t;   // the rollout runs after the loop: once for the whole wave,
        break;          // not once per depth at which some lane reached a leaf
      }
      const int a = select(k, v);
      // the chosen action's record: its obs children (found once the step has
      // produced the observation) and total (for the backup), in flight
      // while the other agent's action and the step are computed
      IM_MARK(IP_SELECT);
      const Rec ra = rec(k, n, a);
      uint4 sa = v.sh[0];
#pragma unroll
      for (int q = 1; q < kNA; ++q)
        sa = sel4(q == a, v.sh[q], sa);
      // the other agent's action (intmcp.py:602-615): at level 1 its
      // history node's view was loaded when the previous level created it
      const bool nested_k = k < kBot && !p.state_belief_only;
      int ao;
      if (nested_k) {
        if (!have_nv) nv = view(k + 1, (int)nested);
        ao = sample_action(k + 1, (int)nested, nv, pn, pn >= 0 ? &pnx : nullptr);
        pn = (int)nested;   // the next level's history node is a child of this one
        pnx = nv.x;
      } else {
        ao = other_action(k, nested);
      }
      // at level 1, the record of the other agent's history extension
      // (nested, ao), in flight during the step
      IM_MARK(IP_OTHER);
      Rec rn;
      if (k < kBot) rn = rec(k + 1, (int)nested, ao);
      uint32_t n0, n1, nn = 0u;
      double r;
      int done;
      const int me = agent(k);
      const uint32_t j = Env::kStepDraws ? d_model(2) : 0u;
      Env::step(m, me, s0, s1, (uint32_t)a, (uint32_t)ao, j, &n0, &n1, &r, &done);
      const uint64_t okey = Env::obs_key(m, me, n0, n1);
      const uint64_t ok = k < kBot ? Env::obs_key(m, agent(k + 1), n0, n1) : 0ull;
      IM_MARK(IP_STEP);
      // the child (a, obs): found in the record, its view loaded; created,
      // its view is known (the descent writes its INode below).  Then, at
      // level 1, the other agent's history extension likewise.  (Loads are
      // issued before the stores of a creation: a wait for a load also waits
      // for every store issued before it.)
      // whether the descent goes on below the child (the loop's own test at
      // the next level: the child's t is x.t + 1): if not, the child's heads
      // and the other agent's next history view are never read -- load only
      // the child's INode (its visits / flags are updated below)
      const bool more = !done && depth + 1 <= p.depth_limit && x.t + depth + 2 <= p.step_limit;
      bool created;
      INode cx;
      const int c = child_rec(k, n, a, okey, ra, &created, x.t, &cx, false);
      if (c < 0) return depth;
      View cv;
      if (!created) cv = more ? view(k, c) : view_node(k, c);
      if (k < kBot) {
        bool ncr;
        INode nx;
        const int cn = child_rec(k + 1, (int)nested, ao, ok, rn, &ncr, nested_k ? nv.x.t : -1, &nx);
        nn = cn < 0 ? 0u : (uint32_t)cn;
        if (nested_k && more) {   // the next level's other-agent view (no wait)
          nv = ncr ? fresh_view(nx) : view(k + 1, (int)nn);
          have_nv = true;
        }
      }
      if (created) cv = fresh_view(cx);
      IM_MARK(IP_CHILD);
      la_fill();   // the next level's RNG words, while the child's view is in flight
      cv.x.visits = created ? 1 : cv.x.visits + 1;
      uint32_t info = cv.x.info;
      if (im_path_ok(x.info)) info |= 1u << 4;   // x: node n, unchanged since loaded
      info = done ? (info | 8u) : (info & ~8u);
      cv.x.info = info;
      *reinterpret_cast<int4*>(&N(k, c)) =          // {parent, info, visits, t}
          make_int4(cv.x.parent, (int)cv.x.info, cv.x.visits, cv.x.t);
      log_add(k, c, n0, n1, nn);
      if (plen >= kImPath) {
        fail(POMCP_E_ARENA);
        return depth;
      }
      const uint4 e0 = make_uint4((uint32_t)n, (uint32_t)a, (uint32_t)done, sa.x);
      const uint4 e1 = make_uint4((uint32_t)__double2loint(r), (uint32_t)__double2hiint(r), sa.z, sa.w);
      const uint4 s2 = make_uint4(ra.w[0].x, ra.w[0].y, 0u, 0u);   // total0
      if (plen < kImRegPath) {
#pragma unroll
        for (int l = 0; l < kImRegPath; ++l)
          if (l == plen) {
            rp[l][0] = e0;
            rp[l][1] = e1;
            rp[l][2] = s2;
          }
      } else {
        path[plen * 3] = make_int4((int)e0.x, (int)e0.y, (int)e0.z, (int)e0.w);
        path[plen * 3 + 1] = make_int4((int)e1.x, (int)e1.y, (int)e1.z, (int)e1.w);
        path[plen * 3 + 2] = make_int4((int)s2.x, (int)s2.y, (int)s2.z, (int)s2.w);
      }
      ++plen;
      IM_MARK(IP_DESCEND);
      if (done) break;
      n = c;
      v = cv;
      s0 = n0;
      s1 = n1;
      nested = nn;
      ++depth;
    }
    if (roll_t >= 0) leaf = rollout(k, s0, s1, roll_t, depth);
    IM_MARK(IP_ROLLOUT);
    double g = leaf;
    auto backup = [&](uint4 e0, uint4 e1, uint4 e2) {   // node.py:166-178
      const double r = hilo_d(e1.x, e1.y);
      g = e0.z ? r : r + p.discount * g;
      const int vis = (int)e0.w + 1;
      const double value0 = hilo_d(e1.z, e1.w);
      const double total = hilo_d(e2.x, e2.y) + g;
      const double value = value0 + (g - value0) / (double)vis;
      const uint4 head = make_uint4((uint32_t)vis, 0u, (uint32_t)__double2loint(value),
                                    (uint32_t)__double2hiint(value));
      *reinterpret_cast<uint3*>(H(k, (int)e0.x, (int)e0.y)) = make_uint3(head.x, head.z, head.w);
      if (k == 0 && (int)e0.x == rv_root) rv[(1 + e0.y) * kWave] = head;   // the cached root view
      set_total(k, (int)e0.x, (int)e0.y, total);
      mm_update(k, value);
    };
    for (int l = plen - 1; l >= kImRegPath; --l) {
      const int4 a0 = path[l * 3], a1 = path[l * 3 + 1], a2 = path[l * 3 + 2];
      backup(make_uint4(a0.x, a0.y, a0.z, a0.w), make_uint4(a1.x, a1.y, a1.z, a1.w),
             make_uint4(a2.x, a2.y, a2.z, a2.w));
    }
#pragma unroll
    for (int l = kImRegPath - 1; l >= 0; --l)
      if (l < plen) backup(rp[l][0], rp[l][1], rp[l][2]);
    IM_MARK(IP_BACKUP);
    return depth;
  }

  // ------------------------------------------------------ beliefs / update
  __device__ uint4* root_buf(int sel) { return rootb + (int64_t)sel * p.Nr; }
  __device__ ISup* sup_tab(int sel) { return sup + (int64_t)sel * p.Nr; }
  __device__ uint2* sup_parts(int sel) { return supp + (int64_t)sel * p.Nsp; }
  // middle tree m + 1's belief table `sel` and its particles
  __device__ ISup* mtab(int m, int sel) { return msup[m] + (int64_t)sel * p.Nr; }
  __device__ uint4* mparts(int m, int sel) { return msupp[m] + (int64_t)sel * p.Nsp; }

  // the slot of node n of tree k in the belief table tab (count entries): the
  // node's `support` field while the caller has that table's slots marked
  // (mark_slots), else a scan
  __device__ int find_slot(int k, const ISup* tab, int n, int count) {
    const uint32_t s = C(k, n).support;
    if (s != kImNoSupport) return (int)s < count && tab[s].node == n ? (int)s : -1;
    for (int i = 0; i < count; ++i)
      if (tab[i].node == n) return i;
    return -1;
  }
  __device__ void mark_slots(int k, const ISup* tab, int count, bool on) {
    for (int i = 0; i < count; ++i) C(k, tab[i].node).support = on ? (uint32_t)i : kImNoSupport;
  }
  // the level-0 tree's support table `sel`
  __device__ int find_support(int sel, int n, int count) { return find_slot(kBot, sup_tab(sel), n, count); }
  __device__ void mark_support(int sel, int count, bool on) { mark_slots(kBot, sup_tab(sel), count, on); }

  // BeliefRejectionSampler (belief.py:145-194, use_rejected_samples=True) for a
  // level-1 node n: parent particles from the previous root buffer; appends to
  // the current root buffer
  __device__ void reinvig_top(int n, int action, uint64_t okey, int target, int* size) {
    const int to_add = target - *size;
    if (to_add <= 0) return;
    const uint4* par = root_buf(h.root_sel ^ 1);
    const int psize = h.pad;   // previous root size (kept in pad during update)
    if (psize <= 0) {
      fail(POMCP_E_STATE);
      return;
    }
    uint4* cur = root_buf(h.root_sel);
    const double limit = p.limit_factor * (double)to_add;
    int count = 0, attempts = 0, nrej = 0;
    const int base = *size;
    if (base + 2 * to_add > p.Nr) {
      fail(POMCP_E_ARENA);
      return;
    }
    // accepted go to [base, base + to_add), rejected to [base + to_add, ...)
    while (count < to_add && (double)attempts < limit) {
      ++attempts;
      const uint4 hp = par[d_bel(0, (uint32_t)psize)];
      const int ao = other_action(0, hp.z);
      uint32_t n0, n1, nn;
      double r;
      int done;
      uint64_t k2;
      step(0, hp.x, hp.y, hp.z, action, ao, &n0, &n1, &r, &done, &k2, &nn);
      const uint4 rec = make_uint4(n0, n1, nn, 0u);
      if (k2 == okey) {
        cur[base + count++] = rec;
      } else if (nrej < to_add) {
        cur[base + to_add + nrej++] = rec;
      }
    }
    int fill = to_add - count;
    if (fill > nrej) fill = nrej;
    for (int q = 0; q < fill; ++q) cur[base + count + q] = cur[base + to_add + q];
    *size = base + count + fill;
  }

  // the same for a level-0 node: parent particles from the previous support
  // table; appends to support entry `si` of table `sel`
  __device__ void reinvig_nested(int n, int action, uint64_t okey, int target, int sel, int si) {
    ISup& e = sup_tab(sel)[si];
    const int to_add = target - e.size;
    if (to_add <= 0) return;
    const int par = N(kBot, n).parent;
    const int pi = find_support(sel ^ 1, par, h.pad);   // previous support count in pad
    if (pi < 0) {
      fail(POMCP_E_UNSUPPORTED);   // parent belief not materialised
      return;
    }
    const ISup pe = sup_tab(sel ^ 1)[pi];
    if (pe.size <= 0) {
      fail(POMCP_E_STATE);
      return;
    }
    const uint2* pp = sup_parts(sel ^ 1) + pe.off;
    uint2* cur = sup_parts(sel) + e.off;
    if (e.size + 2 * to_add > e.cap) {
      fail(POMCP_E_ARENA);
      return;
    }
    const double limit = p.limit_factor * (double)to_add;
    int count = 0, attempts = 0, nrej = 0;
    const int base = e.size;
    while (count < to_add && (double)attempts < limit) {
      ++attempts;
      const uint2 hp = pp[d_bel(kBot, (uint32_t)pe.size)];
      const int ao = (int)d_bel(kBot, (uint32_t)p.A);   // self._rng.choice (level 0)
      uint32_t n0, n1, nn;
      double r;
      int done;
      uint64_t k2;
      step(kBot, hp.x, hp.y, 0u, action, ao, &n0, &n1, &r, &done, &k2, &nn);
      const uint2 rec = make_uint2(n0, n1);
      if (k2 == okey) {
        cur[base + count++] = rec;
      } else if (nrej < to_add) {
        cur[base + to_add + nrej++] = rec;
      }
    }
    int fill = to_add - count;
    if (fill > nrej) fill = nrej;
    for (int q = 0; q < fill; ++q) cur[base + count + q] = cur[base + to_add + q];
    e.size = base + count + fill;
  }

  // the same for a node of middle tree k, whose particles carry the next
  // tree's history (intmcp.py:815-862 at level >= 1: the other agent acts by
  // the level below's sample_action, the particle's history extends in tree
  // k + 1); parents in the previous table of tree k (h.mpad[k - 1] entries),
  // appends to entry `si` of table `sel`
  __device__ void reinvig_mid(int k, int n, int action, uint64_t okey, int target, int sel, int si) {
    const int m = k - 1;
    ISup& e = mtab(m, sel)[si];
    const int to_add = target - e.size;
    if (to_add <= 0) return;
    const int par = N(k, n).parent;
    const int pi = find_slot(k, mtab(m, sel ^ 1), par, h.mpad[m]);
    if (pi < 0) {
      fail(POMCP_E_UNSUPPORTED);   // parent belief not materialised
      return;
    }
    const ISup pe = mtab(m, sel ^ 1)[pi];
    if (pe.size <= 0) {
      fail(POMCP_E_STATE);
      return;
    }
    const uint4* pp = mparts(m, sel ^ 1) + pe.off;
    uint4* cur = mparts(m, sel) + e.off;
    if (e.size + 2 * to_add > e.cap) {
      fail(POMCP_E_ARENA);
      return;
    }
    const double limit = p.limit_factor * (double)to_add;
    int count = 0, attempts = 0, nrej = 0;
    const int base = e.size;
    while (count < to_add && (double)attempts < limit) {
      ++attempts;
      const uint4 hp = pp[d_bel(k, (uint32_t)pe.size)];
      const int ao = other_action(k, hp.z);
      uint32_t n0, n1, nn;
      double r;
      int done;
      uint64_t k2;
      step(k, hp.x, hp.y, hp.z, action, ao, &n0, &n1, &r, &done, &k2, &nn);
      const uint4 rec = make_uint4(n0, n1, nn, 0u);
      if (k2 == okey) {
        cur[base + count++] = rec;
      } else if (nrej < to_add) {
        cur[base + to_add + nrej++] = rec;
      }
      if (h.err != 0) return;
    }
    int fill = to_add - count;
    if (fill > nrej) fill = nrej;
    for (int q = 0; q < fill; ++q) cur[base + count + q] = cur[base + to_add + q];
    e.size = base + count + fill;
  }
};

// The history distribution of a belief (intmcp.py:334-362 for one node of
// probability 1): the distinct tree-k nodes named by the particles rb[0, size)
// (.z) in first-occurrence order, probability count / size; writes each
// particle's slot into .w.  (At nesting level 1: tree 1 from the level-1 root
// belief; at level 2: tree 1 from the level-2 root belief.)
// kWave: the 64 lanes of the wave run the same pair (k_im_update's wave mode,
// every lane holding the same state) and share the scans: 64 records per
// step, grouped per node / slot in lane order, so the result (first-occurrence
// order, insertion order per slot) is the serial loop's.
__device__ __forceinline__ uint64_t im_lanes_below() { return (1ull << (threadIdx.x & 63)) - 1ull; }

template <class Env, int NT, bool kWave = false>
__device__ void im_support(ImPair<Env, NT>& P, int k, ISup* tab, double* prob, uint4* rb, int size,
                           int* nsup) {
  int n = 0;
  // node -> slot through the nodes' `support` field (kImNoSupport outside a
  // materialisation), not a scan of the table per particle: O(size), not
  // O(size x distinct nodes)
  if constexpr (kWave) {
    for (int base = 0; base < size; base += kWave64) {
      const int i = base + (int)(threadIdx.x & 63);
      const bool on = i < size;
      const int nodeid = on ? (int)rb[i].z : -1;
      uint64_t todo = __ballot(on);
      while (todo) {   // each distinct node of the batch, in the order of its first lane
        const int lead = __ffsll((long long)todo) - 1;
        const int ln = __shfl(nodeid, lead);
        const uint64_t peers = __ballot(on && nodeid == ln);
        int s = (int)P.C(k, ln).support;
        if (P.C(k, ln).support == kImNoSupport) {
          s = n++;
          tab[s].node = ln;
          tab[s].size = 0;
          P.C(k, ln).support = (uint32_t)s;
        }
        tab[s].size += __popcll(peers);
        if (on && nodeid == ln) rb[i].w = (uint32_t)s;
        todo &= ~peers;
      }
    }
  } else {
    for (int i = 0; i < size; ++i) {
      const int nodeid = (int)rb[i].z;
      int s = (int)P.C(k, nodeid).support;
      if (P.C(k, nodeid).support == kImNoSupport) {
        s = n++;
        tab[s].node = nodeid;
        tab[s].size = 0;   // count for now
        P.C(k, nodeid).support = (uint32_t)s;
      }
      tab[s].size += 1;
      rb[i].w = (uint32_t)s;
    }
  }
  for (int q = 0; q < n; ++q) P.C(k, tab[q].node).support = kImNoSupport;
  for (int q = 0; q < n; ++q) {
    prob[q] = 0.0 + 1.0 * ((double)tab[q].size / (double)size);
    tab[q].size = 0;
  }
  *nsup = n;
}

// Nesting level >= 2: get_nested_history_dist (intmcp.py:334-362) of middle
// tree kt - 1's distribution (n1 entries of table t1, probabilities p1,
// particles parts1 with the tree-kt node in .z): for each entry in order, each
// distinct tree-kt node of its particles (first occurrence) gains p1 x count /
// size; the nodes in first-occurrence order over all entries.  Writes tree
// kt's table `tab` (sizes zeroed) and `prob`, and each particle's slot into .w.
// (A lane per pair, or the wave's lanes in lockstep on the same pair.)
template <class Env, int NT>
__device__ void im_support_nested(ImPair<Env, NT>& P, int kB, const ISup* t1, const double* p1, int n1,
                                  uint4* parts1, ISup* tab, double* prob, int* nsup) {
  int n = 0;
  for (int q = 0; q < n1; ++q) {
    const ISup e = t1[q];
    if (e.size <= 0) continue;   // (an empty belief contributes nothing; the reference divides by 0)
    // counts of this entry's nodes: tab[].cap as the per-entry counter
    const int first = n;
    for (int i = 0; i < e.size; ++i) {
      const int m = (int)parts1[e.off + i].z;
      int s = (int)P.C(kB, m).support;
      if (P.C(kB, m).support == kImNoSupport) {
        s = n++;
        tab[s].node = m;
        tab[s].size = 0;
        tab[s].cap = 0;
        prob[s] = 0.0;
        P.C(kB, m).support = (uint32_t)s;
      }
      if (tab[s].cap == 0) tab[s].off = -1;   // not yet counted in this entry
      tab[s].cap += 1;
      parts1[e.off + i].w = (uint32_t)s;
    }
    // add in first-occurrence order within the entry (the reference's dict order
    // of h_count); the sum for each node runs over the entries in order
    for (int i = 0; i < e.size; ++i) {
      const int s = (int)parts1[e.off + i].w;
      if (tab[s].off == -1) {
        prob[s] = (s >= first ? 0.0 : prob[s]) + p1[q] * ((double)tab[s].cap / (double)e.size);
        tab[s].off = 0;
        tab[s].cap = 0;
      }
    }
  }
  for (int q = 0; q < n; ++q) {
    P.C(kB, tab[q].node).support = kImNoSupport;
    tab[q].size = 0;
    tab[q].off = 0;
    tab[q].cap = 0;
  }
  *nsup = n;
}

// Materialise the beliefs of tree k's table entries (nsup, probabilities
// prob) from that tree's log (insertion order), leaving room per entry for the
// reinvigoration (accepted + rejected).  Part: uint2 {v0, v1} (the level-0
// tree) or uint4 {v0, v1, level-0 node, -} (the middle tree at nesting 2).
__device__ __forceinline__ void im_part(uint2* d, const IRec& r) { *d = make_uint2(r.v0, r.v1); }
__device__ __forceinline__ void im_part(uint4* d, const IRec& r) { *d = make_uint4(r.v0, r.v1, r.nested, 0u); }

template <class Env, int NT, bool kWave = false, class Part>
__device__ void im_extract_support(ImPair<Env, NT>& P, int k, ISup* tab, Part* parts,
                                   const double* prob, int nsup) {
  for (int q = 0; q < nsup; ++q) P.C(k, tab[q].node).support = (uint32_t)q;
  for (int q = 0; q < nsup; ++q) tab[q].cap = 0;
  const int nlog = P.h.n_log[k];
  if constexpr (kWave) {
    for (int base = 0; base < nlog; base += kWave64) {
      const int i = base + (int)(threadIdx.x & 63);
      const uint32_t s = i < nlog ? P.C(k, P.lg[k][i].node).support : kImNoSupport;
      uint64_t todo = __ballot(s != kImNoSupport);
      while (todo) {
        const uint32_t ls = (uint32_t)__shfl((int)s, __ffsll((long long)todo) - 1);
        const uint64_t peers = __ballot(s == ls);
        tab[ls].cap += __popcll(peers);
        todo &= ~peers;
      }
    }
  } else {
    for (int i = 0; i < nlog; ++i) {
      const uint32_t s = P.C(k, P.lg[k][i].node).support;
      if (s != kImNoSupport) tab[s].cap += 1;
    }
  }
  int off = 0;
  for (int q = 0; q < nsup; ++q) {   // room for the reinvigoration (accepted + rejected)
    tab[q].off = off;
    tab[q].size = 0;
    tab[q].cap += 2 * (int)ceil(prob[q] * (double)P.p.n_target) + 2;
    off += tab[q].cap;
  }
  if (off > P.p.Nsp) {
    P.fail(POMCP_E_ARENA);
    for (int q = 0; q < nsup; ++q) P.C(k, tab[q].node).support = kImNoSupport;
    return;
  }
  if constexpr (kWave) {
    for (int base = 0; base < nlog; base += kWave64) {
      const int i = base + (int)(threadIdx.x & 63);
      IRec r{0u, 0u, 0u, 0u};
      uint32_t s = kImNoSupport;
      if (i < nlog) {
        r = P.lg[k][i];
        s = P.C(k, r.node).support;
      }
      uint64_t todo = __ballot(s != kImNoSupport);
      while (todo) {   // each slot of the batch: its records in lane (= insertion) order
        const uint32_t ls = (uint32_t)__shfl((int)s, __ffsll((long long)todo) - 1);
        const uint64_t peers = __ballot(s == ls);
        const int at = tab[ls].off + tab[ls].size;
        if (s == ls) im_part(parts + at + __popcll(peers & im_lanes_below()), r);
        tab[ls].size += __popcll(peers);
        todo &= ~peers;
      }
    }
  } else {
    for (int i = 0; i < nlog; ++i) {
      const IRec r = P.lg[k][i];
      const uint32_t s = P.C(k, r.node).support;
      if (s != kImNoSupport) im_part(parts + tab[s].off + tab[s].size++, r);
    }
  }
  for (int q = 0; q < nsup; ++q) P.C(k, tab[q].node).support = kImNoSupport;
}

// Every obs-child map slot empty ({0, 0, -1}), grid-stride over all pairs'
// tables (a lane per pair would clear a wall-clock arena's 2 x 2^26 slots alone).
__global__ __launch_bounds__(256) void k_im_clear_hash(IHash* hs, int64_t n) {
  IHash e;
  e.okey = 0;
  e.na = 0;
  e.child = -1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    hs[i] = e;
}

template <class Env>
__global__ __launch_bounds__(64) void k_im_reset(ImParams p) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.B) return;
  IHdr h = p.hdr[b];
  for (int k = 0; k < p.nt; ++k) {   // (the hash tables: k_im_clear_hash, all lanes)
    INode r;
    r.parent = -1;
    r.info = 1u << 4;   // path_ok
    r.visits = 0;
    r.t = 0;
    ICold o;
    o.okey = 0;
    o.stats = -1;
    o.support = kImNoSupport;
    char* const line = p.nodes + im_node_off(p.Nn, p.B, b, k, 0, p.nt);
    *reinterpret_cast<INode*>(line) = r;
    *reinterpret_cast<ICold*>(line + kImCold) = o;
    h.n_nodes[k] = 1;
    h.n_stats[k] = 0;
    h.n_log[k] = 0;
    h.mm_max[k] = p.has_kb ? p.kb_max : -__builtin_inf();
    h.mm_min[k] = p.has_kb ? p.kb_min : __builtin_inf();
  }
  h.cur = 0;
  h.root_sel = 0;
  h.root_size = 0;
  h.sup_sel = 0;
  h.n_sup = 0;
  h.sup_used = 0;
  h.err = 0;
  h.last_action = -1;
  h.num_sims = 0;
  h.search_depth = 0;
  h.sims_done = 0;
  h.pad = 0;
  for (int m = 0; m < kImMaxMid; ++m) {
    h.msel[m] = 0;
    h.n_msup[m] = 0;
    h.msup_used[m] = 0;
    h.mpad[m] = 0;
  }
  p.hdr[b] = h;
}

template <class Env, int NT>
template <bool kWave>
__device__ void ImPair<Env, NT>::clear_old_beliefs(int cur_t) {
  for (int k = 0; k < NT; ++k) {
    const int n = h.n_log[k];
    int out = 0;
    if constexpr (kWave) {   // 64 records per step; the chunk is loaded before it is stored
      for (int base = 0; base < n; base += kWave64) {
        const int i = base + (int)(threadIdx.x & 63);
        IRec r{0u, 0u, 0u, 0u};
        bool keep = false;
        if (i < n) {
          r = lg[k][i];
          keep = N(k, (int)r.node).t >= cur_t - 2;
        }
        const uint64_t m = __ballot(keep);
        if (keep) lg[k][out + __popcll(m & im_lanes_below())] = r;
        out += __popcll(m);
      }
    } else {
      for (int i = 0; i < n; ++i) {
        const IRec r = lg[k][i];
        if (N(k, (int)r.node).t >= cur_t - 2) lg[k][out++] = r;
      }
    }
    h.n_log[k] = out;
  }
}

// INTMCP.update (intmcp.py:198-300) of a nesting-level-0 planner (tree 1, the
// planner p.other): its root belief is support entry 0 -- the support
// {root: 1.0} the level-1 update hands a level-0 planner, so the same
// materialisation and reinvigoration run (_initial_nested_update /
// _nested_update with dist = {cur: 1.0}, intmcp.py:216-300)
template <class Env, bool kWave>
__device__ void im_update_nest0(ImPair<Env>& P, const typename Env::Model& sm, uint64_t obs,
                                int action) {
  const ImParams& p = P.p;
  auto draw_model = [&](uint32_t n) { return P.d_model(n); };
  const int sel = P.h.sup_sel ^ 1;
  ISup* tab = P.sup_tab(sel);
  if (P.N(1, P.h.cur).t == 0) {
    const int node = P.child(1, 0, p.A, obs);
    if (node < 0) return;
    uint32_t s0, s1;   // the probe draw of sample_agent_initial_state(obs[first])
    if (!Env::sample_agent_initial(sm, p.other, obs, draw_model, &s0, &s1)) P.fail(POMCP_E_INVALID);
    P.traverse(1, node);
    uint2* pp = P.sup_parts(sel);
    int m = 0;
    while (P.h.err == 0 && (double)m < 1.0 * (double)p.n_target) {
      if (m >= p.Nsp) {
        P.fail(POMCP_E_ARENA);
        break;
      }
      Env::sample_agent_initial(sm, p.other, obs, draw_model, &s0, &s1);
      pp[m++] = make_uint2(s0, s1);
    }
    tab[0] = ISup{node, 0, m, m};
    P.h.cur = node;
    P.h.root_size = m;
    P.h.sup_sel = sel;
    P.h.n_sup = 1;
    P.h.sup_used = m;
    return;
  }
  const int node = (action >= 0 && action < p.A) ? P.child(1, P.h.cur, action, obs) : -1;
  if (node < 0) {
    P.fail(POMCP_E_NOT_FOUND);
    return;
  }
  P.traverse(1, node);
  // its belief: the log records of `node` in insertion order, then the
  // reinvigoration from the parent's (the previous root's, entry 0 of the
  // previous table)
  tab[0].node = node;
  P.prob[0] = 1.0;
  im_extract_support<Env, 2, kWave>(P, 1, P.sup_tab(sel), P.sup_parts(sel), P.prob, 1);
  if (P.h.err != 0) return;
  P.h.pad = P.h.n_sup;
  P.mark_support(sel ^ 1, P.h.pad, true);
  if (!im_absorbing(P.N(1, node).info))
    P.reinvig_nested(node, action, obs, (int)ceil(1.0 * (double)p.n_target), sel, 0);
  P.mark_support(sel ^ 1, P.h.pad, false);
  P.h.cur = node;
  P.h.root_size = tab[0].size;
  P.h.sup_sel = sel;
  P.h.n_sup = 1;
  P.h.sup_used = tab[0].off + tab[0].cap;
  if (P.h.err == 0) P.template clear_old_beliefs<kWave>(P.N(1, node).t);
}

// The level-0 (bottom, tree kBot) planner's initial beliefs
// (_initial_nested_update, intmcp.py:216-268, at level 0) for the nsup entries
// of table `sel` with probabilities prob: the probe draw of
// sample_agent_initial_state(obs of the first history), then per entry
// ceil-free `len(parts) < prob x target` draws.  Returns the particles used.
template <class Env, int NT>
__device__ int im_initial_bottom(ImPair<Env, NT>& P, const typename Env::Model& sm, int sel, int nsup,
                                 const double* prob) {
  constexpr int kB = NT - 1;
  const ImParams& p = P.p;
  auto draw_model = [&](uint32_t n) { return P.d_model(n); };
  ISup* tab = P.sup_tab(sel);
  uint32_t s0, s1;
  const int who = P.agent(kB);
  Env::sample_agent_initial(sm, who, P.C(kB, tab[0].node).okey, draw_model, &s0, &s1);   // probe
  int off = 0;
  for (int q = 0; q < nsup && P.h.err == 0; ++q) {
    P.traverse(kB, tab[q].node);
    const uint64_t oq = P.C(kB, tab[q].node).okey;
    tab[q].off = off;
    tab[q].size = 0;
    uint2* pp = P.sup_parts(sel) + off;
    int m = 0;
    while ((double)m < prob[q] * (double)p.n_target) {
      if (off + m >= p.Nsp) {
        P.fail(POMCP_E_ARENA);
        break;
      }
      Env::sample_agent_initial(sm, who, oq, draw_model, &s0, &s1);
      pp[m++] = make_uint2(s0, s1);
    }
    tab[q].size = m;
    tab[q].cap = m;
    off += m;
  }
  return off;
}

// The top tree's new root belief at a re-root to `node`: its particle-log
// records in insertion order (rb, returns the count)
template <class Env, int NT, bool kWave>
__device__ int im_extract_root(ImPair<Env, NT>& P, int node, uint4* rb) {
  const ImParams& p = P.p;
  int n = 0;
  const int nlog = P.h.n_log[0];
  if constexpr (kWave) {
    for (int base = 0; base < nlog; base += kWave64) {
      const int i = base + (int)(threadIdx.x & 63);
      IRec r{0u, 0u, 0u, 0u};
      if (i < nlog) r = P.lg[0][i];
      const bool hit = i < nlog && (int)r.node == node;
      const uint64_t m = __ballot(hit);
      if (n + __popcll(m) > p.Nr) {
        P.fail(POMCP_E_ARENA);
        break;
      }
      if (hit) rb[n + __popcll(m & im_lanes_below())] = make_uint4(r.v0, r.v1, r.nested, 0u);
      n += __popcll(m);
    }
  } else {
    for (int i = 0; i < nlog; ++i) {
      const IRec r = P.lg[0][i];
      if ((int)r.node == node) {
        if (n >= p.Nr) {
          P.fail(POMCP_E_ARENA);
          break;
        }
        rb[n++] = make_uint4(r.v0, r.v1, r.nested, 0u);
      }
    }
  }
  return n;
}

// INTMCP.update (intmcp.py:198-300) of a nesting-level-2 or -3 planner: tree
// 0's re-root (or initial belief) and reinvigoration, then each middle
// planner's (tree k = 1 .. NT - 2) _initial_nested_update / _nested_update over
// the history distribution of the belief above (the new root belief for tree
// 1, the nested distribution of tree k - 1's beliefs below that,
// get_nested_history_dist, intmcp.py:334-362, summed over every node of the
// distribution), then the level-0 planner's (tree NT - 1) -- the oracle's
// order (oracle/intmcp.py _Planner.update / _nested_update).
template <class Env, int NT, bool kWave>
__device__ void im_update_nestN(ImPair<Env, NT>& P, const typename Env::Model& sm, uint64_t obs,
                                int action) {
  static_assert(NT >= 3 && NT <= kImMaxT, "a middle tree");
  constexpr int kB = NT - 1;
  const ImParams& p = P.p;
  auto draw_model = [&](uint32_t n) { return P.d_model(n); };
  const bool initial = P.N(0, P.h.cur).t == 0;
  int node, n = 0;
  if (initial) {   // _initial_nested_update, the top level
    node = P.child(0, 0, p.A, obs);
    if (node < 0) return;
    P.traverse(0, node);
    uint32_t s0, s1;
    if (!Env::sample_agent_initial(sm, p.ego, obs, draw_model, &s0, &s1)) P.fail(POMCP_E_INVALID);
    P.h.root_sel ^= 1;
    uint4* rb = P.root_buf(P.h.root_sel);
    while (P.h.err == 0 && (double)n < 1.0 * (double)p.n_target) {
      if (n >= p.Nr) {
        P.fail(POMCP_E_ARENA);
        break;
      }
      Env::sample_agent_initial(sm, p.ego, obs, draw_model, &s0, &s1);
      const uint64_t ok = Env::obs_key(sm, p.other, s0, s1);
      const int c = P.child(1, 0, p.A, ok);
      rb[n++] = make_uint4(s0, s1, (uint32_t)(c < 0 ? 0 : c), 0u);
    }
  } else {         // _nested_update, the top level: re-root to (action, obs)
    node = (action >= 0 && action < p.A) ? P.child(0, P.h.cur, action, obs) : -1;
    if (node < 0) {
      P.fail(POMCP_E_NOT_FOUND);
      return;
    }
    P.traverse(0, node);
    const int prev_size = P.h.root_size;
    P.h.root_sel ^= 1;
    n = im_extract_root<Env, NT, kWave>(P, node, P.root_buf(P.h.root_sel));
    P.h.pad = prev_size;
    if (!im_absorbing(P.N(0, node).info) && P.h.err == 0)
      P.reinvig_top(node, action, obs, p.n_target, &n);   // ceil(1.0 * target)
  }
  P.h.cur = node;
  P.h.root_size = n;
  if (P.h.err != 0 || n == 0) return;
  // ---- the middle planners, top down: tree k's beliefs from the distribution above
  ISup* up_t = nullptr;
  const double* up_p = nullptr;
  uint4* up_q = nullptr;
  int up_n = 0;
  for (int k = 1; k < kB; ++k) {
    const int m = k - 1;
    const int sel1 = P.h.msel[m] ^ 1;
    ISup* t1 = P.mtab(m, sel1);
    uint4* q1 = P.mparts(m, sel1);
    double* pr = P.mprob[m];
    int n1 = 0;
    if (k == 1) im_support<Env, NT, kWave>(P, 1, t1, pr, P.root_buf(P.h.root_sel), n, &n1);
    else im_support_nested<Env, NT>(P, k, up_t, up_p, up_n, up_q, t1, pr, &n1);
    if (n1 == 0) {
      P.fail(POMCP_E_STATE);
      return;
    }
    if (initial) {   // _initial_nested_update, tree k's level
      const int who = P.agent(k);
      uint32_t s0, s1;
      Env::sample_agent_initial(sm, who, P.C(k, t1[0].node).okey, draw_model, &s0, &s1);   // probe
      int off = 0;
      for (int q = 0; q < n1 && P.h.err == 0; ++q) {
        P.traverse(k, t1[q].node);
        const uint64_t oq = P.C(k, t1[q].node).okey;
        t1[q].off = off;
        int c0 = 0;
        while ((double)c0 < pr[q] * (double)p.n_target) {
          if (off + c0 >= p.Nsp) {
            P.fail(POMCP_E_ARENA);
            break;
          }
          Env::sample_agent_initial(sm, who, oq, draw_model, &s0, &s1);
          const uint64_t ok = Env::obs_key(sm, P.agent(k + 1), s0, s1);
          const int c = P.child(k + 1, 0, p.A, ok);
          q1[off + c0++] = make_uint4(s0, s1, (uint32_t)(c < 0 ? 0 : c), 0u);
        }
        t1[q].size = c0;
        t1[q].cap = c0;
        off += c0;
      }
      P.h.msup_used[m] = off;
    } else {         // _nested_update, tree k's level
      im_extract_support<Env, NT, kWave>(P, k, t1, q1, pr, n1);
      if (P.h.err != 0) return;
      P.h.mpad[m] = P.h.n_msup[m];   // the previous table of tree k (parents)
      P.mark_slots(k, P.mtab(m, sel1 ^ 1), P.h.mpad[m], true);
      for (int q = 0; q < n1 && P.h.err == 0; ++q) {
        const int nd = t1[q].node;
        P.traverse(k, nd);
        if (im_absorbing(P.N(k, nd).info)) continue;
        const int tq = (int)ceil(pr[q] * (double)p.n_target);
        P.reinvig_mid(k, nd, (int)im_paction(P.N(k, nd).info), P.C(k, nd).okey, tq, sel1, q);
      }
      P.mark_slots(k, P.mtab(m, sel1 ^ 1), P.h.mpad[m], false);
      int used = 0;
      for (int q = 0; q < n1; ++q) used = max(used, t1[q].off + t1[q].cap);
      P.h.msup_used[m] = used;
    }
    P.h.msel[m] = sel1;
    P.h.n_msup[m] = n1;
    if (P.h.err != 0) return;
    up_t = t1;
    up_p = pr;
    up_q = q1;
    up_n = n1;
  }
  // ---- the level-0 planner: the last middle beliefs' nested history distribution
  const int sel = P.h.sup_sel ^ 1;
  ISup* tab = P.sup_tab(sel);
  int n2 = 0;
  im_support_nested<Env, NT>(P, kB, up_t, up_p, up_n, up_q, tab, P.prob, &n2);
  if (n2 == 0) {
    P.fail(POMCP_E_STATE);
    return;
  }
  if (initial) {
    P.h.sup_used = im_initial_bottom<Env, NT>(P, sm, sel, n2, P.prob);
  } else {
    im_extract_support<Env, NT, kWave>(P, kB, tab, P.sup_parts(sel), P.prob, n2);
    if (P.h.err != 0) return;
    P.h.pad = P.h.n_sup;   // previous support count (parents)
    P.mark_support(sel ^ 1, P.h.pad, true);
    for (int q = 0; q < n2 && P.h.err == 0; ++q) {
      const int nd = tab[q].node;
      P.traverse(kB, nd);
      if (im_absorbing(P.N(kB, nd).info)) continue;
      const int tq = (int)ceil(P.prob[q] * (double)p.n_target);
      P.reinvig_nested(nd, (int)im_paction(P.N(kB, nd).info), P.C(kB, nd).okey, tq, sel, q);
    }
    P.mark_support(sel ^ 1, P.h.pad, false);
    int used = 0;
    for (int q = 0; q < n2; ++q) used = max(used, tab[q].off + tab[q].cap);
    P.h.sup_used = used;
  }
  P.h.sup_sel = sel;
  P.h.n_sup = n2;
  if (P.h.err == 0) P.template clear_old_beliefs<kWave>(P.N(0, node).t);
}

// k_im_update at nesting level 2 or 3 (NT = 3 or 4 trees per pair; as k_im_update)
template <class Env, int NT, bool kWave>
__global__ __launch_bounds__(64) void k_im_updateN(ImParams p) {
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  const int b = kWave ? (int)blockIdx.x : (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (b >= p.B) return;
  ImPair<Env, NT> P(p, sm, b);
  const uint64_t obs = p.in_obs[b];
  if (p.in_actions[b] == kImSkip) {
    p.out[2 * b] = im_absorbing(P.N(0, P.h.cur).info) ? 1 : 0;
    p.out[2 * b + 1] = P.h.err;
    return;
  }
  P.h.num_sims = 0;
  P.h.search_depth = 0;
  if (P.h.err == 0 && !im_absorbing(P.N(0, P.h.cur).info))
    im_update_nestN<Env, NT, kWave>(P, sm, obs, p.in_actions[b]);
  P.h.pad = 0;
  for (int m = 0; m < kImMaxMid; ++m) P.h.mpad[m] = 0;
  P.store();
  p.out[2 * b] = im_absorbing(P.N(0, P.h.cur).info) ? 1 : 0;
  p.out[2 * b + 1] = P.h.err;
}

// INTMCP.update (intmcp.py:198-300) for every pair.
// kWave (few pairs: the drop-in's one): a wave per pair, its 64 lanes running
// the same pair in lockstep (identical state, identical stores) and sharing
// the scans of the episode's particle logs, which grow with every search;
// otherwise a lane per pair.
template <class Env, bool kWave>
__global__ __launch_bounds__(64) void k_im_update(ImParams p) {
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  const int b = kWave ? (int)blockIdx.x : (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (b >= p.B) return;
  ImPair<Env> P(p, sm, b);
  const uint64_t obs = p.in_obs[b];
  const int T = P.top();
  if (p.in_actions[b] == kImSkip) {   // a pair whose episode has ended: untouched
    p.out[2 * b] = im_absorbing(P.N(T, P.h.cur).info) ? 1 : 0;
    p.out[2 * b + 1] = P.h.err;
    return;
  }
  P.h.num_sims = 0;         // the step's counters (intmcp.py:114-136 resets them first)
  P.h.search_depth = 0;
  if (p.nest0) {
    if (P.h.err == 0 && !im_absorbing(P.N(1, P.h.cur).info))
      im_update_nest0<Env, kWave>(P, sm, obs, p.in_actions[b]);
  } else if (P.h.err == 0 && !im_absorbing(P.N(0, P.h.cur).info)) {
    auto draw_model = [&](uint32_t n) { return P.d_model(n); };
    const double* prob = P.prob;
    int nsup = 0;
    if (P.N(0, P.h.cur).t == 0) {
      // _initial_nested_update (intmcp.py:216-268), level 1
      const int node = P.child(0, 0, p.A, obs);
      if (node >= 0) {
        P.traverse(0, node);
        uint32_t s0, s1;
        if (!Env::sample_agent_initial(sm, p.ego, obs, draw_model, &s0, &s1)) P.fail(POMCP_E_INVALID);
        P.h.root_sel ^= 1;
        uint4* rb = P.root_buf(P.h.root_sel);
        int n = 0;
        while (P.h.err == 0 && (double)n < 1.0 * (double)p.n_target) {
          if (n >= p.Nr) {
            P.fail(POMCP_E_ARENA);
            break;
          }
          Env::sample_agent_initial(sm, p.ego, obs, draw_model, &s0, &s1);
          const uint64_t ok = Env::obs_key(sm, p.other, s0, s1);
          const int c = P.child(1, 0, p.A, ok);
          rb[n++] = make_uint4(s0, s1, (uint32_t)(c < 0 ? 0 : c), 0u);
        }
        P.h.cur = node;
        P.h.root_size = n;
        if (P.h.err == 0 && n > 0) {
          // level 0: support of the histories, their initial beliefs
          const int sel = P.h.sup_sel ^ 1;
          im_support<Env, 2, kWave>(P, 1, P.sup_tab(sel), P.prob, P.root_buf(P.h.root_sel), n, &nsup);
          ISup* tab = P.sup_tab(sel);
          const uint64_t o0 = P.C(1, tab[0].node).okey;
          Env::sample_agent_initial(sm, p.other, o0, draw_model, &s0, &s1);   // probe
          int off = 0;
          for (int q = 0; q < nsup && P.h.err == 0; ++q) {
            P.traverse(1, tab[q].node);
            const uint64_t oq = P.C(1, tab[q].node).okey;
            tab[q].off = off;
            tab[q].size = 0;
            uint2* pp = P.sup_parts(sel) + off;
            int m = 0;
            while ((double)m < prob[q] * (double)p.n_target) {
              if (off + m >= p.Nsp) {
                P.fail(POMCP_E_ARENA);
                break;
              }
              Env::sample_agent_initial(sm, p.other, oq, draw_model, &s0, &s1);
              pp[m++] = make_uint2(s0, s1);
            }
            tab[q].size = m;
            tab[q].cap = m;
            off += m;
          }
          P.h.sup_sel = sel;
          P.h.n_sup = nsup;
          P.h.sup_used = off;
        }
      }
    } else {
      // _nested_update (intmcp.py:270-300), level 1: re-root to (action, obs)
      const int action = p.in_actions[b];
      const int node = (action >= 0 && action < p.A) ? P.child(0, P.h.cur, action, obs) : -1;
      if (node < 0) {
        P.fail(POMCP_E_NOT_FOUND);
      } else {
        P.traverse(0, node);
        // its belief: log records of `node`, insertion order
        const int prev_size = P.h.root_size;
        P.h.root_sel ^= 1;
        uint4* rb = P.root_buf(P.h.root_sel);
        int n = 0;
        const int nlog = P.h.n_log[0];
        if constexpr (kWave) {
          for (int base = 0; base < nlog; base += kWave64) {
            const int i = base + (int)(threadIdx.x & 63);
            IRec r{0u, 0u, 0u, 0u};
            if (i < nlog) r = P.lg[0][i];
            const bool hit = i < nlog && (int)r.node == node;
            const uint64_t m = __ballot(hit);
            if (n + __popcll(m) > p.Nr) {
              P.fail(POMCP_E_ARENA);
              break;
            }
            if (hit) rb[n + __popcll(m & im_lanes_below())] = make_uint4(r.v0, r.v1, r.nested, 0u);
            n += __popcll(m);
          }
        } else {
          for (int i = 0; i < nlog; ++i) {
            const IRec r = P.lg[0][i];
            if ((int)r.node == node) {
              if (n >= p.Nr) {
                P.fail(POMCP_E_ARENA);
                break;
              }
              rb[n++] = make_uint4(r.v0, r.v1, r.nested, 0u);
            }
          }
        }
        P.h.pad = prev_size;
        if (!im_absorbing(P.N(0, node).info) && P.h.err == 0)
          P.reinvig_top(node, action, obs, p.n_target, &n);   // ceil(1.0 * target)
        P.h.cur = node;
        P.h.root_size = n;
        // level 0: support of the new root belief, materialised + reinvigorated
        if (P.h.err == 0 && n > 0) {
          const int sel = P.h.sup_sel ^ 1;
          im_support<Env, 2, kWave>(P, 1, P.sup_tab(sel), P.prob, P.root_buf(P.h.root_sel), n, &nsup);
          im_extract_support<Env, 2, kWave>(P, 1, P.sup_tab(sel), P.sup_parts(sel), P.prob, nsup);
          ISup* tab = P.sup_tab(sel);
          P.h.pad = P.h.n_sup;   // previous support count (parents)
          P.mark_support(sel ^ 1, P.h.pad, true);   // parents found by node, not by scan
          for (int q = 0; q < nsup && P.h.err == 0; ++q) {
            const int m = tab[q].node;
            P.traverse(1, m);
            if (im_absorbing(P.N(1, m).info)) continue;
            const int tq = (int)ceil(prob[q] * (double)p.n_target);
            P.reinvig_nested(m, (int)im_paction(P.N(1, m).info), P.C(1, m).okey, tq, sel, q);
          }
          P.mark_support(sel ^ 1, P.h.pad, false);
          int used = 0;
          for (int q = 0; q < nsup; ++q) used = max(used, tab[q].off + tab[q].cap);
          P.h.sup_sel = sel;
          P.h.n_sup = nsup;
          P.h.sup_used = used;
        } else {
          P.h.sup_sel ^= 1;
          P.h.n_sup = 0;
          P.h.sup_used = 0;
        }
        if (P.h.err == 0) P.template clear_old_beliefs<kWave>(P.N(0, node).t);
      }
    }
  }
  P.h.pad = 0;
  P.store();
  p.out[2 * b] = im_absorbing(P.N(T, P.h.cur).info) ? 1 : 0;
  p.out[2 * b + 1] = P.h.err;
}

// INTMCP.get_action (intmcp.py:368-408): sims[0] simulations at level 0, then
// sims[1] at level 1; kImBegin resets the step's counters, kImFinal runs the
// final action selection.  A fixed-count search is one launch with both flags;
// the wall-clock loop of the reference is several launches.
constexpr int kImBegin = 1, kImFinal = 2;
template <class Env>
__global__ __launch_bounds__(64) void k_im_search(ImParams p, int sims0, int sims1, int flags) {
  __shared__ typename Env::Model sm;
  __shared__ double slog[kImLogLds];                  // math.log(N): no global load per selection
  __shared__ uint4 srv[kImRootWords * kWave];         // level-1 root views, one column per lane
  __shared__ double sdp[kImDpowLds];                  // discount powers (rollout)
  __shared__ uint64_t sexp[256];                      // host_exp's 2^(k/128) table
  for (int i = threadIdx.x; i < 256; i += blockDim.x) sexp[i] = kHostExpTab[i];
  const int ltn = p.logtab_n < kImLogLds ? (int)p.logtab_n : kImLogLds;
  for (int i = threadIdx.x; i < ltn; i += blockDim.x) slog[i] = p.logtab[i];
  const bool dp_lds = p.dpow_n <= kImDpowLds;
  if (dp_lds)
    for (int i = threadIdx.x; i < p.dpow_n; i += blockDim.x) sdp[i] = p.dpow[i];
  stage_model(p.model, sm);                           // (synchronises)
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.B) return;
  ImPair<Env> P(p, sm, b);
  P.lt_lds = slog;
  P.lt_n = ltn;
  P.rv = srv + threadIdx.x;
  if (dp_lds) P.dp = sdp;
  P.exp_tab = sexp;
#ifdef POMCP_PHASE_TIMING
  P.pt_last = __builtin_amdgcn_s_memtime();
#endif
  if (flags & kImBegin) {
    P.h.num_sims = 0;
    P.h.search_depth = 0;
  }
  const int root = P.h.cur;
  const int T = P.top();
  if (p.nest0) sims1 = 0;   // one level: the planner's own tree
  int action = 0;
  if (P.h.err == 0 && !im_absorbing(P.N(T, root).info) && P.N(T, root).t > 0) {
    uint4* rb = P.root_buf(P.h.root_sel);
    // _nested_sim(history, level, top_level=True) of the level-1 planner
    // (intmcp.py:410-442) starts with traverse + expand of the root: no draws,
    // and no-ops once done, so they run once per launch.  The depleted-root
    // branch cannot be reached with a valid configuration.
    if (sims0 + sims1 > 0) {
      P.traverse(T, root);
      if (im_nreg(P.N(T, root).info) == 0) P.expand(T, root);
      if (P.h.root_size == 0 || P.h.root_size < p.extra) P.fail(POMCP_E_UNSUPPORTED);
    }
    const ISup* const stab = P.sup_tab(P.h.sup_sel);
    const uint2* const sparts = P.sup_parts(P.h.sup_sel);
    for (int level = 0; level < 2 && P.h.err == 0; ++level) {
      const int num_sims = level == 0 ? sims0 : sims1;
      // the root particle of the next simulation (belief.py:55; the level-1
      // planner's own stream, which nothing else draws during a search) and,
      // at level 0, its history's support entry: loaded one simulation ahead
      uint4 hp_next = make_uint4(0, 0, 0, 0);
      ISup e_next = {0, 0, 0, 0};
      if (num_sims > 0) {
        // nesting level 0: every simulation starts at the root, support entry 0
        if (!p.nest0) hp_next = rb[P.d_bel(0, (uint32_t)P.h.root_size)];
        if (level == 0) e_next = stab[p.nest0 ? 0u : hp_next.w];
        if (level == 1) {   // the root's view, kept current by the backups (ImPair::rv)
          P.rv_put(P.view(0, root));
          P.rv_root = root;
        }
      }
      for (int s = 0; s < num_sims && P.h.err == 0; ++s) {
        const uint4 hp = hp_next;
        const ISup e = e_next;
        if (s + 1 < num_sims && !p.nest0) {
          hp_next = rb[P.d_bel(0, (uint32_t)P.h.root_size)];
          if (level == 0) e_next = stab[hp_next.w];
        }
        if (level == 0) {
          // the level-0 planner's _nested_sim at the particle's history: its
          // node + statistics and the support particle in one round trip
          const int n = p.nest0 ? root : (int)hp.z;
          if (e.size == 0) {
            P.fail(POMCP_E_UNSUPPORTED);   // depleted level-0 node (unreachable)
            break;
          }
          const uint2 q = sparts[e.off + P.d_bel(1, (uint32_t)e.size)];
          auto v = P.view(1, n);
          P.la_fill();   // the RNG words, while the start node's view is in flight
          if (n > 0 && !im_path_ok(v.x.info)) {
            P.traverse(1, n);         // (n itself only gains the path_ok bit)
            v.x.info |= 1u << 4;
          }
          if (im_nreg(v.x.info) == 0) {
            P.expand_known(1, n, v.x);   // nothing registered: fresh, zero statistics
#pragma unroll
            for (int q = 0; q < ImPair<Env>::kNA; ++q) v.sh[q] = make_uint4(0, 0, 0, 0);
          }
          IM_MARK_P(IP_START);
          const int d = P.simulate(1, q.x, q.y, 0u, n, v);
          P.N(1, n).visits = v.x.visits + 1;   // (simulate writes no INode of its start)
          if (p.nest0 && d > P.h.search_depth) P.h.search_depth = d;
        } else {
          const auto v = P.rv_get();
          IM_MARK_P(IP_START);
          const int d = P.simulate(0, hp.x, hp.y, hp.z, root, v);
          P.N(0, root).visits = v.x.visits + 1;
          P.rv[0].z = (uint32_t)(v.x.visits + 1);   // INode.visits: bytes 8-11
          if (d > P.h.search_depth) P.h.search_depth = d;
        }
        P.h.num_sims += 1;
        IM_MARK_P(IP_SIMEND);
      }
    }
#ifdef POMCP_PHASE_TIMING
    if (p.timing != nullptr)
      for (int i = 0; i < kImPhases; ++i) p.timing[(int64_t)b * kImPhases + i] += P.pt[i];
#endif
    if (!(flags & kImFinal) || P.h.err != 0) {   // no action from a failed search
      if (P.h.err != 0 && (flags & kImFinal)) P.h.last_action = -1;
      P.store_search();
      return;
    }
    // max_value_action_selection (intmcp.py:718-732)
    const INode x = P.N(T, root);
    const int nr = im_nreg(x.info);
    if (nr == 0) {
      action = (int)P.d_sel((uint32_t)p.A);
    } else {
      double mx = -__builtin_inf();
      int ties[6], nt = 0;
      for (int i = 0; i < nr; ++i) {
        const int a = im_order(x.info, i);
        const uint32_t* const hd = P.H(T, root, a);
        const double v = hilo_d(hd[1], hd[2]);
        if (v == mx) {
          ties[nt++] = a;
        } else if (v > mx) {
          mx = v;
          ties[0] = a;
          nt = 1;
        }
      }
      action = ties[P.d_sel((uint32_t)nt)];
    }
  }
  if (flags & kImFinal) P.h.last_action = action;
  P.store_search();
}

// INTMCP.get_action (intmcp.py:368-408) at nesting level NT - 1 >= 2:
// sims[l] simulations at level l = 0 .. NT - 1 in turn.  Every simulation
// samples a root particle of the top planner (its stream); below the top it
// dispatches down the levels (_nested_sim, intmcp.py:410-442): each middle
// planner's traverse + expand of the particle's history node and a particle
// of its belief (its stream), down to the planner whose level is the search
// level, which runs _simulate.  (Correctness first: a plain serial lane per
// pair, no lookahead of the next particle.)
template <class Env, int NT>
__global__ __launch_bounds__(64) void k_im_searchN(ImParams p, ImSims sims, int flags) {
  static_assert(NT >= 3 && NT <= kImMaxT, "a middle tree");
  constexpr int kB = NT - 1;
  __shared__ typename Env::Model sm;
  __shared__ double slog[kImLogLds];
  __shared__ uint4 srv[kImRootWords * kWave];
  __shared__ double sdp[kImDpowLds];
  __shared__ uint64_t sexp[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) sexp[i] = kHostExpTab[i];
  const int ltn = p.logtab_n < kImLogLds ? (int)p.logtab_n : kImLogLds;
  for (int i = threadIdx.x; i < ltn; i += blockDim.x) slog[i] = p.logtab[i];
  const bool dp_lds = p.dpow_n <= kImDpowLds;
  if (dp_lds)
    for (int i = threadIdx.x; i < p.dpow_n; i += blockDim.x) sdp[i] = p.dpow[i];
  stage_model(p.model, sm);   // (synchronises)
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.B) return;
  ImPair<Env, NT> P(p, sm, b);
  P.lt_lds = slog;
  P.lt_n = ltn;
  P.rv = srv + threadIdx.x;
  if (dp_lds) P.dp = sdp;
  P.exp_tab = sexp;
  if (flags & kImBegin) {
    P.h.num_sims = 0;
    P.h.search_depth = 0;
  }
  const int root = P.h.cur;
  int action = 0;
  if (P.h.err == 0 && !im_absorbing(P.N(0, root).info) && P.N(0, root).t > 0) {
    const uint4* const rb = P.root_buf(P.h.root_sel);
    int any = 0;
#pragma unroll
    for (int l = 0; l < NT; ++l) any += sims.s[l];
    if (any > 0) {   // the top planner's _nested_sim head (no draws)
      P.traverse(0, root);
      if (im_nreg(P.N(0, root).info) == 0) P.expand(0, root);
      if (P.h.root_size == 0 || P.h.root_size < p.extra) P.fail(POMCP_E_UNSUPPORTED);
    }
    const ISup* const t2 = P.sup_tab(P.h.sup_sel);
    const uint2* const q2s = P.sup_parts(P.h.sup_sel);
    for (int level = 0; level < NT && P.h.err == 0; ++level) {
      const int num_sims = sims.s[level];
      if (level == kB && num_sims > 0) {   // the root's view, kept current by the backups
        P.rv_put(P.view(0, root));
        P.rv_root = root;
      }
      const int kt = kB - level;   // the tree that simulates
      for (int s = 0; s < num_sims && P.h.err == 0; ++s) {
        const uint4 hp = rb[P.d_bel(0, (uint32_t)P.h.root_size)];
        if (kt == 0) {
          const auto v = P.rv_get();
          const int d = P.simulate(0, hp.x, hp.y, hp.z, root, v);
          P.N(0, root).visits = v.x.visits + 1;
          P.rv[0].z = (uint32_t)(v.x.visits + 1);
          if (d > P.h.search_depth) P.h.search_depth = d;
        } else {
          // each middle planner's _nested_sim at the particle's history, down to tree kt
          uint32_t nx = hp.z, slot = hp.w;
          for (int k = 1; k <= kt; ++k) {
            const int nk = (int)nx;
            const ISup e = k < kB ? P.mtab(k - 1, P.h.msel[k - 1])[slot] : t2[slot];
            P.traverse(k, nk);
            if (im_nreg(P.N(k, nk).info) == 0) P.expand(k, nk);
            if (e.size == 0) {
              P.fail(POMCP_E_UNSUPPORTED);   // depleted node (not reached by the goldens)
              break;
            }
            if (k < kB) {
              const uint4 q = P.mparts(k - 1, P.h.msel[k - 1])[e.off + P.d_bel(k, (uint32_t)e.size)];
              if (k == kt) {
                auto v = P.view(k, nk);
                P.simulate(k, q.x, q.y, q.z, nk, v);
                P.N(k, nk).visits = v.x.visits + 1;
              }
              nx = q.z;
              slot = q.w;
            } else {
              const uint2 q = q2s[e.off + P.d_bel(kB, (uint32_t)e.size)];
              auto v = P.view(kB, nk);
              P.simulate(kB, q.x, q.y, 0u, nk, v);
              P.N(kB, nk).visits = v.x.visits + 1;
            }
          }
          if (P.h.err != 0) break;
        }
        P.h.num_sims += 1;
      }
    }
    if (!(flags & kImFinal) || P.h.err != 0) {
      if (P.h.err != 0 && (flags & kImFinal)) P.h.last_action = -1;
      P.store_search();
      return;
    }
    // max_value_action_selection (intmcp.py:718-732)
    const INode x = P.N(0, root);
    const int nr = im_nreg(x.info);
    if (nr == 0) {
      action = (int)P.d_sel((uint32_t)p.A);
    } else {
      double mx = -__builtin_inf();
      int ties[6], nt = 0;
      for (int i = 0; i < nr; ++i) {
        const int a = im_order(x.info, i);
        const uint32_t* const hd = P.H(0, root, a);
        const double v = hilo_d(hd[1], hd[2]);
        if (v == mx) {
          ties[nt++] = a;
        } else if (v > mx) {
          mx = v;
          ties[0] = a;
          nt = 1;
        }
      }
      action = ties[P.d_sel((uint32_t)nt)];
    }
  }
  if (flags & kImFinal) P.h.last_action = action;
  P.store_search();
}

template <class Env>
__global__ __launch_bounds__(64) void k_im_synthetic(ImParams p, uint64_t env_seed_base) {
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.B) return;
  Streams env;
  env.seed = env_seed_base + (uint64_t)b;
  env.tree = 0x40000000u;
  for (int k = 0; k < 5; ++k) env.ctr[k] = 0;
  uint32_t s0, s1;
  Env::sample_initial(sm, [&](uint32_t n) { return env.model(n); }, &s0, &s1);
  p.out_obs[b] = Env::obs_key(sm, p.nest0 ? p.other : p.ego, s0, s1);
}

}  // namespace pb
