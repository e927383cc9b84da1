// POMCP per-simulation loop as hand-written HIP kernels for gfx950 (CDNA4).
//
// Replaces posggym_baselines/planning/mcts.py:269-452 (get_action, _simulate,
// _rollout, UCB/PUCB/min-visit selection, final action choice),
// node.py (ObsNode/ActionNode -> 128 B action records with inline children),
// belief.py (ParticleBelief -> particle log + root belief buffer,
// BeliefRejectionSampler -> k_update) and utils.py:15-42 (MinMaxStats -> two
// registers).  One wavefront per tree; see pomcp_device.h for the lane map.
//
// FP64 arithmetic follows the reference's operation order exactly and is built
// with -ffp-contract=off; log(N) and discount**k come from host tables computed
// with Python's own math.log / float.__pow__ (DESIGN.md "bit-exactness").
#pragma clang fp contract(off)

#include "pomcp_device.h"
#include "envs.h"
#include "host_exp.h"

namespace pb {

__device__ __forceinline__ double hilo(uint32_t lo, uint32_t hi) {
  return __hiloint2double((int)hi, (int)lo);
}
__device__ __forceinline__ uint4 pack_stats0(int visits, double value) {
  return make_uint4((uint32_t)visits, 0u, (uint32_t)__double2loint(value),
                    (uint32_t)__double2hiint(value));
}
__device__ __forceinline__ uint4 pack_stats1(double total, double agg) {
  return make_uint4((uint32_t)__double2loint(total), (uint32_t)__double2hiint(total),
                    (uint32_t)__double2loint(agg), (uint32_t)__double2hiint(agg));
}

// Result of looking up / inserting an obs child (ActionNode.children[obs]).
struct ChildRef {
  uint32_t id;        // obs node id (particle log key)
  int blk;            // action block of the child (-1 = leaf)
  int visits;         // ObsNode.visits after this visit
  int absorbing;
  int code;           // type-based: the child's prior code (pomcp_device.h kCodeShift)
  int lane;           // lane holding the inline slot in the level registers (-1: overflow)
  int32_t* blk_ptr;   // where the child's block index lives (for expansion)
};

template <class Env>
struct Tree {
  using Model = typename Env::Model;
  const DevParams& p;
  const Model& m;
  int tree, lane;
  Line* an;
  OvfSlot* ovf;
  uint4* bel;
  int n_blocks, n_log, n_nodes, err, bsize, bsel, epoch, root_t;
  uint32_t root_id;
  int root_blk, root_visits, root_abs;
  double mm_min, mm_max;
  uint64_t seed;
  uint32_t tkey;
  uint32_t c_belief, c_select, c_model, c_act0, c_act1, c_mix;
  int root_code;
  LdsStream r_belief, r_model, r_act0, r_act1;
  int64_t c_levels, c_expand, c_new, c_rollout, c_probes;

  __device__ Tree(const DevParams& pp, const Model& mm, int t) : p(pp), m(mm), tree(t) {
    lane = lane_id();
    an = p.an + tree_base_lines(t, p.Nb, p.lines);
    ovf = p.ovf + (int64_t)t * p.H;
    bel = p.belief + (int64_t)t * p.Nr;
    const TreeHdr h = p.hdr[t];
    n_blocks = uni(h.n_blocks);
    n_log = uni(h.n_log);
    n_nodes = uni(h.n_nodes);
    err = uni(h.error);
    bsize = uni(h.belief_size);
    bsel = uni(h.belief_sel);
    epoch = uni(h.epoch);
    root_t = uni(h.root_t);
    root_id = uniu(h.root_id);
    root_blk = uni(h.root_blk);
    root_visits = uni(h.root_visits);
    root_abs = uni(h.root_abs);
    mm_min = uni_d(h.mm_min);
    mm_max = uni_d(h.mm_max);
    seed = uni64(h.seed);
    tkey = uniu(h.tree_key);
    c_belief = uniu(h.ctr[0]);
    c_select = uniu(h.ctr[1]);
    c_model = uniu(h.ctr[2]);
    c_act0 = uniu(h.ctr[3]);
    c_act1 = uniu(h.ctr[4]);
    c_mix = uniu(h.ctr_mix);
    root_code = uni(h.root_code);
    c_levels = c_expand = c_new = c_rollout = c_probes = 0;
  }

  __device__ void warm_rng(uint32_t* lds) {   // lds: 4 x kRngPage words for this wave
    r_belief.page = lds;
    r_model.page = lds + kRngPage;
    r_act0.page = lds + 2 * kRngPage;
    r_act1.page = lds + 3 * kRngPage;
    r_belief.refill(seed, tkey, S_BELIEF, c_belief / kRngPage);
    r_model.refill(seed, tkey, S_MODEL, c_model / kRngPage);
    r_act0.refill(seed, tkey, S_ACT_BASE, c_act0 / kRngPage);
    r_act1.refill(seed, tkey, S_ACT_BASE + 1, c_act1 / kRngPage);
  }

  __device__ void store_header() {
    if (lane != 0) return;
    TreeHdr h;
    h.n_blocks = n_blocks;
    h.n_log = n_log;
    h.n_nodes = n_nodes;
    h.error = err;
    h.belief_size = bsize;
    h.belief_sel = bsel;
    h.epoch = epoch;
    h.root_t = root_t;
    h.root_id = root_id;
    h.root_blk = root_blk;
    h.root_visits = root_visits;
    h.root_abs = root_abs;
    h.mm_min = mm_min;
    h.mm_max = mm_max;
    h.seed = seed;
    h.tree_key = tkey;
    h.ctr[0] = c_belief;
    h.ctr[1] = c_select;
    h.ctr[2] = c_model;
    h.ctr[3] = c_act0;
    h.ctr[4] = c_act1;
    h.root_code = root_code;
    h.ctr_mix = c_mix;
    p.hdr[tree] = h;
  }

  // ------------------------------------------------------------- RNG draws
  __device__ __forceinline__ uint32_t draw(LdsStream& cs, uint32_t& ctr, uint32_t stream) {
    const uint32_t j = ctr++;
    if ((j & (kRngPage - 1)) == 0u) cs.refill(seed, tkey, stream, j / kRngPage);
    return cs.get(j);
  }
  __device__ uint32_t d_belief(uint32_t n) { return uniform_int(draw(r_belief, c_belief, S_BELIEF), n); }
  __device__ uint32_t d_model(uint32_t n) { return uniform_int(draw(r_model, c_model, S_MODEL), n); }
  __device__ uint32_t d_act(int agent, uint32_t n) {
    return agent == 0 ? uniform_int(draw(r_act0, c_act0, S_ACT_BASE), n)
                      : uniform_int(draw(r_act1, c_act1, S_ACT_BASE + 1), n);
  }
  __device__ uint32_t d_select(uint32_t n) {
    return uniform_int(uniu(philox_word(seed, tkey, S_SELECT, c_select++)), n);
  }
  __device__ double d_select_float() {
    return uniform_float(uniu(philox_word(seed, tkey, S_SELECT, c_select++)));
  }

  // record i of the root belief / of the belief being built (pomcp_device.h
  // bel_at: one from each end of the tree's region); the room of the latter
  __device__ uint4* rbel(int64_t i) { return bel + bel_at(bsel, p.Nr, i); }
  __device__ uint4* obel(int64_t i) { return bel + bel_at(bsel ^ 1, p.Nr, i); }
  __device__ int64_t obel_room() const { return p.Nr - (int64_t)bsize; }

  __device__ uint4 load_block(int blk) const {
    uint4 q = make_uint4(0, 0, 0, 0);
    if (lane < blk_parts(p.lines)) q = reinterpret_cast<const uint4*>(an + (int64_t)blk * blk_stride_lines(p.lines))[lane];
    return q;
  }

  // ObsNode.add_child for every action (mcts.py:279-281, 318-321): zeroed block.
  __device__ int alloc_block() {
    if (n_blocks >= p.Nb) {
      err = POMCP_E_ARENA;
      return -1;
    }
    const int b = n_blocks++;
    if (lane < blk_parts(p.lines))
      reinterpret_cast<uint4*>(an + (int64_t)b * blk_stride_lines(p.lines))[lane] = make_uint4(0, 0, 0, 0);
    ++c_expand;
    return b;
  }

  __device__ void mm_update(double v) {     // utils.py:29-32
    if (v > mm_max) mm_max = v;
    if (v < mm_min) mm_min = v;
  }

  __device__ double normalize(double v) const {   // utils.py:34-39
    if (mm_max > mm_min) return (v - mm_min) / (mm_max - mm_min);
    return v;
  }

  // model.step (belief.py:165-170): Driving draws its execution-order shuffle
  // from the model stream first; the ego's next observation key
  __device__ void joint_step(uint32_t s0, uint32_t s1, int ego_a, int oth_a, uint32_t* n0,
                             uint32_t* n1, uint64_t* okey) {
    const uint32_t j = Env::kStepDraws ? d_model(2) : 0u;
    double r;
    int done;
    Env::step(m, p.ego, s0, s1, (uint32_t)ego_a, (uint32_t)oth_a, j, n0, n1, &r, &done);
    *n0 = uniu(*n0);
    *n1 = uniu(*n1);
    *okey = uni64(Env::obs_key(m, p.ego, *n0, *n1));
  }

  // Overflow map (children beyond the kSlots inline ones).
  __device__ bool ovf_lookup(uint32_t ani, uint64_t okey, bool insert, int init_visits,
                             int absorbing, ChildRef* c, bool* is_new) {
    const uint64_t key = okey | ((uint64_t)epoch << kEpochShift);
    uint32_t b = ovf_hash(ani, okey) & p.bucket_mask;
    *is_new = false;
    for (uint32_t probe = 0; probe <= p.bucket_mask; ++probe) {
      ++c_probes;
      uint4 s = make_uint4(0, 0, 0, 0), s2 = make_uint4(0, 0, 0, 0);
      OvfSlot* e = ovf + (int64_t)b * kBucket + (lane & (kBucket - 1));
      if (lane < kBucket) {
        s = reinterpret_cast<const uint4*>(e)[0];
        s2 = reinterpret_cast<const uint4*>(e)[1];
      }
      const uint64_t skey = (uint64_t)s.x | ((uint64_t)s.y << 32);
      const bool valid = lane < kBucket && (uint32_t)(skey >> kEpochShift) == (uint32_t)epoch;
      const uint64_t m = __ballot(valid && skey == key && s.z == ani);
      const uint32_t base = (uint32_t)(b * kBucket);
      if (m) {
        const int L = __ffsll((long long)m) - 1;
        c->id = p.ovf_base + base + (uint32_t)L;
        c->blk = rl((int)s2.x, L);
        c->visits = rl((int)s2.y, L);
        c->absorbing = rl((int)s.w, L) & 1;
        c->code = (rl((int)s.w, L) >> 1) & 15;
        c->lane = -1;
        c->blk_ptr = &(ovf + (int64_t)b * kBucket + L)->block;
        return true;
      }
      const uint64_t em = __ballot(lane < kBucket && !valid);
      if (em) {
        if (!insert) return false;
        const int L = __ffsll((long long)em) - 1;
        if (lane == L) {
          reinterpret_cast<uint4*>(e)[0] =
              make_uint4((uint32_t)key, (uint32_t)(key >> 32), ani, (uint32_t)absorbing);
          reinterpret_cast<uint4*>(e)[1] = make_uint4((uint32_t)-1, (uint32_t)init_visits, 0u, 0u);
        }
        c->id = p.ovf_base + base + (uint32_t)L;
        c->blk = -1;
        c->visits = init_visits;
        c->absorbing = absorbing;
        c->code = 0;
        c->lane = -1;
        c->blk_ptr = &(ovf + (int64_t)b * kBucket + L)->block;
        *is_new = true;
        ++n_nodes;
        ++c_new;
        return true;
      }
      b = (b + 1) & p.bucket_mask;
    }
    err = POMCP_E_ARENA;
    return false;
  }

  // ActionNode.children lookup for action a of the block `blk` held in q.
  // Search path (visit): visits += 1 / new child with init_visits=1, is_absorbing
  // overwritten (mcts.py:358-370).  Update path: no visit count change; new
  // child with init_visits=0 and the root's absorbing flag (mcts.py:240-247).
  __device__ bool child_ref(uint4& q, int blk, int a, uint64_t okey, bool visit, int done,
                            ChildRef* c) {
    const uint32_t ani = (uint32_t)(blk * p.A + a);
    const int lo = part_slot(a, 0);   // block layout: pomcp_device.h
    const bool cl = lane >= lo && lane < lo + p.islots;
    const uint64_t skey = (uint64_t)q.x | ((uint64_t)q.y << 32);
    const bool valid = cl && (skey & kValidBit) != 0;
    const uint64_t m = __ballot(valid && (skey & kObsMask) == okey);
    uint4* slots = reinterpret_cast<uint4*>(an + (int64_t)blk * blk_stride_lines(p.lines)) + lo;
    int L;
    bool is_new = false;
    if (m) {
      L = __ffsll((long long)m) - 1;
      c->blk = rl((int)q.z, L);
      c->visits = rl((int)q.w, L);
      c->absorbing = (int)(rlu(q.y, L) >> 31);
      c->code = (int)((rlu(q.y, L) >> (kCodeShift - 32)) & 15u);
    } else {
      const uint64_t em = __ballot(cl && (skey & kValidBit) == 0);
      if (!em) {   // all inline slots taken: overflow map
        bool nw;
        if (!ovf_lookup(ani, okey, true, visit ? 1 : 0, done, c, &nw)) return false;
        if (!nw && visit) {
          c->visits += 1;
          c->absorbing = done;
          OvfSlot* e = ovf + (int64_t)(c->id - p.ovf_base);
          if (lane == 0) {
            e->visits = c->visits;
            e->flags = (uint32_t)done | ((uint32_t)c->code << 1);
          }
        }
        return true;
      }
      L = __ffsll((long long)em) - 1;
      c->blk = -1;
      c->visits = 0;
      c->absorbing = done;
      c->code = 0;   // a root made by update: the meta-policy's expected prior
      is_new = true;
      ++n_nodes;
      ++c_new;
    }
    const int k = L - lo;
    if (visit) {
      c->visits += 1;
      c->absorbing = done;
    }
    if (visit || is_new) {
      const uint64_t nk = okey | kValidBit | ((uint64_t)c->absorbing << 63) |
                          ((uint64_t)c->code << kCodeShift);
      const uint4 ns = make_uint4((uint32_t)nk, (uint32_t)(nk >> 32), (uint32_t)c->blk,
                                  (uint32_t)c->visits);
      if (lane == L) {
        slots[k] = ns;
        q = ns;
      }
    }
    c->id = ani * kSlots + (uint32_t)k + 1u;
    c->lane = L;
    c->blk_ptr = reinterpret_cast<int32_t*>(slots + k) + 2;
    return true;
  }

  // model.sample_agent_initial_state (mcts.py:179-198), model-stream draws
  __device__ bool sample_agent_initial(uint64_t obs, uint32_t* s0, uint32_t* s1) {
    const bool ok = Env::sample_agent_initial(m, p.ego, obs,
                                              [&](uint32_t n) { return d_model(n); }, s0, s1);
    *s0 = uniu(*s0);
    *s1 = uniu(*s1);
    return ok;
  }
};

// ---------------------------------------------------------------- kernels

__device__ void clear_ovf(const DevParams& p, int tree, int lane) {
  uint4* hs = reinterpret_cast<uint4*>(p.ovf + (int64_t)tree * p.H);
  for (int64_t i = lane; i < 2 * p.H; i += kWave) hs[i] = make_uint4(0, 0, 0, 0);
}

__global__ __launch_bounds__(256) void k_reset(DevParams p) {
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  const int lane = lane_id();
  TreeHdr h = p.hdr[tree];
  int epoch = (h.epoch + 1) & (int)kEpochMask;
  if (epoch == 0) {   // generation counter wrapped: clear this tree's overflow map
    clear_ovf(p, tree, lane);
    epoch = 1;
  }
  if (lane == 0 && (tree & (kWave - 1)) == 0) p.wlog[tree / kWave] = 0u;
  if (lane == 0) {
    h.n_blocks = 0;
    h.n_log = 0;
    h.n_nodes = 1;
    h.error = 0;
    h.belief_size = 0;
    h.epoch = epoch;
    h.root_t = 0;
    h.root_id = kRootId;
    h.root_blk = -1;
    h.root_visits = 0;
    h.root_abs = 0;
    h.mm_max = p.has_kb ? p.kb_max : -__builtin_inf();   // utils.py:21-27
    h.mm_min = p.has_kb ? p.kb_min : __builtin_inf();
    p.hdr[tree] = h;
  }
}

// Re-root, step 1 (MCTS._update, mcts.py:236-247): find or create the root's
// child (action, obs) and publish its log id (the records k_compact_log
// extracts into the new root belief) and its block / flags (k_compact's new
// root, k_update's new root fields).
template <class Env>
__global__ __launch_bounds__(256) void k_reroot_child(DevParams p) {
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  Tree<Env> T(p, sm, tree);
  uint32_t want = 0xFFFFFFFFu;
  int4 info = make_int4(-1, 0, 0, 0);
  if (T.err == 0 && !T.root_abs && T.root_t > 0) {
    const int action = uni(p.in_actions[tree]);
    if (T.root_blk >= 0 && action >= 0 && action < p.A) {
      uint4 q = T.load_block(T.root_blk);
      ChildRef c;
      if (T.child_ref(q, T.root_blk, action, uni64(p.in_obs[tree]), false, T.root_abs, &c)) {
        want = c.id | ((uint32_t)(tree & (kWave - 1)) << kIdBits);
        info = make_int4(c.blk, c.absorbing, c.code, 1);
      }
    }
  }
  T.store_header();   // child_ref may have created the child (n_nodes)
  if (T.lane == 0) {
    p.want[tree] = want;
    p.want_info[tree] = info;
  }
}

// Re-root, step 3 (k_compact_log below): one WORKGROUP (kLogWaves waves) per
// SEARCH wave scans that wave's shared log once, in order.  A pass reads
// kLogRecs x 64 kLogWaves consecutive records (sub-pass j: record base + j T +
// thread); all of a pass's loads are issued together and the next pass's while
// it runs.  (One wave per log took ~0.3 s at 65,536 trees x 65,536
// simulations: one dependent round trip per 64 records.)
// 16 waves (1,024 threads, one workgroup per CU), 3 records per thread: 3,072
// records per pass.  The update()-inclusive PursuitEvasion step's update:
// 4 -> 16 waves 142 -> 130 ms (2 waves 237 ms, profiles/r5w_log_waves_ab.txt);
// at 16 waves 4 -> 3 records 115 -> 107.6 ms with 128 VGPRs (the most 1,024
// threads allow; 2 records 111 ms, profiles/r5zc_compact_log_ab.txt)
// LDS: k_compact_log takes ~118-123 KB of static LDS at 16 waves (the visits
// table / deferred-children hash, the places queue, the wave's cmap): it needs
// gfx950's 160 KB per workgroup -- a target with 64 KB fails to compile (the
// static allocation exceeds the limit), it cannot launch wrongly sized.
#ifndef PB_LOG_WAVES   // A/B builds only
#define PB_LOG_WAVES 16
#endif
constexpr int kLogWaves = PB_LOG_WAVES;
#ifndef PB_LOG_RECS   // A/B builds only
#define PB_LOG_RECS 3
#endif
constexpr int kLogRecs = PB_LOG_RECS;   // records per thread per pass
// The streaming scan's materialising pass (k_compact_log<Env, true>): 8 waves,
// so two of its workgroups share a CU (round 6 A/B: 16 -> 8 waves with two
// per CU took the legacy scan's update 211 -> 177 ms,
// profiles/r6c_philox7_and_logscan_ab.txt)
#ifndef PB_MAT_WAVES   // A/B builds only
#define PB_MAT_WAVES 8
#endif
constexpr int kMatWaves = PB_MAT_WAVES;
// The streaming scan's segments (k_log_filter): 512 threads x 4 records
constexpr int kLfThreads = 512;
constexpr int kLfRecs = 4;
constexpr int kLfSeg = kLfThreads * kLfRecs;
// consecutive segments of one log per claim (and look-back record); round 6
// A/B 8 -> 32: update 161 -> 149 ms (profiles/r6i_lf_chunk_ab.txt)
#ifndef PB_LF_CHUNK   // A/B builds only
#define PB_LF_CHUNK 32
#endif
constexpr int kLfChunk = PB_LF_CHUNK;
// the packed block maps (DevParams::cm16): entries per log (the bench: 64 x
// ~171 old blocks) and the offsets record
constexpr int kCm16 = 12288;
constexpr int kCm16Off = kWave + 2;

// The lanes whose 6-bit key equals this lane's, among the active ones (a
// match-any on the tree lane of a log record: 6 ballots).
__device__ __forceinline__ uint64_t same_lane_mask(uint32_t key, bool active) {
  uint64_t m = __ballot(active);
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const bool bit = ((key >> b) & 1u) != 0u;
    const uint64_t bb = __ballot(bit);
    m &= bit ? bb : ~bb;
  }
  return m;
}

template <class Env>
__global__ __launch_bounds__(256) void k_update(DevParams p) {
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  __shared__ uint32_t rng_lds[kTreesPerBlock][4 * kRngPage];
  Tree<Env> T(p, sm, tree);
  T.warm_rng(rng_lds[threadIdx.x >> 6]);
  const int lane = T.lane;
  if (T.err == 0 && !T.root_abs) {   // mcts.py:161-162
    const uint64_t obs = uni64(p.in_obs[tree]);
    if (T.root_t == 0) {
      // _initial_update (mcts.py:175-227): root -> None -> obs node (visits 0)
      uint32_t s0, s1;
      if (!T.sample_agent_initial(obs, &s0, &s1)) T.err = POMCP_E_INVALID;   // probe
      int n = 0;
      while (T.err == 0 && n < p.n_target) {
        if (n >= T.obel_room()) {
          T.err = POMCP_E_ARENA;
          break;
        }
        T.sample_agent_initial(obs, &s0, &s1);
        // type-based: the other agent's policy of the particle,
        // OtherAgentMixturePolicy.sample_initial_state (potmmcp.py:83-87)
        uint32_t pid = 0u;
        if (p.tm && !p.tmt->no_mixture_draw)
          pid = uniform_int(uniu(philox_word(T.seed, T.tkey, S_MIXTURE, T.c_mix++)),
                            (uint32_t)p.tmt->n_other);
        if (lane == 0) *T.obel(n) = make_uint4(1u, s0, s1, pid);
        ++n;
      }
      if (T.err == 0) {
        T.root_code = 0;   // potmmcp.py:44-56: the meta-policy's expected prior
        T.root_id = kRootId;
        T.root_blk = -1;
        T.root_visits = 0;
        T.root_t = 1;
        T.root_abs = 0;
        T.bsel ^= 1;
        T.bsize = n;
        ++T.n_nodes;
      }
    } else {
      // _update (mcts.py:229-263)
      const int action = uni(p.in_actions[tree]);
      // the child k_reroot_child found or created; the tree has been compacted
      // to its subtree since (k_compact: its block is block 0)
      const int4 wi = p.want_info[tree];
      if (uni(wi.w) == 0) {
        T.err = POMCP_E_NOT_FOUND;
      } else {
        ChildRef c;
        c.id = uniu(p.want[tree]) & kIdMask;
        c.blk = uni(wi.x) >= 0 ? 0 : -1;
        c.absorbing = uni(wi.y);
        c.code = uni(wi.z);
        {
          // the child's belief: its particles from the log in insertion order,
          // already gathered into the belief being built by k_compact_log
          int n = uni(p.cnt[tree]);
          // ObsNode.visits of the new root = its particle records (one per
          // arrival, mcts.py:358-371); the slot's count may be stale
          // (pomcp_device.h: cut-off arrivals, children with a block)
          const int visits = n;
          if (n > T.obel_room()) T.err = POMCP_E_ARENA;
          // _reinvigorate (mcts.py:651-700) -> BeliefRejectionSampler (belief.py:145-194)
          const int need = p.n_target - n;
          if (T.err == 0 && !c.absorbing && need > 0) {
            if (n + 2 * need > T.obel_room()) {
              T.err = POMCP_E_ARENA;
            } else {
              const double limit = p.limit_factor * (double)need;
              int got = 0, tries = 0, nrej = 0;
              // 64 tries per pass, one per lane: try i draws word (counter + i) of
              // the belief, the other agent's action and the model stream (one
              // each, independent of the outcomes), so the serial loop's tries
              // are computed in parallel; the ones it would run are the prefix
              // up to the try that completes `need` acceptances (or `limit`),
              // accepted / rejected particles keep their order (ballot ranks)
              const int oth = p.other;
              uint32_t& c_oth = oth == 0 ? T.c_act0 : T.c_act1;
              const uint32_t s_oth = S_ACT_BASE + (uint32_t)oth;
              const uint64_t lt = (1ull << lane) - 1ull;
              while (got < need && (double)tries < limit) {
                const bool valid = (double)(tries + lane) < limit;
                const uint32_t wb = philox_word(T.seed, T.tkey, S_BELIEF, T.c_belief + (uint32_t)lane);
                const uint32_t wa = philox_word(T.seed, T.tkey, s_oth, c_oth + (uint32_t)lane);
                const uint32_t wm = Env::kStepDraws
                                        ? philox_word(T.seed, T.tkey, S_MODEL, T.c_model + (uint32_t)lane)
                                        : 0u;
                const uint4 hp = *T.rbel(uniform_int(wb, (uint32_t)T.bsize));
                // the other agent's action: uniform, or (type-based) by the
                // particle's policy (OtherAgentMixturePolicy.sample_action)
                const uint32_t ao = p.tm && !p.tmt->other_uniform
                                        ? (uint32_t)tm_choice(p.tmt->oth_cum[hp.w], p.tmt->oth_tot[hp.w],
                                                              p.A, wa)
                                        : uniform_int(wa, (uint32_t)p.A);
                uint32_t n0, n1;
                double r;
                int done;
                Env::step(sm, p.ego, hp.y, hp.z, (uint32_t)action, ao,
                          Env::kStepDraws ? uniform_int(wm, 2u) : 0u, &n0, &n1, &r, &done);
                const bool acc = valid && Env::obs_key(sm, p.ego, n0, n1) == obs;
                const uint64_t am = __ballot(acc);
                const int pa = __popcll(am & lt);
                const bool run = valid && got + pa < need;   // the loop head's test before this try
                const uint64_t rm = __ballot(run);
                const uint64_t jm = __ballot(run && !acc);
                const uint4 rec = make_uint4(hp.x + 1u, n0, n1, hp.w);
                if (run && acc) *T.obel(n + got + pa) = rec;
                const int rr = nrej + __popcll(jm & lt);
                if (run && !acc && rr < need) *T.obel(n + need + rr) = rec;
                const int ran = __popcll(rm);
                got += __popcll(am & rm);
                nrej = min(need, nrej + __popcll(jm));
                tries += ran;
                T.c_belief += (uint32_t)ran;
                c_oth += (uint32_t)ran;
                if (Env::kStepDraws) T.c_model += (uint32_t)ran;
              }
              // the LDS pages of the streams advanced here are stale
              T.r_belief.refill(T.seed, T.tkey, S_BELIEF, T.c_belief / kRngPage);
              T.r_model.refill(T.seed, T.tkey, S_MODEL, T.c_model / kRngPage);
              if (oth == 0) T.r_act0.refill(T.seed, T.tkey, S_ACT_BASE, T.c_act0 / kRngPage);
              else T.r_act1.refill(T.seed, T.tkey, S_ACT_BASE + 1, T.c_act1 / kRngPage);
              __builtin_amdgcn_s_waitcnt(0);
              __threadfence_block();
              int fill = need - got;   // rejected samples fill up (belief.py:186-192)
              if (fill > nrej) fill = nrej;
              for (int q0 = 0; q0 < fill; q0 += kWave) {   // disjoint ranges: got < need
                const int q2 = q0 + lane;
                if (q2 < fill) {   // written by other lanes: read past the L1
                  const uint64_t* src = reinterpret_cast<const uint64_t*>(T.obel(n + need + q2));
                  uint64_t* dst = reinterpret_cast<uint64_t*>(T.obel(n + got + q2));
                  dst[0] = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                  dst[1] = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
              }
              n += got + fill;
            }
          }
          if (T.err == 0) {
            T.root_id = c.id;
            T.root_blk = c.blk;
            T.root_visits = visits;
            T.root_t += 1;
            T.root_abs = c.absorbing;
            T.root_code = c.code;
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

// ------------------------------------------------------- subtree compaction
// MCTS._update drops the old root (mcts.py:261-263: `obs_node.parent = None`,
// the rest of the tree is garbage-collected).  Here the arena is compacted
// after every re-root so that it only ever holds the new root's subtree: a
// per-step bound on blocks, overflow entries, particle records and node ids
// (wall-clock searches of the reference's 0.1-20 s budgets, exp_utils.py:27).
// Relabelling only: block order, node ids and overflow slots carry no meaning
// to the search (a node's particles keep their insertion order), so results
// are unchanged -- every golden episode runs through it.
//
// Blocks are allocated when a leaf is expanded, after its parent, so a child's
// block index is always larger than its parent's; the new numbering keeps that
// order (the alive blocks in ascending old order), which lets one ascending pass
// decide reachability and move blocks in place.

// Ordering of a workgroup's own global stores before its later (L1-bypassing,
// ld_agent) loads: every tree (and every search wave's log) is owned by ONE
// workgroup, so workgroup scope suffices.  (__threadfence() is agent scope: on
// gfx950 its release writes back the XCD's whole L2 (buffer_wbl2) -- it was
// 49% of k_compact_log, tools/clog_timing.py.)  The next kernel sees
// everything: the end of a kernel releases at agent scope.
__device__ __forceinline__ void wg_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

__device__ __forceinline__ int32_t ld_agent(const int32_t* p) {   // bypass the (stale) L1
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave per tree: reachability from the new root (the child k_reroot_child
// found), block move, overflow map rebuild.  Runs before k_update (which takes
// its new root from the compacted tree) for trees re-rooted without error.
__global__ __launch_bounds__(256) void k_compact(DevParams p) {
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  const int lane = lane_id();
  TreeHdr h = p.hdr[tree];
  const int4 wi = p.want_info[tree];
  const bool on = uni(h.error) == 0 && uni(wi.w) != 0;
  const int nb = uni(h.n_blocks);
  // read by k_compact_log: 0 = not re-rooted, else 1 + the blocks before the
  // compaction (the entries of cmap it stages in LDS); the streaming scan's
  // per-tree record (DevParams::scan_info)
  if (lane == 0) {
    p.cnt[tree] = on ? 1 + nb : 0;
    if (p.scan_info != nullptr) {
      const uint32_t nsel = (uint32_t)(h.belief_sel ^ 1);
      const uint32_t room = (uint32_t)(p.Nr - (int64_t)h.belief_size);   // (< 2^31: pomcp_create)
      p.scan_info[tree] = make_uint4(p.want[tree], on ? 1u + (uint32_t)nb : 0u, (nsel << 31) | room,
                                     (uint32_t)h.root_t + 1u);
    }
  }
  if (!on) return;
  const int A = p.A;
  const int R = uni(wi.x);   // the new root's block (-1: a leaf)
  Line* const an = p.an + tree_base_lines(tree, p.Nb, p.lines);
  const int64_t bstride = blk_stride_lines(p.lines);
  int32_t* const cmap = p.cmap + (int64_t)tree * p.Nb;
  int32_t* const cpar = p.cpar + (int64_t)tree * p.Nb;
  OvfSlot* const ovf = p.ovf + (int64_t)tree * p.H;
  int32_t* const onew = p.ovf_new + (int64_t)tree * p.H;
  OvfSlot* const otmp = p.ovf_tmp + (int64_t)tree * p.H;
  const uint32_t epoch = (uint32_t)uni(h.epoch);
  // 1. parent of every block: the inline child slots of each block, then the
  //    live overflow entries
  for (int b = lane; b < nb; b += kWave) cpar[b] = -1;
  wg_fence();
  for (int b = lane; b < nb; b += kWave) {
    const uint4* blk = reinterpret_cast<const uint4*>(an + (int64_t)b * bstride);
    for (int a = 0; a < A; ++a) {
#pragma unroll
      for (int k = 0; k < kSlots; ++k) {
        const uint4 sl = blk[part_slot(a, k)];
        if ((sl.y & (uint32_t)(kValidBit >> 32)) != 0u && (int)sl.z >= 0) cpar[(int)sl.z] = b;
      }
    }
  }
  for (int64_t s = lane; s < p.H; s += kWave) {
    const uint4 w0 = reinterpret_cast<const uint4*>(ovf + s)[0];
    const uint4 w1 = reinterpret_cast<const uint4*>(ovf + s)[1];
    const uint64_t key = (uint64_t)w0.x | ((uint64_t)w0.y << 32);
    if ((uint32_t)(key >> kEpochShift) == epoch && (int)w1.x >= 0) cpar[(int)w1.x] = (int)(w0.z / (uint32_t)A);
  }
  wg_fence();
  // 2. reachability and the new numbering (ascending), alive list into cpar
  for (int b = lane; b < (R < 0 ? nb : R); b += kWave) cmap[b] = -1;
  int m = 0;
  for (int base = R < 0 ? nb : R; base < nb; base += kWave) {
    const int b = base + lane;
    const bool in = b < nb;
    const int par = in ? ld_agent(cpar + b) : -1;
    // parents in earlier chunks are final; parents inside this chunk propagate
    // by shuffles (child > parent, so this converges within the chunk depth)
    bool alive = in && (b == R || (par >= 0 && par < base && ld_agent(cmap + par) >= 0));
    const bool local = in && par >= base;
    for (;;) {
      const int src = local ? par - base : lane;
      const bool pa = __shfl((int)alive, src) != 0;
      const bool nw = alive || (local && pa);
      if (__ballot(nw != alive) == 0ull) break;
      alive = nw;
    }
    const uint64_t mk = __ballot(alive);
    const int idx = m + __popcll(mk & ((1ull << lane) - 1ull));
    if (in) cmap[b] = alive ? idx : -1;
    if (alive) cpar[idx] = b;   // idx <= b: entries of this and later chunks already read
    m += __popcll(mk);
    wg_fence();
  }
  wg_fence();
  // 3. move the alive blocks down (in place, ascending), remapping the child
  //    block of every valid inline slot.  8 blocks per pass: all of a pass's
  //    parts are loaded before any is stored (a destination may be a source
  //    of the same pass, never of a later one).
  constexpr int kMoveBlocks = 8;
  const int parts = blk_parts(p.lines);   // <= 56
  for (int i0 = 0; i0 < m; i0 += kMoveBlocks) {
    constexpr int kPer = (kMoveBlocks * 56 + kWave - 1) / kWave;
    uint4 v[kPer];
    int dst[kPer], prt[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int e = lane + q * kWave;
      const int j = e / parts, pp = e % parts;
      dst[q] = -1;
      prt[q] = pp;
      v[q] = make_uint4(0, 0, 0, 0);
      if (j < kMoveBlocks && e < kMoveBlocks * parts && i0 + j < m) {
        const int src = ld_agent(cpar + i0 + j);
        dst[q] = i0 + j;
        v[q] = reinterpret_cast<const uint4*>(an + (int64_t)src * bstride)[pp];
      }
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int pp = prt[q];
      const bool slot = pp >= kLine && pp < kLine * (A + 1) && (pp % kLine) >= 1 && (pp % kLine) <= kSlots;
      const bool vs = dst[q] >= 0 && slot && (v[q].y & (uint32_t)(kValidBit >> 32)) != 0u;
      if (vs && (int)v[q].z >= 0) v[q].z = (uint32_t)ld_agent(cmap + (int)v[q].z);
      if (vs) v[q].w = 0u;   // visits: recounted from the log by k_compact_log
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < kPer; ++q)
      if (dst[q] >= 0) reinterpret_cast<uint4*>(an + (int64_t)dst[q] * bstride)[prt[q]] = v[q];
    wg_fence();
  }
  // 4. overflow map: live entries of alive action nodes are copied out (with the
  //    new action node and child block), the generation is bumped, and they are
  //    re-inserted in slot order; ovf_new maps an old slot to its new node id
  int nlive = 0;
  for (int64_t s0 = 0; s0 < p.H; s0 += kWave) {
    const int64_t s = s0 + lane;
    uint4 w0 = make_uint4(0, 0, 0, 0), w1 = w0;
    bool keep = false;
    if (s < p.H) {
      w0 = reinterpret_cast<const uint4*>(ovf + s)[0];
      w1 = reinterpret_cast<const uint4*>(ovf + s)[1];
      const uint64_t key = (uint64_t)w0.x | ((uint64_t)w0.y << 32);
      if ((uint32_t)(key >> kEpochShift) == epoch) {
        const int pb = ld_agent(cmap + (int)(w0.z / (uint32_t)A));
        if (pb >= 0) {
          keep = true;
          w0.z = (uint32_t)pb * (uint32_t)A + w0.z % (uint32_t)A;
          if ((int)w1.x >= 0) w1.x = (uint32_t)ld_agent(cmap + (int)w1.x);
          w1.y = 0u;            // visits: recounted by k_compact_log
          w1.z = (uint32_t)s;   // the old slot (pad word)
        }
      }
      onew[s] = -1;
    }
    const uint64_t mk = __ballot(keep);
    if (keep) {
      const int at = nlive + __popcll(mk & ((1ull << lane) - 1ull));
      reinterpret_cast<uint4*>(otmp + at)[0] = w0;
      reinterpret_cast<uint4*>(otmp + at)[1] = w1;
    }
    nlive += __popcll(mk);
  }
  uint32_t ne = (epoch + 1u) & kEpochMask;
  if (ne == 0u) {   // generation counter wrapped: clear the map
    clear_ovf(p, tree, lane);
    ne = 1u;
  }
  wg_fence();
  for (int i = 0; i < nlive; ++i) {
    const uint4 w0 = reinterpret_cast<const uint4*>(otmp + i)[0];
    const uint4 w1 = reinterpret_cast<const uint4*>(otmp + i)[1];
    const uint64_t okey = ((uint64_t)w0.x | ((uint64_t)w0.y << 32)) & kObsMask;
    uint32_t b = ovf_hash(w0.z, okey) & p.bucket_mask;
    for (uint32_t probe = 0; probe <= p.bucket_mask; ++probe) {
      OvfSlot* e = ovf + (int64_t)b * kBucket + (lane & (kBucket - 1));
      uint32_t ky = 0u;   // the key's high word (generation); this loop's inserts are not in L1
      if (lane < kBucket) ky = ld_agent_u32(reinterpret_cast<const uint32_t*>(e) + 1);
      const uint64_t em = __ballot(lane < kBucket && (ky >> (kEpochShift - 32)) != ne);
      if (em) {
        const int L = __ffsll((long long)em) - 1;
        if (lane == L) {
          const uint64_t key = okey | ((uint64_t)ne << kEpochShift);
          reinterpret_cast<uint4*>(e)[0] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), w0.z, w0.w);
          reinterpret_cast<uint4*>(e)[1] = make_uint4(w1.x, w1.y, 0u, 0u);
          onew[w1.z] = (int32_t)(p.ovf_base + b * kBucket + (uint32_t)L);
        }
        wg_fence();
        break;
      }
      b = (b + 1) & p.bucket_mask;
    }
  }
  if (lane == 0) {
    h.n_blocks = m;
    h.root_blk = R >= 0 ? 0 : -1;
    h.epoch = (int32_t)ne;
    p.hdr[tree] = h;
  }
}

__device__ __forceinline__ uint64_t ld_agent_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One WORKGROUP (kLogWaves waves) per SEARCH wave: filter that
// wave's shared particle log to the records of obs nodes that survived
// k_compact (insertion order kept) and relabel them; every tree's record count
// is recounted.  The same scan extracts the new root's records (the child
// k_reroot_child found, by its old id) into the tree's other belief buffer as
// {root_t + 1, v0, v1, aux}, in insertion order (mcts.py:248-252): a record's
// place is its tree's count before the pass + the same tree's records in the
// earlier sub-passes, then earlier waves of its sub-pass + its rank in its wave
// (same_lane_mask); k_update takes the count as the new root's belief size and
// visits.  (A separate extraction scan before k_update read the whole log once
// more: 31 ms of the PursuitEvasion step's 130 ms update.)  A deferred record (pomcp_device.h: an arrival at a child
// beyond the depth / step limits, never looked up by k_search) whose action
// node survived gets its child here: the child's observation key and
// absorbing flag follow from the record's state (Env::obs_key, Env::done_of);
// it is found among the action node's inline slots or inserted there
// (compare-and-swap: the threads insert concurrently), else in the overflow
// map (a chunk's such records one at a time, by wave 0), and its absorbing
// flag is that of its LAST arrival (mcts.py:370; records in log order).  Which
// slot a child takes is a label (ActionNode.children is only ever looked up by
// observation in the reference), so results are unchanged.  A pass reads
// kLogRecs x 64 kLogWaves consecutive records; all of them are loaded before
// any is stored, and a kept record goes to a place at or before its own, so
// the log is filtered in place.  Deferred records are kept and stored like
// the others but materialised in bulk: each pass appends them (log order) to
// a workgroup queue in LDS, and when the queue is full (and at the end) its
// records are materialised T at a time -- full chunks instead of a barrier-
// heavy block per sub-pass with ~1 in 8 threads active -- and only their id
// words are rewritten in place (the place stays reserved: nothing reads
// below the pass's read frontier).
// Section timing of k_compact_log (diagnostics builds, -DPB_CLOG_TIMING): thread
// 0's s_memtime deltas per section and per-workgroup counters into
// p.timing[search wave][16] (tools/clog_timing.py).
#ifdef PB_CLOG_TIMING
#define CL_MARK(s)                                                  \
  do {                                                              \
    if (t == 0) {                                                   \
      __builtin_amdgcn_s_waitcnt(0);                                \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();           \
      clt[s] += now_ - cl_last;                                     \
      cl_last = now_;                                               \
    }                                                               \
  } while (0)
#define CL_CNT(s, f)                                                \
  do {                                                              \
    const uint64_t m_ = __ballot(f);                                \
    if (lane == 0 && m_) atomicAdd(&clc[s], (uint32_t)__popcll(m_)); \
  } while (0)
#else
#define CL_MARK(s) \
  do {             \
  } while (0)
#define CL_CNT(s, f) \
  do {               \
  } while (0)
#endif
// kMatOnly (the streaming scan's second kernel, k_log_filter below): the log
// has been filtered and relabelled already; this pass only counts every
// tree's records and materialises the deferred children of the re-rooted
// trees in log order (records stay where they are: a queued place is the
// record's own), the extracted counts come from the look-back records.
#ifdef PB_LOG_WPE   // A/B builds only: waves per SIMD the register allocation must allow
#define PB_LOG_ATTR __attribute__((amdgpu_waves_per_eu(PB_LOG_WPE)))
#else
#define PB_LOG_ATTR
#endif
template <class Env, bool kMatOnly = false>
__global__ __launch_bounds__(64 * (kMatOnly ? kMatWaves : kLogWaves)) PB_LOG_ATTR void k_compact_log(DevParams p) {
  constexpr int LW = kMatOnly ? kMatWaves : kLogWaves;   // waves of the workgroup
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  constexpr int T = 64 * LW;
  const int sw = blockIdx.x;
  const int w = (int)(threadIdx.x >> 6);
  const int lane = lane_id();
  const int t = (int)threadIdx.x;
  __shared__ int32_t kept[kWave];
  __shared__ int32_t act[kWave];
  __shared__ uint32_t want[kWave];  // the new root's log id per tree (k_reroot_child) ...
  __shared__ int32_t xcnt[kWave];   // ... its records extracted so far
  __shared__ uint32_t tval[kWave];
  __shared__ int64_t xdst[kWave];   // the tree's belief region ...
  __shared__ int32_t xsel[kWave];   // ... the end the new belief grows from ...
  __shared__ int32_t xroom[kWave];  // ... and its room (the current belief holds the rest)
  __shared__ uint8_t xw[kLogRecs][LW][kWave];   // this pass's extracted records per
                                                      // sub-pass, wave and tree (<= 64)
  __shared__ int32_t made[kWave];   // children materialised per tree
  __shared__ int32_t bad[kWave];    // overflow map full
  __shared__ int32_t wsum[LW];
  __shared__ int32_t ovq[T];        // threads whose child goes to the overflow map, in order
  __shared__ int32_t ovres[T];      // per thread: its overflow entry (-1: map full)
  __shared__ uint32_t ovd[5][T];    // per thread: tree lane, action node, key lo / hi, done
  // a chunk's children (flag word addresses), hashed: the last thread naming
  // each and its number of arrivals
  constexpr int kH = 2 * T;
  constexpr int kHBits = kH == 256 ? 8 : kH == 512 ? 9 : kH == 1024 ? 10 : kH == 2048 ? 11 : -1;
  static_assert(kHBits > 0, "the hash takes log2(kH) bits (mat_block)");
  __shared__ unsigned long long hk[kH];
  __shared__ int32_t hl[kH], hc[kH];
  // between flushes the same LDS holds a pass's visits table: 2 kH keys (the
  // relabelled record id: node id | tree lane, unique in the workgroup) in hk,
  // their arrival counts in hl then hc -- one visits atomic per node and pass
  constexpr int kV = 2 * kH;
  constexpr int kVBits = kHBits + 1;
  static_assert(kLogRecs * T <= kV, "a pass's records fit the visits table");
  uint32_t* const vkey = reinterpret_cast<uint32_t*>(hk);
  auto vcnt = [&](int h) -> int32_t* { return h < kH ? &hl[h] : &hc[h - kH]; };
  auto vclear = [&]() {
#pragma unroll
    for (int q = 0; q < kV / T; ++q) {
      vkey[q * T + t] = 0xFFFFFFFFu;   // (ids < kIdMask: pomcp_create)
      *vcnt(q * T + t) = 0;
    }
  };
  // deferred-record queue: a pass's records always fit.  Only their places: the
  // record is stored there with its relabelled action node (cut_base + new
  // action node | lane) and the flush reads it back (state -> key and done)
  constexpr int kQ = kLogRecs * T;
  __shared__ uint32_t q_at[kQ];
  // cmap (k_compact: old block -> new block, -1 dropped) of the wave's 64 trees,
  // staged in LDS when their old blocks fit (the bench: ~64 x 171): the
  // classification of a record then issues no global load, so its wait never
  // includes the next pass's prefetched records (vmcnt completes in order)
  constexpr int kCmapLds = kMatOnly ? 8 : 16384;   // (kMatOnly classifies nothing)
  __shared__ int16_t cml[kCmapLds];
  __shared__ int32_t cmo[kWave + 1];   // per tree lane: its first entry in cml
  __shared__ int32_t cml_ok;
#ifdef PB_CLOG_TIMING
  uint64_t clt[6] = {0, 0, 0, 0, 0, 0};
  uint64_t cl_last = __builtin_amdgcn_s_memtime();
  __shared__ uint32_t clc[8];
  if (t < 8) clc[t] = 0u;
#endif
  if (w == 0) {
    const int mytree = sw * kWave + lane;
    kept[lane] = 0;
    made[lane] = 0;
    bad[lane] = 0;
    const int c = mytree < p.B ? p.cnt[mytree] : 0;   // k_compact: 1 + old blocks, 0 = off
    act[lane] = c > 0 ? 1 : 0;
    const int nbo = c > 0 ? c - 1 : 0;
    int inc = nbo;   // inclusive scan over the wave's trees
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int y = __shfl_up(inc, d);
      if (lane >= d) inc += y;
    }
    cmo[lane] = inc - nbo;
    if (lane == kWave - 1) cmo[kWave] = inc;
    const bool fit = __ballot(nbo > 32767) == 0ull && __shfl(inc, kWave - 1) <= kCmapLds;
    if (lane == 0) cml_ok = fit ? 1 : 0;
    const bool valid = mytree < p.B;
    const TreeHdr h = p.hdr[valid ? mytree : 0];
    want[lane] = valid ? p.want[mytree] : 0xFFFFFFFFu;
    xcnt[lane] = 0;
    tval[lane] = (uint32_t)h.root_t + 1u;
    xdst[lane] = (int64_t)mytree * p.Nr;
    xsel[lane] = h.belief_sel ^ 1;
    xroom[lane] = (int32_t)(p.Nr - (int64_t)h.belief_size);
  }
  // the streaming scan: the kept records and each tree's extracted count from
  // the last segment's look-back record
  uint32_t n_mat = 0u;
  if constexpr (kMatOnly) {
    const uint32_t n0 = p.wlog[sw];
    if (n0 > 0u) {
      const int nchunk = (p.lf_nseg + kLfChunk - 1) / kLfChunk;
      const LfDesc& d = p.lf_desc[(int64_t)sw * nchunk + (int64_t)((n0 - 1u) / kLfSeg / kLfChunk)];
      n_mat = d.kept_inc;
      if (w == 0) xcnt[lane] = (int32_t)d.ex_inc[lane];
    }
  }
  vclear();
  __syncthreads();
#ifdef PB_NO_CMAP_LDS   // A/B builds only: classify from the global cmap
  const bool cml_on = false;
#else
  const bool cml_on = !kMatOnly && cml_ok != 0;
#endif
  if (cml_on) {   // entry e belongs to the tree lane L with cmo[L] <= e < cmo[L + 1]
    for (int e = t; e < cmo[kWave]; e += T) {
      int lo = 0, hi = kWave - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (cmo[mid] <= e) lo = mid;
        else hi = mid - 1;
      }
      cml[e] = (int16_t)p.cmap[(int64_t)(sw * kWave + lo) * p.Nb + (e - cmo[lo])];
    }
  }
  __syncthreads();
  // the new block of old block b of tree lane l (tree = sw * 64 + l)
  auto cm = [&](uint32_t l, int tr, uint32_t b) -> int {
    return cml_on ? (int)cml[cmo[l] + (int)b] : p.cmap[(int64_t)tr * p.Nb + (int)b];
  };
  // a thread's place among the workgroup's threads with f set (thread order);
  // every thread calls it
  auto wg_rank = [&](bool f, int* total) -> int {
    const uint64_t m = __ballot(f);
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int v = 0; v < LW; ++v) {
      pre += v < w ? wsum[v] : 0;
      tot += wsum[v];
    }
    __syncthreads();
    *total = tot;
    return pre + __popcll(m & ((1ull << lane) - 1ull));
  };
  const WaveLog wl(p.plog, p.Np, sw, p.tm);
  const uint32_t n = kMatOnly ? n_mat : p.wlog[sw];
  const uint32_t A = (uint32_t)p.A;
  // x / A by a multiply: amag = ceil(2^32 / A) is exact for x < 2^32 / A
  // (x < 2^26: node ids, pomcp_create; A <= 5)
  const uint64_t amag = (0x100000000ull + A - 1u) / A;
  auto divA = [&](uint32_t x) -> uint32_t { return (uint32_t)(((uint64_t)x * amag) >> 32); };
  const int64_t bstride = blk_stride_lines(p.lines);
  constexpr int R = kLogRecs;
  const uint64_t below = (1ull << lane) - 1ull;
  __shared__ int32_t ksum[R][LW];   // kept records per sub-pass and wave
  __shared__ int32_t msum[R][LW];   // deferred records to materialise, likewise
  // A deferred record's child, found or inserted (inline slots by CAS, else the
  // overflow map in log order), its absorbing flag set by the last arrival of
  // the chunk and its visits raised by the chunk's arrivals (one atomic per
  // child); every thread calls it (workgroup barriers inside)
  auto mat_block = [&](bool mat, int tree, uint32_t l, uint32_t nani, uint64_t okey, int done,
                       int32_t& nid, bool& keep) {
    hk[t] = 0ull;
    hk[t + T] = 0ull;
    hl[t] = -1;
    hl[t + T] = -1;
    hc[t] = 0;
    hc[t + T] = 0;
    if (__syncthreads_or(mat ? 1 : 0)) {
      int32_t* vis = nullptr;
      uint32_t* flagw = nullptr;   // the word holding the child's absorbing flag ...
      uint32_t fbit = 0u;          // ... and its bit
      int curf = 2;                // the flag as this thread last saw it (2: not known)
      bool need_ovf = false;
      bool ovf_look = false;   // (diagnostics counter: looked up in the overflow map)
      (void)ovf_look;
      if (mat) {   // inline slots, filled in order; concurrent inserts by CAS on the key
        const uint32_t nq = divA(nani);
        uint4* const sl0 = reinterpret_cast<uint4*>(p.an + tree_base_lines(tree, p.Nb, p.lines) +
                                                    (int64_t)nq * bstride) +
                           part_slot((int)(nani - nq * A), 0);
        const uint64_t nk = okey | kValidBit | ((uint64_t)done << 63);
        uint64_t kk[kSlots];
#ifndef PB_MAT_EAGER_SLOTS
        // slots 0-1 first, the others only when both hold other observations
        // (valid slots are a prefix: an insert takes the first slot it saw
        // empty); an unread slot is taken as empty and the CAS below checks it.
        // Round 6 A/B: update 149 -> 137 ms at 65,536 PursuitEvasion roots (the
        // pass is bound by its slot-line requests; 1 / 1-1 / 1-2 / 2-1 tiers
        // within 1 ms, profiles/r6q_lazy_slots_ab.txt)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          kk[q] = q < p.islots ? ld_agent_u64(reinterpret_cast<const uint64_t*>(sl0 + q)) : kValidBit;
        const bool more = ((kk[0] & kk[1]) & kValidBit) != 0ull && (kk[0] & kObsMask) != okey &&
                          (kk[1] & kObsMask) != okey;
#pragma unroll
        for (int q = 2; q < kSlots; ++q)
          kk[q] = q < p.islots ? (more ? ld_agent_u64(reinterpret_cast<const uint64_t*>(sl0 + q)) : 0ull)
                               : kValidBit;
#else   // A/B builds only: every slot read
#pragma unroll
        for (int q = 0; q < kSlots; ++q)
          kk[q] = q < p.islots ? ld_agent_u64(reinterpret_cast<const uint64_t*>(sl0 + q)) : kValidBit;
#endif
        int ks = -1;
#pragma unroll
        for (int q = kSlots - 1; q >= 0; --q)
          if ((kk[q] & kValidBit) != 0ull && (kk[q] & kObsMask) == okey) {
            ks = q;
            curf = (int)(kk[q] >> 63);
          }
        for (int q = 0; ks < 0 && q < p.islots; ++q) {
          uint64_t exp = 0ull;
#pragma unroll
          for (int e = 0; e < kSlots; ++e) exp = e == q ? kk[e] : exp;   // (selects: registers)
          if ((exp & kValidBit) != 0ull) continue;   // taken by another observation
          uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(sl0 + q),
                                   (unsigned long long)exp, (unsigned long long)nk);
#ifndef PB_MAT_EAGER_SLOTS
          if (old != exp && (old & kValidBit) == 0ull) {   // an unread empty slot's word was not 0
            exp = old;
            old = atomicCAS(reinterpret_cast<unsigned long long*>(sl0 + q), (unsigned long long)exp,
                            (unsigned long long)nk);
          }
#endif
          if (old == exp) {   // inserted: a leaf child (no block), visits counted below
            __hip_atomic_store(reinterpret_cast<int32_t*>(sl0 + q) + 2, -1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            atomicAdd(&made[l], 1);
            ks = q;
            curf = done;
          } else if ((old & kValidBit) != 0ull && (old & kObsMask) == okey) {
            ks = q;   // another thread of this pass inserted it
            curf = (int)(old >> 63);
          }
        }
        if (ks >= 0) {
          nid = (int32_t)(nani * kSlots + (uint32_t)ks + 1u);
          vis = reinterpret_cast<int32_t*>(sl0 + ks) + 3;
          flagw = reinterpret_cast<uint32_t*>(sl0 + ks) + 1;
          fbit = 1u << 31;
        } else {
          ovf_look = true;
          // an overflow child made by an earlier pass (or by the search): every
          // thread looks its own up (read-only probe in insertion order: a bucket
          // holding the key, else the first bucket with a free entry ends it)
          OvfSlot* const ovf = p.ovf + (int64_t)tree * p.H;
          const uint32_t epoch = (uint32_t)p.hdr[tree].epoch;   // k_compact's generation
          const uint64_t key = okey | ((uint64_t)epoch << kEpochShift);
          uint32_t b = ovf_hash(nani, okey) & p.bucket_mask;
          int32_t jid = -1;
          for (uint32_t probe = 0; probe <= p.bucket_mask; ++probe) {
            bool free = false;
#pragma unroll 4
            for (int e = 0; e < kBucket; ++e) {
              OvfSlot* const ep = ovf + (int64_t)b * kBucket + e;
              const uint64_t sk = ld_agent_u64(&ep->key);
              const uint32_t san = ld_agent_u32(&ep->an);
              const bool live = (uint32_t)(sk >> kEpochShift) == epoch;
              if (jid < 0 && live && sk == key && san == nani) jid = (int32_t)(b * kBucket + (uint32_t)e);
              free |= !live;
            }
            if (jid >= 0 || free) break;
            b = (b + 1) & p.bucket_mask;
          }
          if (jid >= 0) {
            nid = (int32_t)(p.ovf_base + (uint32_t)jid);
            vis = &ovf[jid].visits;
            flagw = &ovf[jid].flags;
            fbit = 1u;
          } else {
            need_ovf = true;   // a new child: inserted below, in log order
          }
        }
      }
      // overflow map: the pass's records of NEW overflow children (and of the
      // ones inserted earlier in the same pass), in thread (= log) order, one at
      // a time, by wave 0 (its 16 lanes probe a bucket)
      CL_CNT(5, ovf_look);
      CL_MARK(1);
      CL_CNT(2, need_ovf);
      int novf = 0;
      const int opos = wg_rank(need_ovf, &novf);
      if (need_ovf) {
        ovq[opos] = t;
        ovd[0][t] = l;
        ovd[1][t] = nani;
        ovd[2][t] = (uint32_t)okey;
        ovd[3][t] = (uint32_t)(okey >> 32);
        ovd[4][t] = (uint32_t)done;
      }
      __syncthreads();
      if (novf > 0) {
        if (w == 0) {
          for (int x = 0; x < novf; ++x) {
            const int jt = ovq[x];
            const int jl = (int)ovd[0][jt];
            const int jtree = sw * kWave + jl;
            const uint32_t jani = ovd[1][jt];
            const uint64_t jkey = ((uint64_t)ovd[3][jt] << 32) | ovd[2][jt];
            const uint32_t jdone = ovd[4][jt];
            OvfSlot* const ovf = p.ovf + (int64_t)jtree * p.H;
            const uint32_t epoch = (uint32_t)p.hdr[jtree].epoch;   // k_compact's generation
            const uint64_t key = jkey | ((uint64_t)epoch << kEpochShift);
            uint32_t b = ovf_hash(jani, jkey) & p.bucket_mask;
            int32_t jid = -1;
            for (uint32_t probe = 0; probe <= p.bucket_mask && jid < 0; ++probe) {
              OvfSlot* const e = ovf + (int64_t)b * kBucket + (lane & (kBucket - 1));
              uint64_t sk = 0ull;
              uint32_t san = 0u;
              if (lane < kBucket) {
                sk = ld_agent_u64(&e->key);
                san = ld_agent_u32(&e->an);
              }
              const bool live = lane < kBucket && (uint32_t)(sk >> kEpochShift) == epoch;
              const uint64_t mm = __ballot(live && sk == key && san == jani);
              const uint64_t em = __ballot(lane < kBucket && !live);
              if (mm != 0ull || em != 0ull) {
                const int L = __ffsll((long long)(mm != 0ull ? mm : em)) - 1;
                if (mm == 0ull && lane == L) {   // insert a leaf child
                  reinterpret_cast<uint4*>(e)[0] =
                      make_uint4((uint32_t)key, (uint32_t)(key >> 32), jani, jdone);
                  reinterpret_cast<uint4*>(e)[1] = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
                  atomicAdd(&made[jl], 1);
                }
                wg_fence();
                jid = (int32_t)(b * kBucket + (uint32_t)L);
              }
              b = (b + 1) & p.bucket_mask;
            }
            if (lane == 0) ovres[jt] = jid;
          }
        }
        __syncthreads();
        if (need_ovf) {
          const int32_t jid = ovres[t];
          if (jid >= 0) {
            OvfSlot* const ovf = p.ovf + (int64_t)tree * p.H;
            nid = (int32_t)(p.ovf_base + (uint32_t)jid);
            vis = &ovf[jid].visits;
            flagw = &ovf[jid].flags;
            fbit = 1u;
          } else {   // the overflow map is full
            keep = false;
            bad[l] = 1;
          }
        }
      }
      CL_MARK(2);
      // the absorbing flag of each child = that of its last arrival (thread
      // order = log order): the chunk's children in an LDS hash (open
      // addressing on the flag word's address) holding the highest thread and
      // the arrival count; that thread sets the flag and adds the visits
      const unsigned long long fp = (unsigned long long)reinterpret_cast<uintptr_t>(flagw);
      int h = 0;
      if (flagw != nullptr) {
        uint32_t x = (uint32_t)(fp >> 2) ^ (uint32_t)(fp >> 34);
        x *= 0x9E3779B1u;
        h = (int)(x >> (32 - kHBits)) & (kH - 1);
        for (;;) {
          const unsigned long long old = atomicCAS(&hk[h], 0ull, fp);
          if (old == 0ull || old == fp) break;
          h = (h + 1) & (kH - 1);
        }
        atomicMax(&hl[h], t);
        atomicAdd(&hc[h], 1);
      }
      __syncthreads();
      if (flagw != nullptr && hl[h] == t) {
        // an inline child's flag as the last arrival saw it is current (earlier
        // chunks' atomics landed before its read, and only the last arrival of
        // this chunk writes it): unchanged, no atomic
#ifdef PB_MAT_ALWAYS_FLAG   // A/B builds only
        curf = 2;
#endif
        if (done && curf != 1) atomicOr(flagw, fbit);
        else if (!done && curf != 0) atomicAnd(flagw, ~fbit);
        atomicAdd(vis, hc[h]);
      }
      wg_fence();   // the chunk's inserts, flags and visits land before the next chunk's
      CL_MARK(3);
      CL_CNT(3, flagw != nullptr);
    }
    __syncthreads();   // (the hash is cleared by the next chunk)
  };
  // materialise the queue's qn records (log order), T per chunk; each record's
  // id word gets its child's id.  Every thread calls it.
  auto flush = [&](int qn) {
    wg_fence();        // the queued records were stored by this workgroup: they land
    __syncthreads();   // before the (L1-bypassing) reads below
    // each chunk's records are read during the previous chunk (their wait is
    // then the previous chunk's slot loads' own)
    uint32_t n_rid = 0u, n_v0 = 0u, n_v1 = 0u;
    if (t < qn) {
      const uint32_t at0 = q_at[t];
      n_rid = ld_agent_u32(wl.id + at0);
      n_v0 = ld_agent_u32(wl.v0 + at0);
      n_v1 = ld_agent_u32(wl.v1 + at0);
    }
    for (int c = 0; c < qn; c += T) {
      const int e = c + t;
      const bool m = e < qn;
      uint32_t at = 0u, nani = 0u, ll = 0u;
      uint64_t ok = 0ull;
      int dn = 0;
      if (m) {   // the child's observation key and absorbing flag from the record's state
        at = q_at[e];
        const uint32_t rid = n_rid, v0 = n_v0, v1 = n_v1;
        ll = rid >> kIdBits;
        nani = (rid & kIdMask) - p.cut_base;
        ok = Env::obs_key(sm, p.ego, v0, v1);
        dn = Env::done_of(p.ego, v0, v1);
      }
      if (e + T < qn) {
        const uint32_t at1 = q_at[e + T];
        n_rid = ld_agent_u32(wl.id + at1);
        n_v0 = ld_agent_u32(wl.v0 + at1);
        n_v1 = ld_agent_u32(wl.v1 + at1);
      }
      int32_t nid = -1;
      bool keep = true;
      mat_block(m, sw * kWave + (int)ll, ll, nani, ok, dn, nid, keep);
      // the overflow map is full (keep false): the tree has failed (bad[] ->
      // POMCP_E_ARENA) and the record gets an id no node ever has (kIdMask), so
      // it can never be read as a live deferred record
      if (m) wl.id[at] = (keep ? (uint32_t)nid : kIdMask) | (ll << kIdBits);
    }
  };
  int qn = 0;   // queued deferred records (uniform over the workgroup)
  uint32_t out = 0;
  // a pass = kLogRecs sub-passes of T records (sub-pass j: record base + j T +
  // t), all loaded before any is stored, the next pass's loaded while this one
  // runs; a kept record lands at or before its own place (in-place filter)
  LogRec rn[R];
  uint32_t auxn[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t i = (uint32_t)(j * T + t);
    rn[j] = LogRec{0u, 0u, 0u};
    auxn[j] = 0u;
    if (i < n) {
      if constexpr (kMatOnly) {   // (ids only: the flush reads a deferred record's state)
        rn[j].id = wl.id[i];
      } else {
        rn[j] = wl.load(i);
        if (p.tm) auxn[j] = wl.aux[i];
      }
    }
  }
  for (uint32_t base = 0; base < n; base += (uint32_t)(R * T)) {
    LogRec r[R];
    uint32_t aux[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      r[j] = rn[j];
      aux[j] = auxn[j];
      const uint32_t i2 = base + (uint32_t)((R + j) * T + t);
      if (i2 < n) {
        if constexpr (kMatOnly) {
          rn[j].id = wl.id[i2];
        } else {
          rn[j] = wl.load(i2);
          if (p.tm) auxn[j] = wl.aux[i2];
        }
      }
    }
    bool keep[R], mat[R], ex[R];
    uint32_t l[R], nani[R];
    int tree[R];
    int32_t nid[R];
    int32_t* vis[R];   // the node's visits (zeroed by k_compact): + 1 per record
    int xr[R];         // an extracted record's rank among its wave's of the same tree
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t i = base + (uint32_t)(j * T + t);
      keep[j] = false;
      mat[j] = false;
      ex[j] = false;
      l[j] = 0u;
      nani[j] = 0u;
      nid[j] = -1;
      vis[j] = nullptr;
      tree[j] = sw * kWave + (int)((i < n ? r[j].id : 0u) >> kIdBits);
      if (i < n) {
        l[j] = r[j].id >> kIdBits;
        const uint32_t id = r[j].id & kIdMask;
        keep[j] = true;
        if constexpr (kMatOnly) {   // filtered and relabelled by k_log_filter
          if (act[l[j]] && id >= p.cut_base && id < kIdMask) {
            mat[j] = true;
            nani[j] = id - p.cut_base;
          }
        } else {
        ex[j] = want[l[j]] == r[j].id;   // a record of the new root (never kept below)
        if (act[l[j]]) {
          if (id >= p.cut_base) {   // deferred record: its child is materialised below
            const uint32_t ani = id - p.cut_base;
            const uint32_t aq = divA(ani);
            const int nb = cm(l[j], tree[j], aq);
            if (nb >= 0) {
              mat[j] = true;
              nani[j] = (uint32_t)nb * A + (ani - aq * A);   // (key and done: at the flush, dense)
            }
          } else if (id >= p.ovf_base) {
            nid[j] = p.ovf_new[(int64_t)tree[j] * p.H + (id - p.ovf_base)];
            if (nid[j] >= 0) vis[j] = &p.ovf[(int64_t)tree[j] * p.H + ((uint32_t)nid[j] - p.ovf_base)].visits;
          } else if (id >= 1u) {
            const uint32_t ani = (id - 1u) / kSlots, k = (id - 1u) % kSlots;
            const uint32_t aq = divA(ani), ar = ani - aq * A;
            const int nb = cm(l[j], tree[j], aq);
            if (nb >= 0) {
              nid[j] = (int32_t)(((uint32_t)nb * A + ar) * kSlots + k + 1u);
              uint4* const bp = reinterpret_cast<uint4*>(p.an + tree_base_lines(tree[j], p.Nb, p.lines) +
                                                         (int64_t)nb * bstride);
              vis[j] = reinterpret_cast<int32_t*>(bp + part_slot((int)ar, (int)k)) + 3;
            }
          }
          keep[j] = nid[j] >= 0 || mat[j];
        }
        }
      }
      CL_CNT(0, i < n);
      CL_CNT(1, mat[j]);
    }
    CL_MARK(0);
    __syncthreads();   // (the visits table is clear)
    // visits (each record's node counted in the table; the thread that entered
    // the node adds its count below), relabelling (a deferred record keeps its
    // id until its child is materialised), per-tree counts, the pass's places
    int vh[R];   // the table entry this thread adds to its node's visits (-1: none)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t i = base + (uint32_t)(j * T + t);
      vh[j] = -1;
      if (i < n && act[l[j]]) {
        if (vis[j] != nullptr) {
          const uint32_t key = (uint32_t)nid[j] | (l[j] << kIdBits);
          int h = (int)((key * 0x9E3779B1u) >> (32 - kVBits));
          bool first = false;
          for (;;) {   // (a pass holds at most kV records: a free entry remains)
            const uint32_t old = atomicCAS(&vkey[h], 0xFFFFFFFFu, key);
            if (old == 0xFFFFFFFFu) first = true;
            if (old == 0xFFFFFFFFu || old == key) break;
            h = (h + 1) & (kV - 1);
          }
          atomicAdd(vcnt(h), 1);
          vh[j] = first ? h : -1;
        }
        if constexpr (!kMatOnly) {
          if (keep[j] && !mat[j]) r[j].id = (uint32_t)nid[j] | (l[j] << kIdBits);
          if (mat[j]) r[j].id = (p.cut_base + nani[j]) | (l[j] << kIdBits);   // (the flush reads it)
        }
      }
      // (a count only: one LDS atomic per kept record -- a wave's records mostly
      // belong to distinct trees, lane = tree lane, so they seldom collide)
      if (keep[j]) atomicAdd(&kept[l[j]], 1);
      xw[j][w][lane] = 0;
      xr[j] = 0;
      if (__ballot(ex[j]) != 0ull) {
        const uint64_t xs = same_lane_mask(l[j], ex[j]);
        xr[j] = __popcll(xs & below);
        asm volatile("" ::: "memory");   // (the zero lands first: one wave's LDS ops run in order)
        if (ex[j] && (xs >> lane) == 1ull) xw[j][w][l[j]] = (uint8_t)__popcll(xs);   // the tree's last lane
      }
    }
    uint64_t mk[R], mm[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      mk[j] = __ballot(keep[j]);
      mm[j] = __ballot(mat[j]);
      if (lane == 0) {
        ksum[j][w] = __popcll(mk[j]);
        msum[j][w] = __popcll(mm[j]);
      }
    }
    __syncthreads();
    // the new root belief ({root_t + 1, v0, v1, aux}, mcts.py:248-252): a record's
    // place = its tree's count before the pass + the same tree's records in
    // earlier sub-passes, then earlier waves of its sub-pass + its rank in its wave
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (ex[j]) {
        const int lj = (int)l[j];
        int pos = xcnt[lj] + xr[j];
        for (int jj = 0; jj < j; ++jj)
          for (int v = 0; v < LW; ++v) pos += xw[jj][v][lj];
        for (int v = 0; v < w; ++v) pos += xw[j][v][lj];
        if (pos < xroom[lj])   // (beyond: k_update fails the tree, POMCP_E_ARENA)
          p.belief[xdst[lj] + bel_at(xsel[lj], p.Nr, pos)] = make_uint4(tval[lj], r[j].v0, r[j].v1, aux[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (vh[j] >= 0) atomicAdd(vis[j], *vcnt(vh[j]));   // the node's arrivals in this pass
    int xadd = 0;   // wave 0: this pass's extracted records of tree `lane`
    if (w == 0) {
#pragma unroll
      for (int j = 0; j < R; ++j)
#pragma unroll
        for (int v = 0; v < LW; ++v) xadd += xw[j][v][lane];
    }
    int mtot = 0;
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int v = 0; v < LW; ++v) mtot += msum[j][v];
    CL_MARK(4);
    if (qn + mtot > kQ) {   // (uniform) materialise the queue first
      __syncthreads();   // (the visits table's counts are read: mat_block reuses its LDS)
      flush(qn);
      qn = 0;
    }
    int tot = 0, mt = qn;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      int pre = 0, tj = 0, mpre = 0, mj = 0;
#pragma unroll
      for (int v = 0; v < LW; ++v) {
        pre += v < w ? ksum[j][v] : 0;
        tj += ksum[j][v];
        mpre += v < w ? msum[j][v] : 0;
        mj += msum[j][v];
      }
      if (keep[j]) {   // (kMatOnly: every record is kept, so `at` is its own place)
        const uint32_t at = out + (uint32_t)(tot + pre + __popcll(mk[j] & below));
        if constexpr (!kMatOnly) {
          wl.store(at, r[j]);
          if (p.tm) wl.aux[at] = aux[j];
        }
        if (mat[j]) q_at[mt + mpre + __popcll(mm[j] & below)] = at;
      }
      tot += tj;
      mt += mj;
    }
    qn += mtot;
    out += (uint32_t)tot;
    __syncthreads();   // (ksum and xw are rewritten by the next pass)
    if (w == 0) xcnt[lane] += xadd;   // (read again after the next pass's first barrier)
    vclear();
#pragma unroll
    for (int j = 0; j < R; ++j) CL_CNT(4, keep[j]);
    CL_MARK(4);
  }
  __syncthreads();
  if (qn > 0) flush(qn);
#ifdef PB_CLOG_TIMING
  if (t == 0 && p.timing != nullptr) {
    for (int q = 0; q < 5; ++q) p.timing[sw * 16 + q] = clt[q];
    for (int q = 0; q < 6; ++q) p.timing[sw * 16 + 8 + q] = clc[q];
  }
#endif
  if (w == 0) {
    const int mytree = sw * kWave + lane;
    if (mytree < p.B) {
      p.cnt[mytree] = xcnt[lane];   // the new root's particles (k_update)
      p.hdr[mytree].n_log = kept[lane];
      if (made[lane] != 0) p.hdr[mytree].n_nodes += made[lane];
      if (bad[lane] != 0) {
        p.hdr[mytree].error = POMCP_E_ARENA;
        p.upd_out[2 * mytree + 1] = POMCP_E_ARENA;
      }
    }
    if (lane == 0) p.wlog[sw] = out;
  }
}

// --------------------------------------------- the streaming re-root scan
// k_pack_cmap: one workgroup per search wave packs its 64 trees' block maps
// (k_compact's cmap, entries 0 .. old blocks - 1) as int16 back to back, with
// the offsets and a fit flag, so that every k_log_filter chunk stages them in
// LDS by one contiguous copy (when they do not fit, the filter reads the
// global cmap)
__global__ __launch_bounds__(256) void k_pack_cmap(DevParams p, int allow) {   // allow 0: tests only
  const int sw = blockIdx.x;
  const int t = (int)threadIdx.x, w = t >> 6, lane = lane_id();
  __shared__ int32_t off[kWave + 1];
  __shared__ int32_t ok;
  if (w == 0) {
    const int tr = sw * kWave + lane;
    const uint32_t c = tr < p.B ? p.scan_info[tr].y : 0u;   // 1 + old blocks (0: not re-rooted)
    const int nbo = c > 0u ? (int)c - 1 : 0;
    int inc = nbo;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int y = __shfl_up(inc, d);
      if (lane >= d) inc += y;
    }
    off[lane] = inc - nbo;
    if (lane == kWave - 1) off[kWave] = inc;
    const bool fit = __ballot(nbo > 32767) == 0ull && __shfl(inc, kWave - 1) <= kCm16;
    if (lane == 0) ok = fit && allow ? 1 : 0;
  }
  __syncthreads();
  int32_t* const o = p.cm16_off + (int64_t)sw * kCm16Off;
  if (t <= kWave) o[t] = off[t];
  if (t == kWave + 1) o[t] = ok;
  if (!ok) return;
  int16_t* const dst = p.cm16 + (int64_t)sw * kCm16;
  for (int l = w; l < kWave; l += 4) {   // wave w: tree lanes w, w + 4, ...
    const int32_t* const src = p.cmap + (int64_t)(sw * kWave + l) * p.Nb;
    const int b0 = off[l], nb = off[l + 1] - b0;
    for (int b = lane; b < nb; b += kWave) dst[b0 + b] = (int16_t)src[b];
  }
}

// (round 6) The re-root's scan of every search wave's log as two kernels.
//
// k_log_filter: the logs are cut into segments of kLfSeg records, processed by
// a persistent grid that claims chunks of kLfChunk consecutive segments of one
// log in increasing order (one atomic counter; chunk c is chunk c / waves of
// wave c % waves), so every segment a segment waits for was claimed earlier by
// a running workgroup: no deadlock whatever the residency.  A chunk's first
// segment waits only for the previous chunk of its log, claimed `waves`
// chunks earlier (long done); the others for the same workgroup's previous
// segment (done).  Only a chunk publishes (its last segment: the counts
// through it) and only a chunk's first segment looks back (at the previous
// chunk's publication); within a chunk the workgroup carries the prefix, and
// loads each segment's records while the previous one is being stored.  A segment classifies its records as k_compact_log
// does (kept and relabelled; deferred, kept with its new action node; the new
// root's, extracted; dropped), publishes its kept and per-tree extracted
// counts and learns those of the segments before it by decoupled look-back
// (LfDesc: write-through counts, then one write-through tag; the reader polls
// the tag), then stores its kept records at their final places and the
// extracted ones into the tree's next belief, and adds the kept records'
// visits (an LDS table per segment, one atomic per node).  In place: a segment
// publishes only after it has loaded all its records, a later segment stores
// only after reading that publication, and every place lies below the storing
// segment's own end -- no store lands on a record not yet read.  No workgroup
// walks a whole log: one search wave's 12.6 M records (the bench) spread over
// the whole GPU instead of one CU.
// k_log_mat = k_compact_log<Env, true>: one workgroup per wave over the
// compacted log (the kept records only, ~1/4): every tree's record count and
// the deferred children materialised in log order.
constexpr int kLfWaves = kLfThreads / kWave;
constexpr int kLfV = 2 * kLfSeg;   // a segment's visits table (entries)
constexpr int kLfVBits = kLfV == 4096 ? 12 : kLfV == 2048 ? 11 : -1;
static_assert(kLfVBits > 0, "the visits table takes log2(kLfV) bits");
constexpr int kLfSpin = 1 << 22;   // look-back polls before giving up (lf_fail[0])

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* q) {
  return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* q, uint32_t v) {
  __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class Env>
__global__ __launch_bounds__(kLfThreads) void k_log_filter(DevParams p, int nwaves) {
  constexpr int T = kLfThreads, R = kLfRecs, NW = kLfWaves;
  const int t = (int)threadIdx.x, w = t >> 6, lane = lane_id();
  __shared__ uint4 si[kWave];               // scan_info of the chunk's 64 trees
  __shared__ int32_t kc[R][NW];             // kept records per sub-pass and wave
  __shared__ uint8_t xw[R][NW][kWave];      // extracted records per sub-pass, wave, tree lane
  __shared__ uint16_t xq[R][NW][kWave];     // ... their exclusive prefix in the segment
  __shared__ uint32_t xpre[kWave];          // per tree lane: extracted before the segment
  __shared__ uint32_t kpre;                 // kept records before the segment
  __shared__ uint32_t vkey[kLfV];           // the visits table: node id | tree lane ...
  __shared__ int32_t vcnt[kLfV];            // ... and its kept records in this segment
  __shared__ uint32_t claim;
  // the log's cmap in LDS for the chunk (as k_compact_log: int16, when the 64
  // trees' old blocks fit), so a record's classification issues no dependent
  // global load
  constexpr int kCm = kCm16;
  __shared__ __attribute__((aligned(16))) int16_t cml[kCm];
  __shared__ int32_t cmo[kCm16Off];   // offsets per tree lane, [kWave + 1]: the fit flag
  const uint32_t A = (uint32_t)p.A;
  const uint64_t amag = (0x100000000ull + A - 1u) / A;   // x / A by a multiply (k_compact_log)
  auto divA = [&](uint32_t x) -> uint32_t { return (uint32_t)(((uint64_t)x * amag) >> 32); };
  const int64_t bstride = blk_stride_lines(p.lines);
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t ep = p.lf_epoch & 0x3FFFFFFFu;
  for (int i = t; i < kLfV; i += T) {
    vkey[i] = 0xFFFFFFFFu;   // (ids < kIdMask: pomcp_create)
    vcnt[i] = 0;
  }
  const int nchunk = (p.lf_nseg + kLfChunk - 1) / kLfChunk;   // chunks per log
  const int64_t total = (int64_t)nwaves * nchunk;
  for (;;) {
    if (t == 0) claim = atomicAdd(p.lf_fail + 1, 1u);   // (lf_fail[1]: the claims)
    __syncthreads();
    const int64_t c = claim;
    __syncthreads();   // (read before the next claim overwrites it)
    if (c >= total) break;
    const int sw = (int)(c % nwaves);
    const int ch = (int)(c / nwaves);
    const uint32_t n = p.wlog[sw];
    const int s0 = ch * kLfChunk;
    int s1 = s0 + kLfChunk < p.lf_nseg ? s0 + kLfChunk : p.lf_nseg;
    const int sn = (int)((n + (uint32_t)kLfSeg - 1u) / (uint32_t)kLfSeg);   // the log's segments
    if (s1 > sn) s1 = sn;
    if (s0 >= s1) continue;   // (no such chunk: none waits for it)
    const WaveLog wl(p.plog, p.Np, sw, p.tm);
    if (w == 0) {
      const int tr = sw * kWave + lane;
      si[lane] = tr < p.B ? p.scan_info[tr] : make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
    }
    if (t < kCm16Off) cmo[t] = p.cm16_off[(int64_t)sw * kCm16Off + t];   // (k_pack_cmap)
    // the chunk's first segment's records (each later one is loaded during the
    // previous one, after its dependent loads and before its stores)
    LogRec rn[R];
    uint32_t auxn[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t i = (uint32_t)s0 * (uint32_t)kLfSeg + (uint32_t)(j * T + t);
      rn[j] = LogRec{0u, 0u, 0u};
      auxn[j] = 0u;
      if (i < n) {
        rn[j] = wl.load(i);
        if (p.tm) auxn[j] = wl.aux[i];
      }
    }
    __syncthreads();
    const bool cml_on = cmo[kWave + 1] != 0;
    if (cml_on) {   // one contiguous copy, 8 entries per 16 B load, all loads issued first
      constexpr int kPer = (kCm / 8 + T - 1) / T;
      const int nq = (cmo[kWave] + 7) >> 3;
      const uint4* const src = reinterpret_cast<const uint4*>(p.cm16 + (int64_t)sw * kCm);
      uint4 v[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int e = q * T + t;
        v[q] = e < nq ? src[e] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int e = q * T + t;
        if (e < nq) reinterpret_cast<uint4*>(cml)[e] = v[q];
      }
    }
    __syncthreads();
    auto cm = [&](uint32_t ll, int tr, uint32_t b) -> int {
      return cml_on ? (int)cml[cmo[ll] + (int)b] : p.cmap[(int64_t)tr * p.Nb + (int)b];
    };
    for (int sg = s0; sg < s1; ++sg) {
      const uint32_t base = (uint32_t)sg * (uint32_t)kLfSeg;
      LogRec r[R];
      uint32_t aux[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        r[j] = rn[j];
        aux[j] = auxn[j];
      }
      // classification (k_compact_log's rules)
      bool keep[R], ex[R];
      uint32_t l[R];
      int32_t* vis[R];
      int vh[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const uint32_t i = base + (uint32_t)(j * T + t);
        keep[j] = false;
        ex[j] = false;
        l[j] = 0u;
        vis[j] = nullptr;
        vh[j] = -1;
        if (i < n) {
          l[j] = r[j].id >> kIdBits;
          const uint32_t id = r[j].id & kIdMask;
          const int tree = sw * kWave + (int)l[j];
          const uint4 inf = si[l[j]];
          ex[j] = inf.x == r[j].id;   // a record of the new root (never kept)
          keep[j] = true;
          if (inf.y != 0u) {   // re-rooted: only the new root's subtree stays
            int32_t nid = -1;
            if (id >= p.cut_base) {   // deferred: kept with its relabelled action node
              const uint32_t ani = id - p.cut_base, aq = divA(ani);
              const int nb = cm(l[j], tree, aq);
              keep[j] = nb >= 0;
              if (nb >= 0) r[j].id = (p.cut_base + (uint32_t)nb * A + (ani - aq * A)) | (l[j] << kIdBits);
            } else {
              if (id >= p.ovf_base) {
                nid = p.ovf_new[(int64_t)tree * p.H + (id - p.ovf_base)];
                if (nid >= 0) vis[j] = &p.ovf[(int64_t)tree * p.H + ((uint32_t)nid - p.ovf_base)].visits;
              } else if (id >= 1u) {
                const uint32_t ani = (id - 1u) / kSlots, k = (id - 1u) % kSlots;
                const uint32_t aq = divA(ani), ar = ani - aq * A;
                const int nb = cm(l[j], tree, aq);
                if (nb >= 0) {
                  nid = (int32_t)(((uint32_t)nb * A + ar) * kSlots + k + 1u);
                  uint4* const bp = reinterpret_cast<uint4*>(p.an + tree_base_lines(tree, p.Nb, p.lines) +
                                                             (int64_t)nb * bstride);
                  vis[j] = reinterpret_cast<int32_t*>(bp + part_slot((int)ar, (int)k)) + 3;
                }
              }
              keep[j] = nid >= 0;
              if (nid >= 0) r[j].id = (uint32_t)nid | (l[j] << kIdBits);
            }
          }
        }
      }
      // the next segment's records, in flight from here (issued after this
      // segment's dependent loads, before its stores: vmcnt retires in order)
      if (sg + 1 < s1) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const uint32_t i = base + (uint32_t)kLfSeg + (uint32_t)(j * T + t);
          rn[j] = LogRec{0u, 0u, 0u};
          auxn[j] = 0u;
          if (i < n) {
            rn[j] = wl.load(i);
            if (p.tm) auxn[j] = wl.aux[i];
          }
        }
      }
      // the kept records' nodes counted in the table (the entering thread adds
      // them below); ranks: kept records in segment order (sub-pass, wave,
      // lane), extracted records per tree lane likewise
      uint64_t mk[R];
      int xr[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (vis[j] != nullptr) {
          const uint32_t key = r[j].id;   // node id | tree lane (unique in the segment)
          int h = (int)((key * 0x9E3779B1u) >> (32 - kLfVBits));
          for (;;) {   // (a segment holds kLfSeg records: a free entry remains)
            const uint32_t old = atomicCAS(&vkey[h], 0xFFFFFFFFu, key);
            if (old == 0xFFFFFFFFu) vh[j] = h;
            if (old == 0xFFFFFFFFu || old == key) break;
            h = (h + 1) & (kLfV - 1);
          }
          atomicAdd(&vcnt[h], 1);
        }
        mk[j] = __ballot(keep[j]);
        if (lane == 0) kc[j][w] = __popcll(mk[j]);
        xw[j][w][lane] = 0;
        xr[j] = 0;
        if (__ballot(ex[j]) != 0ull) {
          const uint64_t xs = same_lane_mask(l[j], ex[j]);
          xr[j] = __popcll(xs & below);
          asm volatile("" ::: "memory");   // (the zero lands first: one wave's LDS ops run in order)
          if (ex[j] && (xs >> lane) == 1ull) xw[j][w][l[j]] = (uint8_t)__popcll(xs);
        }
      }
      __syncthreads();
      uint32_t xs_seg = 0u, ks_seg = 0u;   // (wave 0: this segment's counts)
      if (w == 0) {
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
          for (int v = 0; v < NW; ++v) {
            xq[j][v][lane] = (uint16_t)xs_seg;
            xs_seg += xw[j][v][lane];
            ks_seg += (uint32_t)kc[j][v];
          }
        if (sg == s0) {   // the counts before the chunk: the previous chunk's publication
          uint32_t kp = 0u, xp = 0u;
          if (ch > 0) {
            const LfDesc* const e = p.lf_desc + (int64_t)sw * nchunk + (ch - 1);
            for (int spin = 0;; ++spin) {
              const uint32_t tg = __builtin_amdgcn_readfirstlane(ld_sc1(&e->tag));
              if (tg == (ep << 2 | 2u)) break;
              if (spin >= kLfSpin) {   // (never expected: the previous chunk was claimed first)
                if (lane == 0) atomicExch(p.lf_fail, 1);
                break;
              }
              __builtin_amdgcn_s_sleep(2);
            }
            kp = ld_sc1(&e->kept_inc);
            xp = ld_sc1(&e->ex_inc[lane]);
          }
          xpre[lane] = xp;
          if (lane == 0) kpre = kp;
        }
      }
      __syncthreads();
      // stores: kept records at their final places, extracted ones into the
      // tree's next belief ({root_t + 1, v0, v1, aux}, mcts.py:248-252), the
      // visits one atomic per node
      const uint32_t kp = kpre;
      int pre = 0;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        int pw = 0, tj = 0;
#pragma unroll
        for (int v = 0; v < NW; ++v) {
          pw += v < w ? kc[j][v] : 0;
          tj += kc[j][v];
        }
        if (keep[j]) {
          const uint32_t at = kp + (uint32_t)(pre + pw + __popcll(mk[j] & below));
          wl.store(at, r[j]);
          if (p.tm) wl.aux[at] = aux[j];
        }
        if (ex[j]) {
          const uint4 inf = si[l[j]];
          const uint32_t pos = xpre[l[j]] + xq[j][w][l[j]] + (uint32_t)xr[j];
          const uint32_t room = inf.z & 0x7FFFFFFFu;
          if (pos < room)   // (beyond: k_update fails the tree, POMCP_E_ARENA)
            p.belief[(int64_t)(sw * kWave + (int)l[j]) * p.Nr + bel_at((int)(inf.z >> 31), p.Nr, pos)] =
                make_uint4(inf.w, r[j].v0, r[j].v1, aux[j]);
        }
        if (vh[j] >= 0) atomicAdd(vis[j], vcnt[vh[j]]);
        pre += tj;
      }
      __syncthreads();   // (every count read: clear the table, advance the prefix)
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (vh[j] >= 0) {
          vkey[vh[j]] = 0xFFFFFFFFu;
          vcnt[vh[j]] = 0;
        }
      if (w == 0) {
        const uint32_t kn = kp + ks_seg, xn = xpre[lane] + xs_seg;
        xpre[lane] = xn;
        if (lane == 0) kpre = kn;
        if (sg + 1 == s1) {   // the chunk's counts through its last segment, for the next chunk
          LfDesc* const d = p.lf_desc + (int64_t)sw * nchunk + ch;
          st_sc1(&d->ex_inc[lane], xn);
          if (lane == 0) st_sc1(&d->kept_inc, kn);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) st_sc1(&d->tag, ep << 2 | 2u);
        }
      }
      __syncthreads();
    }
  }
}

// Synthetic roots: env b0 sample for tree b under key (env_seed_base + b,
// 0x40000000), the ego's initial observation.
template <class Env>
__global__ __launch_bounds__(256) void k_synthetic_obs(DevParams p, uint64_t env_seed_base) {
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  Streams env;
  env.seed = env_seed_base + (uint64_t)tree;
  env.tree = 0x40000000u;
  for (int k = 0; k < 5; ++k) env.ctr[k] = 0;
  uint32_t s0, s1;
  Env::sample_initial(sm, [&](uint32_t n) { return env.model(n); }, &s0, &s1);
  const uint64_t key = Env::obs_key(sm, p.ego, s0, s1);
  if (lane_id() == 0) p.out_obs[tree] = key;
}

// Synthetic environment step (bench: an update()-inclusive planning step): tree
// b's true initial state again (the same draws as k_synthetic_obs), one joint
// step with the ego's action in_actions[b] and the other agent's action drawn
// uniformly from the env key's action stream, the ego's next observation.
template <class Env>
__global__ __launch_bounds__(256) void k_synthetic_step(DevParams p, uint64_t env_seed_base) {
  __shared__ typename Env::Model sm;
  stage_model(p.model, sm);
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  Streams env;
  env.seed = env_seed_base + (uint64_t)tree;
  env.tree = 0x40000000u;
  for (int k = 0; k < 5; ++k) env.ctr[k] = 0;
  uint32_t s0, s1;
  Env::sample_initial(sm, [&](uint32_t n) { return env.model(n); }, &s0, &s1);
  const int a = p.in_actions[tree];
  const uint32_t ao = env.act(p.other, (uint32_t)p.A);
  const uint32_t j = Env::kStepDraws ? env.model(2) : 0u;
  uint32_t n0, n1;
  double r;
  int done;
  Env::step(sm, p.ego, s0, s1, (uint32_t)(a >= 0 && a < p.A ? a : 0), ao, j, &n0, &n1, &r, &done);
  const uint64_t key = Env::obs_key(sm, p.ego, n0, n1);
  if (lane_id() == 0) p.out_obs[tree] = key;
}

// Restore of the post-initial-update root state (see pomcp_snapshot).  The
// live stream key (seed) is kept: a pomcp_rekey after the snapshot (root-
// parallel ranks, bench.py) must survive every restore.
__global__ __launch_bounds__(256) void k_restore(DevParams p, const TreeHdr* snap) {
  const int tree = blockIdx.x * kTreesPerBlock + (threadIdx.x >> 6);
  if (tree >= p.B) return;
  const int lane = lane_id();
  const TreeHdr live = p.hdr[tree];
  int epoch = (live.epoch + 1) & (int)kEpochMask;
  if (epoch == 0) {
    clear_ovf(p, tree, lane);
    epoch = 1;
  }
  if (lane == 0 && (tree & (kWave - 1)) == 0) p.wlog[tree / kWave] = 0u;   // snapshot: empty logs
  if (lane == 0) {
    TreeHdr h = snap[tree];
    h.epoch = epoch;
    h.seed = live.seed;
    p.hdr[tree] = h;
  }
}

// Root-parallel merge: trees [g * group, (g + 1) * group) are
// the root-parallel replicas of planner g on every rank; their exchange
// records (pomcp.h POMCP_XREC: (visits, total) per root action + step
// statistics, written by k_search) are read from `src` = [world][B][R] (one
// rank's merge buffer, or the all-gathered buffers of `world` ranks in rank
// order), replica j = r * group + k being tree g * group + k of rank r, and the
// merged action chosen:
//   * PUCB  (max_visit_action_selection, mcts.py:565-581): argmax of summed visits;
//   * UCB / uniform (max_value_action_selection, mcts.py:583-600): argmax of
//     summed total / summed visits over the visited actions;
// lowest action on ties (the replicas' choice must be the same everywhere, so
// the reference's random tie-break is not drawn); 0 when nothing was visited
// (action_space[0], mcts.py:270-272).  Summation order is fixed: lane l of the
// group's wave sums replicas [l * c, (l + 1) * c), c = ceil(N / 64), in replica
// order from 0.0, then lane 0 sums the 64 partials in lane order from 0.0
// (restated by oracle/root_parallel.py, bit-exact), so every rank takes the
// same decision and it does not depend on how the records were exchanged.
// The step statistics of the replicas (search depth, simulations, root visits,
// MinMaxStats, errors) are reduced alongside.
__global__ __launch_bounds__(64) void k_merge_roots(const double* src, int B, int A, int sel,
                                                    int group, int world,
                                                    pomcp_merged_root* out) {
  __shared__ double part[2][POMCP_MAX_ACTIONS][kWave];
  __shared__ double pmm[2][kWave];
  __shared__ int64_t pn[2][kWave];
  __shared__ int32_t pi[2][kWave];
  const int g = blockIdx.x, lane = lane_id();
  const int R = POMCP_XREC(A);
  const int n = world * group;
  const int c = (n + kWave - 1) / kWave;
  const int j0 = min(lane * c, n), j1 = min(j0 + c, n);
  double v[POMCP_MAX_ACTIONS], t[POMCP_MAX_ACTIONS];
#pragma unroll
  for (int a = 0; a < POMCP_MAX_ACTIONS; ++a) v[a] = t[a] = 0.0;
  double mn = __builtin_inf(), mx = -__builtin_inf();
  int64_t sims = 0, rv = 0;
  int depth = 0, err = 0;
  for (int j = j0; j < j1; ++j) {
    const int r = j / group, k = j - r * group;
    const double* m = src + ((int64_t)r * B + (int64_t)g * group + k) * R;
#pragma unroll
    for (int a = 0; a < POMCP_MAX_ACTIONS; ++a)
      if (a < A) {
        v[a] = v[a] + m[2 * a];
        t[a] = t[a] + m[2 * a + 1];
      }
    const double* s = m + 2 * A;
    sims += (int64_t)s[0];
    rv += (int64_t)s[1];
    depth = max(depth, (int)s[2]);
    if (err == 0) err = (int)s[3];
    if (s[4] < mn) mn = s[4];
    if (s[5] > mx) mx = s[5];
  }
#pragma unroll
  for (int a = 0; a < POMCP_MAX_ACTIONS; ++a) {
    part[0][a][lane] = v[a];
    part[1][a][lane] = t[a];
  }
  pmm[0][lane] = mn;
  pmm[1][lane] = mx;
  pn[0][lane] = sims;
  pn[1][lane] = rv;
  pi[0][lane] = depth;
  pi[1][lane] = err;
  __syncthreads();
  if (lane != 0) return;
  pomcp_merged_root r;
  r.action = 0;
  r.num_trees = n;
  r.search_depth = 0;
  r.error = 0;
  r.num_sims = 0;
  r.root_visits = 0;
  r.min_value = __builtin_inf();
  r.max_value = -__builtin_inf();
  for (int l = 0; l < kWave; ++l) {
    r.search_depth = max(r.search_depth, pi[0][l]);
    if (r.error == 0) r.error = pi[1][l];
    r.num_sims += pn[0][l];
    r.root_visits += pn[1][l];
    if (pmm[0][l] < r.min_value) r.min_value = pmm[0][l];
    if (pmm[1][l] > r.max_value) r.max_value = pmm[1][l];
  }
  double best = 0.0;
  bool any = false;
  for (int a = 0; a < POMCP_MAX_ACTIONS; ++a) {
    double sv = 0.0, st = 0.0;
    if (a < A)
      for (int l = 0; l < kWave; ++l) {
        sv = sv + part[0][a][l];
        st = st + part[1][a][l];
      }
    r.visits[a] = sv;
    r.totals[a] = st;
    if (a >= A || !(sv > 0.0)) continue;
    const double score = sel == POMCP_SEL_PUCB ? sv : st / sv;
    if (!any || score > best) {
      best = score;
      r.action = a;
      any = true;
    }
  }
  out[g] = r;
}

__global__ void k_exp_selftest(const double* x, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = host_exp(x[i]);   // the I-NTMCP softmax's exp (host_exp.h)
}

__global__ void k_fast_recip(const double* x, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[2 * i + 0] = rcp_nr(x[i]);
  out[2 * i + 1] = rsq_nr(x[i]);
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
