// Device-side data layout and wave-level helpers of the POMCP engine.
//
// The search (k_search, pomcp_search.hip) runs one tree per lane.  The
// re-root / reset kernels (pomcp_kernels.hip) run one tree per wavefront and
// spread the data-parallel parts over lanes:
//   * a block load = one coalesced (A + 1) x 128 B load, lane l holds part l
//   * obs-child lookup among the 6 inline slots -> 6 lanes, 1 ballot
//   * the ego observation window (15 cells)    -> lanes 0..14, 2 ballots
//   * belief extraction at re-root             -> 64 log records / step
//   * RNG: an LDS page of Philox blocks, one per lane, a draw is a broadcast read
// A tree is touched by exactly one wave (or lane), so no atomics are needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "driving.h"
#include "philox.h"
#include "../../include/pomcp.h"

namespace pb {

constexpr int kWave = 64;
constexpr int kTreesPerBlock = 4;      // 256-thread workgroups, one tree per wave
constexpr int kSlots = 6;              // inline obs children per action node
constexpr int kLine = 8;               // 16 B parts per 128 B line
constexpr int kBucket = 16;            // overflow map bucket (16 x 32 B)
constexpr int kEpochShift = 50;        // obs keys use bits 0..49
constexpr uint32_t kEpochMask = 0x3FFF;
constexpr uint64_t kObsMask = (1ull << 50) - 1;
constexpr uint64_t kValidBit = 1ull << 62;
constexpr uint64_t kAbsorbBit = 1ull << 63;
constexpr int kMaxPath = 64;           // tree levels per simulation (one lane each)
constexpr uint32_t kRootId = 0;        // obs node id of a root created by the initial update

// Action nodes (node.py:120-178) with their obs children inline (node.py:144-160).
// An expanded obs node owns a block of (A + 1) x 128 B lines, in 16 B parts:
//   line 0 (the node line), A <= 5:
//     bytes   0..19  visits of action a (u32 at 4a)             ActionNode.visits
//     bytes  20..23  the node's own visits                       ObsNode.visits
//     bytes  24..31  math.log(node visits + 1): log(N) of the next arrival
//     bytes 32 + 16a {value, total} of action a (f64, f64)       value / total_value
//   line 1 + a : parts 1..6 = child slots k of action a (ChildSlot), part 0 unused
// A tree level reads the node line (selection, with the node's N and log(N) in
// it: no host-table load on the path) and the chosen action's slot line; its
// backup writes the node line only (bytes 0..31 and the action's 16 B).
// ActionNode.agg (node.py:141-178, the running variance) is not kept: only
// ActionNode.variance reads it and only __str__ reads that.
// ObsNode.visits of an EXPANDED child is its block's bytes 20..23; the slot's
// visits field is authoritative only while the child has no block, and only
// while it is within the depth / step limits: an arrival cut off there
// (mcts.py:315) does not rewrite its slot (k_search), so k_compact /
// k_compact_log recount every slot's visits from the particle log (one record
// per arrival) at each re-root.
struct ChildSlot {
  uint64_t key;     // obs key | valid << 62 | is_absorbing << 63
  int32_t block;    // action block of the child obs node (-1 = leaf)
  int32_t visits;   // ObsNode.visits while block == -1 (see above)
};
constexpr int kNodeVisByte = 20;   // node line: the node's visits (u32)
constexpr int kNodeLogByte = 24;   // node line: math.log(visits + 1) (f64)
__host__ __device__ constexpr int part_vt(int a) { return 2 + a; }   // {value, total} of a
// Particle log record (ObsNode.belief.add_particle, mcts.py:371): the particle
// (v0, v1) entered obs node `id` of the tree in lane `lane` of the search wave.
// Its time step is not stored: every particle of a node has the same t (the
// root's particles have t = root_t, a node at depth d below it t = root_t + d),
// so re-rooting restores it as root_t + 1.
// The log is shared by the 64 trees of a search wavefront (one tree per lane):
// the lanes appending in one step write consecutive records, so one store
// instruction writes whole lines instead of 64 scattered 12 B pieces.  A
// tree's records keep their insertion order; the re-root (k_compact_log)
// separates them again.
constexpr int kIdBits = 26;                       // obs node ids < 2^26 (pomcp_create checks)
constexpr uint32_t kIdMask = (1u << kIdBits) - 1u;
// Deferred records (k_search): a simulation that reaches an obs node whose
// children lie beyond the depth / step limits (mcts.py:315) only needs its
// child for the particle record -- the child is never stepped into during this
// search (mcts.py:315 returns 0 for it, whatever its slot holds).  Such a record
// carries id = cut_base + action node index instead of the child's id, and
// the child slot is neither read nor written by the search; the child's
// observation key and absorbing flag follow from the record's state (both are
// functions of the next state, envs.h), so the re-root materialises the
// children of the records it keeps (k_compact_log) and drops the rest with
// the garbage-collected part of the tree.  Only labels and the time of the
// slot writes change: every arrival is still one record, in order.
struct LogRec {
  uint32_t id;      // obs node id | lane << kIdBits
  uint32_t v0, v1;
};

// A search wave's particle log in memory: structure of arrays, ids[cap] then
// v0[cap] then v1[cap] (cap = 64 Np records), so an append of the wave's
// records is three fully coalesced dword stores instead of one 12 B-strided
// store (+1% measured; the log's cost is its bytes: without any log store
// the search runs 12% faster, tools/ablate.sh).  A type-based context
// (POTMMCP, pomcp_set_type_policies) adds aux[cap]: the particle's
// other-agent policy index (HistoryPolicyState.policy_state, potmmcp.py:83-98).
struct WaveLog {
  uint32_t* id;
  uint32_t* v0;
  uint32_t* v1;
  uint32_t* aux;   // null unless type-based
  __device__ __forceinline__ WaveLog(LogRec* plog, int64_t Np, int64_t wave, int tm = 0) {
    const int64_t cap = (int64_t)64 * Np;
    id = reinterpret_cast<uint32_t*>(plog) + wave * (3 + tm) * cap;
    v0 = id + cap;
    v1 = v0 + cap;
    aux = tm ? v1 + cap : nullptr;
  }
  __device__ __forceinline__ LogRec load(int64_t i) const { return LogRec{id[i], v0[i], v1[i]}; }
  __device__ __forceinline__ void store(int64_t i, const LogRec& r) const {
    id[i] = r.id;
    v0[i] = r.v0;
    v1[i] = r.v1;
  }
};

struct alignas(16) Line {   // allocation unit of the block arena
  uint4 part[kLine];
};
// Lines per block: the node line + one per action, + the prior line of a
// type-based context (POTMMCP: ObsNode.action_probs, A doubles at line A + 1).
__host__ __device__ constexpr int blk_lines(int A, int tm = 0) { return A + 1 + tm; }
__host__ __device__ constexpr int blk_parts(int L) { return kLine * L; }   // L: lines per block
__host__ __device__ constexpr int part_slot(int a, int k) { return kLine * (1 + a) + 1 + k; }
__host__ __device__ constexpr int part_prior(int A) { return kLine * (A + 1); }

// The block arena is interleaved by search wave ([wave][block][lane] of
// L-line blocks, L = blk_lines): block b of tree t starts at line
//   ((t / 64 * Nb + b) * 64 + t % 64) * L
// so the 64 trees of a k_search wave (one per lane) keep their blocks in one
// contiguous region whose size follows the blocks in use, not Nb.  With a
// per-tree layout a wave's accesses spread over 64 regions of Nb blocks each
// and the address translation caches thrash (tools/ubench).
// A block is still one contiguous L x 128 B piece (coalesced loads of the
// wave-per-tree kernels are unchanged); consecutive blocks of one tree are
// blk_stride_lines(L) apart.
__host__ __device__ inline int64_t tree_base_lines(int t, int64_t Nb, int L) {
  return ((int64_t)(t / kWave) * Nb * kWave + (t % kWave)) * L;
}
__host__ __device__ constexpr int64_t blk_stride_lines(int L) { return (int64_t)kWave * L; }
__host__ __device__ inline int64_t arena_lines(int B, int64_t Nb, int L) {
  return (int64_t)((B + kWave - 1) / kWave) * kWave * Nb * L;
}

// Type-based search (POTMMCP, potmmcp.py:18-301) with fixed-distribution
// policies (planning/policies.py): every table holds the doubles Python's
// random.choices bisects (cumulative weights and total = cum[-1] + 0.0).
constexpr int kTmMax = 8;               // ego / other-agent policies
constexpr int kCodeShift = 50;          // inline slot key bits 50..53: the child's prior code
constexpr uint64_t kCodeMask = 15ull << kCodeShift;
// Prior code of an obs node (its ObsNode.action_probs at creation): 0 = the
// meta-policy's expected prior (get_expected_action_probs, potmmcp.py:391-431:
// roots made by update), k + 1 = ego policy k's get_pi (a child created by a
// simulation that sampled ego policy k, potmmcp.py:275-287).  Overflow
// entries keep it in flags bits 1..4.
struct TmTables {
  int32_t n_ego, n_other, pad[2];
  // the base planner's modes (pomcp_type_policies): no sample_policy draw, no
  // mixture draw per initial particle, Discrete.sample() for the ego's rollout /
  // the other agent
  int32_t no_meta_draw, no_mixture_draw, ego_uniform, other_uniform;
  double prior[kTmMax + 1][kTmMax];     // [code][a]: the action_probs a node starts with
  double ego_cum[kTmMax][kTmMax];       // ego policy k's action draw (rollouts)
  double ego_tot[kTmMax];
  double oth_cum[kTmMax][kTmMax];       // other-agent policy j's action draw
  double oth_tot[kTmMax];
  double meta_cum[kTmMax][kTmMax];      // sample_policy: meta_policy[j] in its dict order
  double meta_tot[kTmMax];
  int32_t meta_idx[kTmMax][kTmMax];     // ego policy of meta_policy[j]'s i-th key
  int32_t meta_len[kTmMax];
};
// random.choices(population, weights): bisect_right(cum, x, 0, n - 1) for
// x = random() * total, as CPython computes it (a linear scan: n <= 8).
__device__ __forceinline__ int tm_choice(const double* cum, double total, int n, uint32_t w) {
  const double x = uniform_float(w) * total;
  int i = n - 1;
  for (int q = n - 2; q >= 0; --q)
    if (x < cum[q]) i = q;
  return i;
}

// Overflow children (> kSlots per action node): open-addressing map keyed by
// (action node, obs).  32 B entries; valid when key's epoch matches.
struct OvfSlot {
  uint64_t key;     // obs | epoch << 50
  uint32_t an;      // action node index
  uint32_t flags;   // bit 0: is_absorbing
  int32_t block;
  int32_t visits;
  uint64_t pad;
};

// Per-tree header (device resident between calls).
struct TreeHdr {
  int32_t n_blocks, n_log, n_nodes, error;
  int32_t belief_size, belief_sel, epoch, root_t;
  uint32_t root_id;
  int32_t root_blk, root_visits, root_abs;
  double mm_min, mm_max;
  uint64_t seed;
  uint32_t tree_key;
  uint32_t ctr[5];     // belief, select, model, act0, act1
  int32_t root_code;   // type-based: the root's prior code while it has no block
  uint32_t ctr_mix;    // type-based: S_MIXTURE draws (the other agent's policy per particle)
};

// Streaming re-root scan (k_log_filter, round 6): one look-back record per
// segment of a search wave's log.  `tag` = epoch << 2 | state (1: the
// segment's own counts published, 2: the counts through it); the counts are
// stored write-through before the tag (MI355X guide: sc1 payload, drained,
// then one sc1 flag store; the reader polls the tag with sc1 loads).
struct alignas(16) LfDesc {
  uint32_t tag, kept_agg, kept_inc, pad;
  uint32_t ex_agg[64];   // extracted records of tree lane l in the segment ...
  uint32_t ex_inc[64];   // ... and in the segments up to it
};

struct DevParams {
  int32_t B, A, ego, other, sel, depth_limit, step_limit, n_target, has_kb, ncells;
  double discount, c, pucb_f, limit_factor, kb_min, kb_max;
  int64_t Nb, Np, Nr, H;
  uint32_t bucket_mask;
  uint32_t ovf_base;    // node ids >= ovf_base are overflow entries
  uint32_t cut_base;    // ids >= cut_base: deferred records (cut_base + action node index), below
  int32_t islots;       // inline obs slots in use per action node (kSlots; fewer only in
                        // tests of the overflow map: pomcp_debug_set_inline_slots)
  int32_t lines;        // lines per block (blk_lines(A, tm))
  int32_t spin_max;     // k_search_lds: polls of a late step-tree hand-off before the search
                        // wave runs on without producers (0: the default; tests shrink it)
  int32_t tm;           // type-based search (POTMMCP): tmt, prior lines, log aux
  int32_t defer;        // k_search: defer cut-off children to the re-root (pomcp_set_defer_cutoff)
  double sel_margin;    // k_search: fast-selection margin (1e-12; pomcp_debug_set_select_margin)
  const TmTables* tmt;
  TreeHdr* hdr;
  Line* an;             // [B][Nb][lines] action blocks
  OvfSlot* ovf;         // [B][H]
  LogRec* plog;         // [waves][64 * Np] per-search-wave particle log
  LogRec* lscr;         // [B][Np] k_search_lds: one launch's records per tree (allocated on
                        // first use), appended to plog by k_log_merge
  uint32_t* wlog;       // [waves] records in each wave's log
  uint32_t* want;       // [B] re-root: log id of the child to extract (0xFFFFFFFF: none)
  int4* want_info;      // [B] re-root: that child's {block, absorbing, code, found} (k_update)
  int32_t* cnt;         // [B] re-root: particles extracted into the new root belief
  uint4* belief;        // [B][Nr] {t, v0, v1, aux}: the root belief and the one being
                        // built, one from each end (bel_at)
  uint4* path;          // [B][3 * kMaxPath] search path of the running simulation
  const double* logtab;
  int64_t logtab_n;
  const double* dpow;
  int32_t dpow_n;
  const void* model;    // Env::Model (envs.h), staged in LDS by every kernel
  int32_t env;          // pomcp_env
  pomcp_root_stats* stats;
  double* merge;        // [B][POMCP_XREC(A)] exchange records (pomcp.h)
  int32_t* upd_out;     // [B][2] {root_abs, error}
  const int32_t* in_actions;
  const uint64_t* in_obs;
  uint64_t* out_obs;
  uint64_t* timing;     // [waves][16] phase cycles (diagnostics build only), may be null
  // subtree compaction at re-root (k_compact / k_compact_log), allocated on the
  // first re-root: block -> new index (-1: not in the new root's subtree), the
  // parent block / alive list, overflow slot -> new obs node id, the live
  // overflow entries being re-inserted
  int32_t* cmap;        // [B][Nb]
  int32_t* cpar;        // [B][Nb]
  int32_t* ovf_new;     // [B][H]
  OvfSlot* ovf_tmp;     // [B][H]
  // the streaming re-root scan (k_log_filter / k_log_mat, pomcp_kernels.hip),
  // allocated on the first re-root: per tree {want, 1 + old blocks (0: not
  // re-rooted), end of the next belief << 31 | its room, t of the new root}
  // (k_compact), the look-back records of every wave's log segments
  uint4* scan_info;     // [B]
  LfDesc* lf_desc;      // [waves][chunks per log]
  // every log's block map packed for the filter (k_pack_cmap): per wave its 64
  // trees' cmap entries as int16, back to back, and their offsets (+ a fit flag)
  int16_t* cm16;        // [waves][kCm16]
  int32_t* cm16_off;    // [waves][kCm16Off]: 65 offsets, fit flag
  int32_t lf_nseg;      // segments per wave log (its capacity / kLfSeg)
  uint32_t lf_epoch;    // this re-root's tag epoch (1, 2, ...; older tags are stale)
  uint32_t* lf_fail;    // [2] a look-back wait that gave up (never expected: POMCP_E_HIP);
                        // the segment claims of the running k_log_filter
};

// Root belief region of a tree: Nr records holding the current root belief and
// the next one (built by the re-root while the current one is still read by
// the reinvigoration), one from each end: belief_sel 0 keeps particle i at
// record i, belief_sel 1 at record Nr - 1 - i.  A re-root therefore needs
// old + new particles <= Nr (checked: POMCP_E_ARENA), not two full buffers --
// the update()-inclusive bench step (a few hundred root particles before, up to
// one per simulation after) fits 65,536 trees in HBM.
__host__ __device__ __forceinline__ int64_t bel_at(int sel, int64_t Nr, int64_t i) {
  return sel ? Nr - 1 - i : i;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t rlu(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

__device__ __forceinline__ double rl_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// c ? a : b for uint4, component by component.  A conditional operator or a
// conditional assignment on the vector struct is an aggregate copy whose
// source clang picks by address (a select of pointers): an array read that way
// ("if (q == a) x = arr[q]") stays in scratch memory instead of registers.
__device__ __forceinline__ uint4 sel4(bool c, uint4 a, uint4 b) {
  return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

__device__ __forceinline__ double hilo_d(uint32_t lo, uint32_t hi) {
  return __hiloint2double((int)hi, (int)lo);
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t uniu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (uint64_t)uniu((uint32_t)v) | ((uint64_t)uniu((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ double uni_d(double v) {
  return __hiloint2double(uni(__double2hiint(v)), uni(__double2loint(v)));
}

// 1 / x and 1 / sqrt(x) in FP64: the hardware estimates (v_rcp_f64 /
// v_rsq_f64, relative error ~2^-24) refined by one Newton step each: relative
// error <= 5e-15 measured on every visit count below 2^20 and random doubles
// (tools/recip_err.py, test_fast_ucb_reciprocals_error_bound), far inside the
// fast UCB scores' 1e-12 fallback margin (select_action: the exact scores
// decide near-ties).  A second step (round 4) measured -0.3% (r5n).
#ifndef PB_NR_STEPS   // A/B builds: Newton steps of the fast reciprocals
#define PB_NR_STEPS 1
#endif
__device__ __forceinline__ double rcp_nr(double x) {
  double y = __builtin_amdgcn_rcp(x);
#pragma unroll
  for (int i = 0; i < PB_NR_STEPS; ++i) {
    const double e = __builtin_fma(-x, y, 1.0);
    y = __builtin_fma(y, e, y);
  }
  return y;
}
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
#pragma unroll
  for (int i = 0; i < PB_NR_STEPS; ++i) y = y * __builtin_fma(-hx, y * y, 1.5);
  return y;
}
// sqrt(x) for a fast score (x >= 0): the IEEE square root (PB_FAST_SQRT A/B
// builds: x rsq_nr(x), measured +-0%)
__device__ __forceinline__ double sqrt_fast(double x) {
#ifdef PB_FAST_SQRT
  return x > 0.0 ? x * rsq_nr(x) : 0.0;
#else
  return __builtin_sqrt(x);
#endif
}

__device__ __forceinline__ uint32_t spread16(uint32_t x) {
  x &= 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}

// Ego observation key, one window cell per lane.
__device__ __forceinline__ uint64_t obs_key_wave(const DrvGrid& g, uint32_t self, uint32_t other,
                                                 int ncells) {
  const int lane = lane_id();
  const int cell = lane < ncells ? obs_cell(g, self, other, lane) : 0;
  const uint64_t b0 = __ballot(cell & 1);
  const uint64_t b1 = __ballot(cell & 2);
  const uint64_t cells = (uint64_t)(spread16((uint32_t)b0) | (spread16((uint32_t)b1) << 1));
  return uni64(cells | obs_tail(g, self));
}

__device__ __forceinline__ uint32_t ovf_hash(uint32_t an, uint64_t key) {
  uint64_t h = key ^ ((uint64_t)an * 0x9E3779B97F4A7C15ull);
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return (uint32_t)h;
}

// Wave-cached Philox stream in LDS: a page of kRngPage consecutive draws
// (kRngPage / 4 Philox blocks, one per lane, each written with one
// ds_write_b128) is refilled by the wave in one pass; a draw is one broadcast
// LDS read.  Same words as philox_word() (philox.h).
constexpr uint32_t kRngPage = 128;
struct LdsStream {
  uint32_t* page;   // this wave's kRngPage-word LDS page
  __device__ __forceinline__ void refill(uint64_t seed, uint32_t tree, uint32_t stream,
                                         uint32_t pg) {
    const uint32_t lane = (uint32_t)lane_id();
    if (lane < kRngPage / 4) {
      uint32_t c[4] = {pg * (kRngPage / 4) + lane, 0u, stream, (uint32_t)(seed >> 32)};
      philox4x32(c, (uint32_t)seed, tree);
      reinterpret_cast<uint4*>(page)[lane] = make_uint4(c[0], c[1], c[2], c[3]);
    }
  }
  __device__ __forceinline__ uint32_t get(uint32_t j) const {
    return uniu(page[j & (kRngPage - 1)]);
  }
};

}  // namespace pb
