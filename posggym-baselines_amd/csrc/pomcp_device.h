// Device-side data layout and wave-level helpers of the POMCP engine.
//
// One 64-lane wavefront owns one search tree (one planner).  Serial parts of
// the reference's per-simulation loop run wave-uniform (every lane holds the
// same value), the data-parallel parts are spread over lanes:
//   * UCB / PUCB scores of the A action children  -> lanes 0..A-1
//   * the ego observation window (15 cells)       -> lanes 0..14, 2 ballots
//   * obs-child lookup (16-slot hash bucket)      -> lanes 0..15, 1 ballot
//   * belief extraction at re-root                -> 64 log records / step
// A tree is touched by exactly one wave, so no atomics are needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "driving.h"
#include "philox.h"
#include "../../include/pomcp.h"

namespace pb {

constexpr int kWave = 64;
constexpr int kTreesPerBlock = 4;        // 256-thread workgroups, one tree per wave
constexpr int kBucket = 16;              // hash bucket = 16 slots = 256 B
constexpr int kEpochShift = 50;          // obs keys use bits 0..49
constexpr uint32_t kEpochMask = 0x3FFF;
constexpr int kMaxPath = 64;             // tree levels per simulation (one VGPR lane each)

// Action node: ActionNode.{visits, value, total_value, agg} (node.py:120-178).
struct ActRec {
  int32_t visits;
  int32_t pad;
  double value;
  double total;
  double agg;
};

// obs-child map entry: (action node, observation) -> obs node (node.py:144-160).
struct Slot {
  uint64_t key;      // obs key | epoch << 50
  uint32_t an;       // action node index
  uint32_t child;    // obs node index
};

// Per-tree header (device resident between calls).
struct TreeHdr {
  int32_t root, n_obs, n_blocks, n_log;
  int32_t belief_size, belief_sel, epoch, error;
  int32_t root_t, root_abs, pad0, pad1;
  double mm_min, mm_max;
  uint64_t seed;
  uint32_t tree_key;
  uint32_t ctr[5];
};

struct DevParams {
  int32_t B, A, ego, other, sel, depth_limit, step_limit, n_target, has_kb, ncells;
  double discount, c, pucb_f, limit_factor, kb_min, kb_max;
  int64_t No, Nb, Np, Nr, H;
  uint32_t bucket_mask;
  TreeHdr* hdr;
  int2* onode;          // {block, visits}
  int32_t* ometa;       // t << 1 | is_absorbing
  ActRec* an;
  Slot* hash;
  uint4* plog;          // {obs node, t, v0, v1}
  uint4* belief;        // 2 x Nr per tree: {t, v0, v1, 0}
  const double* logtab;
  int64_t logtab_n;
  const double* dpow;
  int32_t dpow_n;
  const DrvGrid* grid;
  pomcp_root_stats* stats;
  double* merge;        // [B][A][2]
  int32_t* upd_out;     // [B][2] {root_abs, error}
  const int32_t* in_actions;
  const uint64_t* in_obs;
  uint64_t* out_obs;
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

__device__ __forceinline__ double rl_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

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
  return cells | obs_tail(g, self);
}

__device__ __forceinline__ uint32_t slot_hash(uint32_t an, uint64_t key) {
  uint64_t h = key ^ ((uint64_t)an * 0x9E3779B97F4A7C15ull);
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return (uint32_t)h;
}

}  // namespace pb
