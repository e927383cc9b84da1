// C-ABI host side of libpomcp_hip.so (include/pomcp.h).
//
// Owns every device allocation of a planner batch, validates the
// MCTSConfig-derived parameters (config.py:33-55 asserts) and launches the
// kernels of pomcp_kernels.hip on one HIP stream.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

// Single translation unit: the kernels are compiled together with their launchers.
#include "pomcp_kernels.hip"
// the host-only entry points (environment models, RNG words, log / exp tables):
// plain C++, also built on its own with the host sanitizers (tests/test_host_sanitize.py)
#include "host_api.cpp"
#include "pomcp_search.hip"
#include "pomcp_search_lds.hip"
#include "../../include/intmcp.h"   // (INTMCP_MAX_TREES)
#include "intmcp.hip"
#include "../../include/pomcp_debug.h"

using namespace pb;

// k_search lives in pomcp_search_tu.hip (a translation unit of its own)
const void* pb_search_kernel(int row, int e, int sel);

static_assert(sizeof(pomcp_grid) == sizeof(DrvGrid), "grid layout");
static_assert(sizeof(pomcp_pe_grid) == 1344, "pe grid layout");
static_assert(sizeof(Line) == 128, "block line layout");
static_assert(sizeof(OvfSlot) == 32, "overflow slot layout");

struct pomcp_ctx {
  pomcp_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  DevParams dp{};
  std::vector<void*> allocs;
  std::string err;
  bool have_snapshot = false;
  TreeHdr* snap_hdr = nullptr;
  std::vector<int32_t> host_upd;
  std::vector<pomcp_root_stats> host_stats;
  DrvModel host_drv;      // the configured environment's device tables
  PeModel host_pe;
  const void* host_model = nullptr;
  size_t model_bytes = 0;
  pomcp_merged_root* merged = nullptr;   // [B] device results of pomcp_merge_roots
  double* gather = nullptr;              // [gather_world][B][R] pomcp_root_gather_buffer
  int gather_world = 0;
  int search_kind = POMCP_SEARCH_AUTO;
  TmTables host_tm{};                    // type-based contexts (pomcp_set_type_policies)
  bool tm_set = false;
  // a lane search with deferred cut-off records ran since the last update /
  // reset / restore: the mode and the kernel stay fixed until the re-root
  // materialises those children (a record's absorbing flag must not race an
  // eager arrival's, mcts.py:370)
  bool defer_pending = false;
  // the re-root's log scan: the streaming kernels (k_log_filter + the
  // materialising pass) unless POMCP_LOG_SCAN=legacy (one workgroup per log,
  // k_compact_log: A/B and fallback); the look-back tags' epoch
  bool log_scan_legacy = false;
  bool lf_packed_cmap = true;   // POMCP_LF_PACKED_CMAP=off: tests only
  uint32_t lf_epoch = 0;
  int lf_grid = 0;
};

// Wave-per-tree search (k_search_lds) for batches up to this many trees: one
// tree per CU at a time, so beyond one round of 256 trees the tree-per-lane
// kernel's throughput wins (DESIGN.md §6, 65,536 simulations per tree: 256
// trees 44.7 M vs ~24 M simulations/s; 1,024 trees would run four rounds,
// ~45 M, vs 86-95 M).
constexpr int kWaveSearchMaxTrees = 256;
// and only while its per-tree scratch log stays small
constexpr int64_t kWaveSearchMaxScratch = (int64_t)4 << 30;
// step-tree producers for depth limits up to this (use_step_tree)
constexpr int kStepTreeMaxDepth = 8;


// Launch `KERNEL<Env>` for the context's environment.
#define PB_ENV_LAUNCH(ctx, KERNEL, grid, block, ...)                                          \
  do {                                                                                         \
    if ((ctx)->dp.env == POMCP_ENV_PURSUIT_EVASION)                                            \
      hipLaunchKernelGGL(KERNEL<EnvPursuitEvasion>, grid, block, 0, (ctx)->stream, __VA_ARGS__); \
    else                                                                                       \
      hipLaunchKernelGGL(KERNEL<EnvDriving>, grid, block, 0, (ctx)->stream, __VA_ARGS__);    \
  } while (0)

#define HIP_TRY(ctx, expr)                                                          \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return POMCP_E_HIP;                                                           \
    }                                                                               \
  } while (0)

static int fail(pomcp_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

static int dev_alloc(pomcp_ctx* ctx, void** out, size_t bytes) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
  if (e != hipSuccess) {
    ctx->err = "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e);
    return POMCP_E_HIP;
  }
  ctx->allocs.push_back(p);
  *out = p;
  return POMCP_OK;
}

static unsigned grid_blocks(int B) { return (unsigned)((B + kTreesPerBlock - 1) / kTreesPerBlock); }
static unsigned search_blocks(int B) { return (unsigned)((B + kTPB - 1) / kTPB); }
// Workgroup size of a search launch: one-wave workgroups while the launch has
// at most 3 waves per CU (3 such workgroups fit a CU's LDS: root cache 35 KB +
// model tables each), so a small launch's waves spread over all 256 CUs; a
// full launch uses 256-lane workgroups, one per CU.
static int search_tpb(int B) { return (B + kWave - 1) / kWave <= 3 * 256 ? kTPBSmall : kTPB; }
static int search_waves(int B) { return (B + kWave - 1) / kWave; }

extern "C" {

int32_t pomcp_abi_version(void) { return POMCP_ABI_VERSION; }

const char* pomcp_last_error(const pomcp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int pomcp_set_stream(pomcp_ctx* ctx, void* hip_stream) {
  if (!ctx) return POMCP_E_INVALID;
  if (hip_stream) {
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    ctx->stream = (hipStream_t)hip_stream;
    ctx->own_stream = false;
  }
  return POMCP_OK;
}

static int validate(const pomcp_config* c, std::string* why) {
  auto bad = [&](const char* m) {
    *why = m;
    return POMCP_E_INVALID;
  };
  if (c->abi_version != POMCP_ABI_VERSION) return bad("ABI version mismatch");
  if (c->env_id != POMCP_ENV_DRIVING && c->env_id != POMCP_ENV_PURSUIT_EVASION) {
    *why = "env_id: Driving-v1 or PursuitEvasion-v1";
    return POMCP_E_UNSUPPORTED;
  }
  if (c->num_agents != 2) { *why = "the engine's models are 2-agent"; return POMCP_E_UNSUPPORTED; }
  if (c->num_actions != (c->env_id == POMCP_ENV_DRIVING ? 5 : 4)) return bad("num_actions of the model");
  if (c->env_id == POMCP_ENV_PURSUIT_EVASION) {
    const pomcp_pe_grid& g = c->pe_grid;
    if (g.width < 1 || g.width > 16 || g.height < 1 || g.height > 16) return bad("pe grid size");
    if (g.n_evader_start < 1 || g.n_evader_start > 4 || g.n_pursuer_start < 1 ||
        g.n_pursuer_start > 4 || g.n_goal < 1 || g.n_goal > 4)
      return bad("pe starts / goals (1..4 each)");
    if (g.max_obs_distance < 0 || g.max_obs_distance > 15) return bad("max_obs_distance 0..15");
    if (!(g.reward_norm > 0.0)) return bad("reward_norm > 0");
  }
  if (c->ego_agent < 0 || c->ego_agent >= c->num_agents) return bad("ego_agent out of range");
  if (c->num_actions < 1 || c->num_actions > POMCP_MAX_ACTIONS) return bad("num_actions");
  if (c->action_selection < 0 || c->action_selection > 2) return bad("action_selection");
  if (!(c->discount >= 0.0 && c->discount <= 1.0)) return bad("discount in [0,1]");
  if (!(c->c > 0.0)) return bad("c > 0");
  if (!(c->pucb_exploration_fraction >= 0.0 && c->pucb_exploration_fraction <= 1.0))
    return bad("pucb_exploration_fraction in [0,1]");
  if (!(c->reinvigoration_sample_limit_factor >= 1.0)) return bad("sample_limit_factor >= 1");
  if (c->depth_limit < 0 || c->step_limit < 0) return bad("depth/step limit");
  if (c->num_particles < 1 || c->extra_particles < 0) return bad("num_particles");
  if (c->num_trees < 1) return bad("num_trees >= 1");
  if (c->type_based != 0 && c->type_based != 1) return bad("type_based is 0 or 1");
  if (c->max_blocks < 1 || c->max_blocks * blk_lines(c->num_actions, c->type_based) * 128 > INT32_MAX)
    return bad("max_blocks");
  if (c->num_actions < 2 || c->num_actions > kMaxA) { *why = "the search kernel supports 2 to 5 actions"; return POMCP_E_UNSUPPORTED; }
  if (c->max_particles < 1 || c->max_particles * kWave > UINT32_MAX) return bad("max_particles");
  // ids: inline slots (max_blocks * A * 6), overflow entries, deferred records
  // (max_blocks * A, pomcp_device.h)
  if (c->max_blocks * c->num_actions * (kSlots + 1) + 1 + c->overflow_slots >= (int64_t)kIdMask)
    return bad("obs node ids exceed 2^26 (max_blocks * A * 7 + overflow_slots)");
  // max_belief: the root belief region (the root belief and the next, one from
  // each end: pomcp_device.h bel_at)
  if (c->max_belief < 2 * (c->num_particles + c->extra_particles)) return bad("max_belief too small");
  if (c->max_belief > INT32_MAX) return bad("max_belief < 2^31");
  if (c->overflow_slots < kBucket || (c->overflow_slots & (c->overflow_slots - 1)) != 0 ||
      c->overflow_slots > (1ll << 28))
    return bad("overflow_slots must be a power of two in [16, 2^28]");
  if (!c->log_table || c->log_table_size < 2) return bad("log_table");
  if (!c->discount_pow || c->discount_pow_size < 1) return bad("discount_pow");
  if (c->env_id != POMCP_ENV_DRIVING) return POMCP_OK;
  const pomcp_grid& g = c->grid;
  if (g.width < 1 || g.width > 16 || g.height < 1 || g.height > 16) return bad("grid size");
  if (g.num_locs < 2 || g.num_locs > 8) return bad("grid locations");
  const int ncells = (g.obs_front + g.obs_back + 1) * (2 * g.obs_side + 1);
  if (g.obs_front < 0 || g.obs_back < 0 || g.obs_side < 0 || ncells > 15)
    return bad("obs window must have <= 15 cells");
  return POMCP_OK;
}

int pomcp_create(const pomcp_config* cfg, int32_t device, void* hip_stream, pomcp_ctx** out) {
  if (!cfg || !out) return POMCP_E_INVALID;
  *out = nullptr;
  auto* ctx = new pomcp_ctx();
  ctx->cfg = *cfg;
  std::string why;
  int rc = validate(cfg, &why);
  if (rc != POMCP_OK) {
    std::fprintf(stderr, "pomcp_create: %s\n", why.c_str());
    delete ctx;
    return rc;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
    delete ctx;
    return POMCP_E_NO_DEVICE;
  }
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete ctx;
    return POMCP_E_NO_DEVICE;
  }
  if (hip_stream) {
    ctx->stream = (hipStream_t)hip_stream;
  } else {
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
      delete ctx;
      return POMCP_E_HIP;
    }
    ctx->own_stream = true;
  }
  const pomcp_config& c = *cfg;
  DevParams& d = ctx->dp;
  d.env = c.env_id;
  if (c.env_id == POMCP_ENV_PURSUIT_EVASION) {
    build_pe_model(c.pe_grid, &ctx->host_pe);
    ctx->host_model = &ctx->host_pe;
    ctx->model_bytes = sizeof(PeModel);
  } else {
    make_model(&c.grid, &ctx->host_drv);
    ctx->host_model = &ctx->host_drv;
    ctx->model_bytes = sizeof(DrvModel);
  }
  d.B = c.num_trees;
  d.A = c.num_actions;
  d.ego = c.ego_agent;
  d.other = 1 - c.ego_agent;
  d.sel = c.action_selection;
  d.depth_limit = c.depth_limit;
  d.step_limit = c.step_limit;
  d.n_target = c.num_particles + c.extra_particles;
  d.has_kb = c.has_known_bounds;
  d.ncells = (c.grid.obs_front + c.grid.obs_back + 1) * (2 * c.grid.obs_side + 1);
  d.discount = c.discount;
  d.c = c.c;
  d.pucb_f = c.pucb_exploration_fraction;
  d.limit_factor = c.reinvigoration_sample_limit_factor;
  d.kb_min = c.known_min;
  d.kb_max = c.known_max;
  d.Nb = c.max_blocks;
  d.Np = c.max_particles;
  d.Nr = c.max_belief;
  d.H = c.overflow_slots;
  d.bucket_mask = (uint32_t)(c.overflow_slots / kBucket - 1);
  d.ovf_base = (uint32_t)(c.max_blocks * c.num_actions * kSlots + 1);
  d.cut_base = d.ovf_base + (uint32_t)c.overflow_slots;
  d.defer = 1;   // deferred cut-off records (pomcp_set_defer_cutoff)
  d.sel_margin = 1e-12;   // fast-selection margin (pomcp_debug_set_select_margin)
  d.islots = kSlots;
  d.tm = c.type_based;
  d.lines = blk_lines(d.A, d.tm);
  const int64_t B = c.num_trees;
  void* p;
#define ALLOC(field, type, count)                                               \
  do {                                                                          \
    if ((rc = dev_alloc(ctx, &p, sizeof(type) * (size_t)(count))) != POMCP_OK) {\
      pomcp_destroy(ctx);                                                       \
      return rc;                                                                \
    }                                                                           \
    d.field = reinterpret_cast<decltype(d.field)>(p);                           \
  } while (0)
  ALLOC(hdr, TreeHdr, B);
  ALLOC(an, Line, arena_lines((int)B, d.Nb, d.lines));   // interleaved by search wave
  ALLOC(ovf, OvfSlot, B * d.H);
  // pomcp_device.h WaveLog: 3 u32 arrays per search wave (+ aux when type-based)
  ALLOC(plog, uint32_t, (int64_t)search_waves((int)B) * kWave * d.Np * (3 + d.tm));
  if (d.tm) ALLOC(tmt, TmTables, 1);
  ALLOC(wlog, uint32_t, search_waves((int)B));
  ALLOC(want, uint32_t, B);
  ALLOC(want_info, int4, B);
  ALLOC(cnt, int32_t, B);
  ALLOC(belief, uint4, B * d.Nr);
  ALLOC(path, uint4, B * 3 * kMaxPath);
  ALLOC(logtab, double, c.log_table_size);
  ALLOC(dpow, double, c.discount_pow_size);
  ALLOC(model, uint8_t, ctx->model_bytes);
  ALLOC(stats, pomcp_root_stats, B);
  ALLOC(merge, double, B * POMCP_XREC(d.A));
  ALLOC(upd_out, int32_t, B * 2);
  ALLOC(in_actions, int32_t, B);
  ALLOC(in_obs, uint64_t, B);
  ALLOC(out_obs, uint64_t, B);
#undef ALLOC
  if ((rc = dev_alloc(ctx, &p, sizeof(pomcp_merged_root) * (size_t)B)) != POMCP_OK) {
    pomcp_destroy(ctx);
    return rc;
  }
  ctx->merged = reinterpret_cast<pomcp_merged_root*>(p);
  d.logtab_n = c.log_table_size;
  d.dpow_n = (int32_t)(c.discount_pow_size > INT32_MAX ? INT32_MAX : c.discount_pow_size);
  hipStream_t s = ctx->stream;
  // zero: hash epoch 0 is never valid, headers start empty
  if (hipMemsetAsync(d.ovf, 0, sizeof(OvfSlot) * (size_t)(B * d.H), s) != hipSuccess ||
      hipMemsetAsync(d.hdr, 0, sizeof(TreeHdr) * (size_t)B, s) != hipSuccess ||
      hipMemsetAsync(d.stats, 0, sizeof(pomcp_root_stats) * (size_t)B, s) != hipSuccess ||
      hipMemcpyAsync((void*)d.logtab, c.log_table, sizeof(double) * c.log_table_size,
                     hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync((void*)d.dpow, c.discount_pow, sizeof(double) * c.discount_pow_size,
                     hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync((void*)d.model, ctx->host_model, ctx->model_bytes, hipMemcpyHostToDevice,
                     s) != hipSuccess) {
    ctx->err = "initial upload failed";
    pomcp_destroy(ctx);
    return POMCP_E_HIP;
  }
  // headers: keys and counters
  std::vector<TreeHdr> h((size_t)B);
  for (int64_t t = 0; t < B; ++t) {
    std::memset(&h[t], 0, sizeof(TreeHdr));
    h[t].seed = c.seed;
    h[t].tree_key = c.tree_key_base + (uint32_t)t;
  }
  // same stream as the zeroing memset above (the engine stream is non-blocking:
  // a null-stream copy would not be ordered after it)
  if (hipMemcpyAsync(d.hdr, h.data(), sizeof(TreeHdr) * (size_t)B, hipMemcpyHostToDevice, s) !=
      hipSuccess) {
    ctx->err = "header upload failed";
    pomcp_destroy(ctx);
    return POMCP_E_HIP;
  }
  ctx->host_upd.resize((size_t)(2 * B));
  ctx->host_stats.resize((size_t)B);
  // tables and headers were copied asynchronously from caller / local memory:
  // finish before returning
  if (hipStreamSynchronize(s) != hipSuccess) {
    pomcp_destroy(ctx);
    return POMCP_E_HIP;
  }
  rc = pomcp_reset(ctx);
  if (rc != POMCP_OK) {
    pomcp_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return POMCP_OK;
}

void pomcp_destroy(pomcp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (void* p : ctx->allocs) (void)hipFree(p);
  if (ctx->snap_hdr) (void)hipFree(ctx->snap_hdr);
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int pomcp_reset(pomcp_ctx* ctx) {
  if (!ctx) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_reset, dim3(grid_blocks(ctx->dp.B)), dim3(256), 0, ctx->stream, ctx->dp);
  HIP_TRY(ctx, hipGetLastError());
  ctx->have_snapshot = false;
  ctx->defer_pending = false;
  return POMCP_OK;
}

static int first_tree_error(pomcp_ctx* ctx, const int32_t* codes, int stride, int off,
                            const char* what) {
  for (int t = 0; t < ctx->dp.B; ++t) {
    const int e = codes[(size_t)t * stride + off];
    if (e != 0) {
      const char* kind = e == POMCP_E_ARENA ? "arena capacity exceeded"
                         : e == POMCP_E_NOT_FOUND ? "root has no child node for action"
                         : e == POMCP_E_STATE ? "call out of order"
                         : e == POMCP_E_INVALID ? "invalid observation"
                                                : "error";
      return fail(ctx, e, std::string(what) + ": tree " + std::to_string(t) + ": " + kind);
    }
  }
  return POMCP_OK;
}

// Scratch of the subtree compaction (k_compact), allocated on the first
// re-root: a batch that is only ever searched from its initial update (the
// bench's restore loop) never pays for it.
static int ensure_compaction_scratch(pomcp_ctx* ctx) {
  DevParams& d = ctx->dp;
  if (d.cmap) return POMCP_OK;
  const int64_t B = d.B;
  void* p = nullptr;
  int rc;
  if ((rc = dev_alloc(ctx, &p, sizeof(int32_t) * (size_t)(B * d.Nb))) != POMCP_OK) return rc;
  d.cmap = reinterpret_cast<int32_t*>(p);
  if ((rc = dev_alloc(ctx, &p, sizeof(int32_t) * (size_t)(B * d.Nb))) != POMCP_OK) return rc;
  d.cpar = reinterpret_cast<int32_t*>(p);
  if ((rc = dev_alloc(ctx, &p, sizeof(int32_t) * (size_t)(B * d.H))) != POMCP_OK) return rc;
  d.ovf_new = reinterpret_cast<int32_t*>(p);
  if ((rc = dev_alloc(ctx, &p, sizeof(OvfSlot) * (size_t)(B * d.H))) != POMCP_OK) return rc;
  d.ovf_tmp = reinterpret_cast<OvfSlot*>(p);
  if ((rc = dev_alloc(ctx, &p, sizeof(uint4) * (size_t)B)) != POMCP_OK) return rc;
  d.scan_info = reinterpret_cast<uint4*>(p);
  // the streaming scan's look-back records: every wave log's capacity in
  // segments; zeroed (tag epoch 0 is never current)
  const int waves = search_waves((int)B);
  d.lf_nseg = (int32_t)((kWave * d.Np + kLfSeg - 1) / kLfSeg);
  const size_t nd = sizeof(LfDesc) * (size_t)waves * (size_t)((d.lf_nseg + kLfChunk - 1) / kLfChunk);
  if ((rc = dev_alloc(ctx, &p, nd)) != POMCP_OK) return rc;
  d.lf_desc = reinterpret_cast<LfDesc*>(p);
  if ((rc = dev_alloc(ctx, &p, 2 * sizeof(uint32_t))) != POMCP_OK) return rc;
  d.lf_fail = reinterpret_cast<uint32_t*>(p);
  if ((rc = dev_alloc(ctx, &p, sizeof(int16_t) * (size_t)waves * kCm16)) != POMCP_OK) return rc;
  d.cm16 = reinterpret_cast<int16_t*>(p);
  if ((rc = dev_alloc(ctx, &p, sizeof(int32_t) * (size_t)waves * kCm16Off)) != POMCP_OK) return rc;
  d.cm16_off = reinterpret_cast<int32_t*>(p);
  HIP_TRY(ctx, hipMemsetAsync(d.lf_desc, 0, nd, ctx->stream));
  ctx->lf_epoch = 0;
  const char* ls = std::getenv("POMCP_LOG_SCAN");
  ctx->log_scan_legacy = ls != nullptr && std::string(ls) == "legacy";
  // tests only: the filter classifies from the global block maps (the path of
  // logs whose 64 trees' maps do not fit the packed table)
  const char* pk = std::getenv("POMCP_LF_PACKED_CMAP");
  ctx->lf_packed_cmap = !(pk != nullptr && std::string(pk) == "off");
  // the persistent grid: as many workgroups as are resident at once
  int per_cu = 0, ncu = 0;
  HIP_TRY(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(
                   &per_cu, reinterpret_cast<const void*>(d.env == POMCP_ENV_PURSUIT_EVASION
                                                              ? &k_log_filter<EnvPursuitEvasion>
                                                              : &k_log_filter<EnvDriving>),
                   kLfThreads, 0));
  HIP_TRY(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
  ctx->lf_grid = (per_cu > 0 ? per_cu : 1) * (ncu > 0 ? ncu : 1);
  return POMCP_OK;
}

int pomcp_update(pomcp_ctx* ctx, const int32_t* actions, const uint64_t* obs_keys,
                 int32_t* root_absorbing_out) {
  if (!ctx || !obs_keys) return POMCP_E_INVALID;
  if (ctx->dp.tm && !ctx->tm_set) return fail(ctx, POMCP_E_STATE, "update: pomcp_set_type_policies first");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int B = ctx->dp.B;
  std::vector<int32_t> acts((size_t)B, -1);
  if (actions) std::memcpy(acts.data(), actions, sizeof(int32_t) * (size_t)B);
  HIP_TRY(ctx, hipMemcpyAsync((void*)ctx->dp.in_actions, acts.data(), sizeof(int32_t) * B,
                              hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync((void*)ctx->dp.in_obs, obs_keys, sizeof(uint64_t) * B,
                              hipMemcpyHostToDevice, ctx->stream));
  // re-root: child lookup per tree; subtree compaction to the child's subtree
  // (re-roots only: an initial update leaves an empty arena) with one ordered
  // scan of each search wave's log that also extracts the child's particles;
  // then the per-tree update (initial belief / new root + reinvigoration)
  PB_ENV_LAUNCH(ctx, k_reroot_child, dim3(grid_blocks(B)), dim3(256), ctx->dp);
  HIP_TRY(ctx, hipGetLastError());
  bool reroot = false;
  for (int t = 0; t < B && !reroot; ++t) reroot = acts[t] >= 0;
  if (reroot) {
    int rc = ensure_compaction_scratch(ctx);
    if (rc != POMCP_OK) return rc;
    hipLaunchKernelGGL(k_compact, dim3(grid_blocks(B)), dim3(256), 0, ctx->stream, ctx->dp);
    HIP_TRY(ctx, hipGetLastError());
    if (ctx->log_scan_legacy) {
      PB_ENV_LAUNCH(ctx, k_compact_log, dim3((unsigned)search_waves(B)), dim3(64 * kLogWaves),
                    ctx->dp);
    } else {
      // the streaming scan: the filter over every log's segments, then the
      // materialising pass over the kept records
      if (++ctx->lf_epoch >= (1u << 30)) {   // (tags hold 30 bits: start over on zeroed records)
        HIP_TRY(ctx, hipMemsetAsync(ctx->dp.lf_desc, 0,
                                    sizeof(LfDesc) * (size_t)search_waves(B) *
                                        (size_t)((ctx->dp.lf_nseg + kLfChunk - 1) / kLfChunk),
                                    ctx->stream));
        ctx->lf_epoch = 1;
      }
      ctx->dp.lf_epoch = ctx->lf_epoch;
      HIP_TRY(ctx, hipMemsetAsync(ctx->dp.lf_fail, 0, 2 * sizeof(uint32_t), ctx->stream));
      hipLaunchKernelGGL(k_pack_cmap, dim3((unsigned)search_waves(B)), dim3(256), 0, ctx->stream, ctx->dp,
                         ctx->lf_packed_cmap ? 1 : 0);
      HIP_TRY(ctx, hipGetLastError());
      PB_ENV_LAUNCH(ctx, k_log_filter, dim3((unsigned)ctx->lf_grid), dim3(kLfThreads), ctx->dp,
                    search_waves(B));
      HIP_TRY(ctx, hipGetLastError());
      if (ctx->dp.env == POMCP_ENV_PURSUIT_EVASION)
        hipLaunchKernelGGL((k_compact_log<EnvPursuitEvasion, true>), dim3((unsigned)search_waves(B)),
                           dim3(64 * kMatWaves), 0, ctx->stream, ctx->dp);
      else
        hipLaunchKernelGGL((k_compact_log<EnvDriving, true>), dim3((unsigned)search_waves(B)),
                           dim3(64 * kMatWaves), 0, ctx->stream, ctx->dp);
    }
    HIP_TRY(ctx, hipGetLastError());
  }
  PB_ENV_LAUNCH(ctx, k_update, dim3(grid_blocks(B)), dim3(256), ctx->dp);
  HIP_TRY(ctx, hipGetLastError());
  HIP_TRY(ctx, hipMemcpyAsync(ctx->host_upd.data(), ctx->dp.upd_out, sizeof(int32_t) * 2 * B,
                              hipMemcpyDeviceToHost, ctx->stream));
  uint32_t lf_fail = 0u;
  if (reroot && !ctx->log_scan_legacy)
    HIP_TRY(ctx, hipMemcpyAsync(&lf_fail, ctx->dp.lf_fail, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (lf_fail != 0u) return fail(ctx, POMCP_E_HIP, "update: the log scan's look-back gave up");
  ctx->defer_pending = false;   // k_compact_log materialised the surviving deferred children
  if (root_absorbing_out)
    for (int t = 0; t < B; ++t) root_absorbing_out[t] = ctx->host_upd[2 * t];
  return first_tree_error(ctx, ctx->host_upd.data(), 2, 1, "update");
}

static bool wave_search_fits(const pomcp_ctx* ctx) {
  return ctx->dp.A <= kMaxA &&
         (int64_t)ctx->dp.B * ctx->dp.Np * (int64_t)sizeof(LogRec) <= kWaveSearchMaxScratch;
}

static int resolve_search_kind(const pomcp_ctx* ctx) {
  if (ctx->dp.tm) return POMCP_SEARCH_LANE;   // the type-based search is k_search<..., TM = 1>
  if (ctx->search_kind == POMCP_SEARCH_WAVE) return POMCP_SEARCH_WAVE;
  if (ctx->search_kind == POMCP_SEARCH_LANE) return POMCP_SEARCH_LANE;
  return ctx->dp.B <= kWaveSearchMaxTrees && wave_search_fits(ctx) ? POMCP_SEARCH_WAVE
                                                                   : POMCP_SEARCH_LANE;
}

int pomcp_set_search_kernel(pomcp_ctx* ctx, int32_t kind) {
  if (!ctx || kind < POMCP_SEARCH_AUTO || kind > POMCP_SEARCH_WAVE) return POMCP_E_INVALID;
  if (kind == POMCP_SEARCH_WAVE && !wave_search_fits(ctx))
    return fail(ctx, POMCP_E_UNSUPPORTED, "set_search_kernel: wave search scratch too large");
  if (kind == POMCP_SEARCH_WAVE && ctx->dp.tm)
    return fail(ctx, POMCP_E_UNSUPPORTED, "set_search_kernel: the type-based search is lane-per-tree");
  if (ctx->defer_pending) {
    const int was = ctx->search_kind;
    ctx->search_kind = kind;
    const bool same = resolve_search_kind(ctx) == POMCP_SEARCH_LANE;
    ctx->search_kind = was;
    if (!same)
      return fail(ctx, POMCP_E_STATE, "set_search_kernel: deferred cut-off records are pending "
                                      "(update, reset or restore first)");
  }
  ctx->search_kind = kind;
  return POMCP_OK;
}

int32_t pomcp_search_kernel_used(const pomcp_ctx* ctx) {
  return ctx ? resolve_search_kind(ctx) : POMCP_E_INVALID;
}

int pomcp_set_defer_cutoff(pomcp_ctx* ctx, int32_t on) {
  if (!ctx || (on != 0 && on != 1)) return POMCP_E_INVALID;
  if (ctx->defer_pending && on != ctx->dp.defer)
    return fail(ctx, POMCP_E_STATE, "set_defer_cutoff: deferred cut-off records are pending "
                                    "(update, reset or restore first)");
  ctx->dp.defer = on;
  return POMCP_OK;
}

// The wave search with step-tree producer waves (pomcp_search_lds.hip) when
// simulations are short enough that the producers' prediction of their draws
// (depth_limit + 1 words per simulation) mostly holds and the first three
// levels are most of a simulation; POMCP_STEP_TREE=0/1 forces it off / on.
static bool use_step_tree(const pomcp_ctx* ctx) {
  const char* f = std::getenv("POMCP_STEP_TREE");
  if (f != nullptr && f[0] != '\0') return f[0] != '0';
  return ctx->dp.depth_limit <= kStepTreeMaxDepth;
}

static int launch_search_wave(pomcp_ctx* ctx, int32_t num_sims, int final_sel) {
  if (!ctx->dp.lscr) {   // the per-tree scratch log, on first use
    void* q = nullptr;
    int rc = dev_alloc(ctx, &q, sizeof(LogRec) * (size_t)ctx->dp.B * (size_t)ctx->dp.Np);
    if (rc != POMCP_OK) return rc;
    ctx->dp.lscr = reinterpret_cast<LogRec*>(q);
  }
  using KFn = void (*)(DevParams, int, int);
#define PB_LDS_ROW(NP)                                                                          \
  {{k_search_lds<EnvDriving, POMCP_SEL_PUCB, 5, NP>, k_search_lds<EnvDriving, POMCP_SEL_UCB, 5, NP>, \
    k_search_lds<EnvDriving, POMCP_SEL_UNIFORM, 5, NP>},                                         \
   {k_search_lds<EnvPursuitEvasion, POMCP_SEL_PUCB, 4, NP>,                                      \
    k_search_lds<EnvPursuitEvasion, POMCP_SEL_UCB, 4, NP>,                                       \
    k_search_lds<EnvPursuitEvasion, POMCP_SEL_UNIFORM, 4, NP>}}
  static const KFn table[2][2][3] = {PB_LDS_ROW(0), PB_LDS_ROW(kSpecProducers)};
#undef PB_LDS_ROW
  const int e = ctx->dp.env == POMCP_ENV_PURSUIT_EVASION ? 1 : 0;
  const int spec = use_step_tree(ctx) ? 1 : 0;
  hipLaunchKernelGGL(table[spec][e][ctx->dp.sel], dim3((unsigned)ctx->dp.B),
                     dim3((unsigned)(kWave * (1 + spec * kSpecProducers))), 0, ctx->stream, ctx->dp,
                     (int)num_sims, final_sel);
  HIP_TRY(ctx, hipGetLastError());
  const int nsw = search_waves(ctx->dp.B);
  hipLaunchKernelGGL(k_log_merge, dim3((unsigned)(ctx->dp.B < kWave ? ctx->dp.B : kWave), (unsigned)nsw),
                     dim3(256), 0, ctx->stream, ctx->dp);
  HIP_TRY(ctx, hipGetLastError());
  hipLaunchKernelGGL(k_log_merge_end, dim3((unsigned)((nsw + 63) / 64)), dim3(64), 0, ctx->stream,
                     ctx->dp, nsw);
  HIP_TRY(ctx, hipGetLastError());
  return POMCP_OK;
}

static int launch_search(pomcp_ctx* ctx, int32_t num_sims, int final_sel) {
  if (!ctx || num_sims < 0) return POMCP_E_INVALID;
  if (ctx->dp.tm && !ctx->tm_set) return fail(ctx, POMCP_E_STATE, "search: pomcp_set_type_policies first");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  if (resolve_search_kind(ctx) == POMCP_SEARCH_WAVE) return launch_search_wave(ctx, num_sims, final_sel);
  const int tpb = search_tpb(ctx->dp.B);
  const dim3 grid((unsigned)((ctx->dp.B + tpb - 1) / tpb)), block((unsigned)tpb);
  // kernel per (environment, selection rule, workgroup size); the action count is the model's
  const int e = ctx->dp.env == POMCP_ENV_PURSUIT_EVASION ? 1 : 0;
  const int row = (ctx->dp.tm ? 2 : 0) + (tpb == kTPB ? 0 : 1);
  int sims = (int)num_sims, fsel = final_sel;
  void* args[] = {&ctx->dp, &sims, &fsel};
  HIP_TRY(ctx, hipLaunchKernel(pb_search_kernel(row, e, ctx->dp.sel), grid, block, args, 0, ctx->stream));
  HIP_TRY(ctx, hipGetLastError());
  if (ctx->dp.defer && !ctx->dp.tm && num_sims > 0) ctx->defer_pending = true;
  return POMCP_OK;
}

int pomcp_search(pomcp_ctx* ctx, int32_t num_sims, int32_t* actions_out) {
  int rc = launch_search(ctx, num_sims, 1);
  if (rc != POMCP_OK || !actions_out) return rc;
  rc = pomcp_get_root_stats(ctx, ctx->host_stats.data());
  if (rc != POMCP_OK) return rc;
  for (int t = 0; t < ctx->dp.B; ++t) actions_out[t] = ctx->host_stats[t].action;
  return POMCP_OK;
}

int pomcp_search_continue(pomcp_ctx* ctx, int32_t num_sims) { return launch_search(ctx, num_sims, 0); }

int pomcp_get_root_stats(pomcp_ctx* ctx, pomcp_root_stats* out) {
  if (!ctx || !out) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipMemcpyAsync(out, ctx->dp.stats, sizeof(pomcp_root_stats) * ctx->dp.B,
                              hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (int t = 0; t < ctx->dp.B; ++t)
    if (out[t].error != 0) {
      std::vector<int32_t> codes((size_t)ctx->dp.B);
      for (int k = 0; k < ctx->dp.B; ++k) codes[k] = out[k].error;
      return first_tree_error(ctx, codes.data(), 1, 0, "search");
    }
  return POMCP_OK;
}

int pomcp_set_root_belief(pomcp_ctx* ctx, int32_t tree, const uint32_t* particles, int32_t count) {
  if (!ctx || tree < 0 || tree >= ctx->dp.B || count < 1 || !particles)
    return fail(ctx, POMCP_E_INVALID, "set_root_belief: bad arguments");
  if (ctx->dp.tm)
    return fail(ctx, POMCP_E_UNSUPPORTED, "set_root_belief: type-based particles carry a policy");
  if (count > ctx->dp.Nr / 2)   // (the next belief needs room too: half the region)
    return fail(ctx, POMCP_E_ARENA, "set_root_belief: more particles than max_belief / 2");
  const uint32_t t = particles[0];
  for (int32_t i = 0; i < count; ++i)
    if (particles[3 * i] != t || t < 1u)
      return fail(ctx, POMCP_E_INVALID, "set_root_belief: every particle needs the same t >= 1");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  TreeHdr h;
  HIP_TRY(ctx, hipMemcpyAsync(&h, ctx->dp.hdr + tree, sizeof(TreeHdr), hipMemcpyDeviceToHost,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (h.root_t != 0 || h.n_blocks != 0 || h.error != 0)
    return fail(ctx, POMCP_E_STATE, "set_root_belief: the tree must be fresh (pomcp_reset)");
  // the region's records [at, at + count) in memory order (bel_at: the end of
  // the region, reversed, when the belief grows from there)
  const int sel = h.belief_sel ^ 1;
  const int64_t at = sel ? ctx->dp.Nr - count : 0;
  std::vector<uint4> b((size_t)count);
  for (int32_t i = 0; i < count; ++i)
    b[bel_at(sel, ctx->dp.Nr, i) - at] =
        make_uint4(particles[3 * i], particles[3 * i + 1], particles[3 * i + 2], 0u);
  uint4* dst = ctx->dp.belief + (int64_t)tree * ctx->dp.Nr + at;
  HIP_TRY(ctx, hipMemcpyAsync(dst, b.data(), sizeof(uint4) * (size_t)count, hipMemcpyHostToDevice,
                              ctx->stream));
  h.belief_sel = sel;
  h.belief_size = count;
  h.root_t = (int32_t)t;
  h.root_id = kRootId;
  h.root_blk = -1;
  h.root_visits = 0;
  h.root_abs = 0;
  h.n_nodes += 1;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->dp.hdr + tree, &h, sizeof(TreeHdr), hipMemcpyHostToDevice,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

// The first n particles of a tree's root belief, in order (pomcp_device.h
// bel_at: a belief grown from the region's end is stored reversed)
static int read_root_belief(pomcp_ctx* ctx, int32_t tree, const TreeHdr& h, int n, uint4* out) {
  const int sel = h.belief_sel;
  const int64_t at = sel ? ctx->dp.Nr - n : 0;
  std::vector<uint4> raw((size_t)n);
  HIP_TRY(ctx, hipMemcpyAsync(raw.data(), ctx->dp.belief + (int64_t)tree * ctx->dp.Nr + at,
                              sizeof(uint4) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < n; ++i) out[i] = raw[bel_at(sel, ctx->dp.Nr, i) - at];
  return POMCP_OK;
}

int pomcp_get_root_belief(pomcp_ctx* ctx, int32_t tree, uint32_t* out, int32_t capacity,
                          int32_t* count) {
  if (!ctx || !count || tree < 0 || tree >= ctx->dp.B) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  TreeHdr h;
  HIP_TRY(ctx, hipMemcpyAsync(&h, ctx->dp.hdr + tree, sizeof(TreeHdr), hipMemcpyDeviceToHost,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  *count = h.belief_size;
  if (!out || capacity <= 0) return POMCP_OK;
  const int n = h.belief_size < capacity ? h.belief_size : capacity;
  std::vector<uint4> tmp((size_t)n);
  if (n > 0) {
    int rc = read_root_belief(ctx, tree, h, n, tmp.data());
    if (rc != POMCP_OK) return rc;
  }
  for (int i = 0; i < n; ++i) {
    out[3 * i + 0] = tmp[i].x;
    out[3 * i + 1] = tmp[i].y;
    out[3 * i + 2] = tmp[i].z;
  }
  return POMCP_OK;
}

int pomcp_set_type_policies(pomcp_ctx* ctx, const pomcp_type_policies* tp) {
  if (!ctx || !tp) return POMCP_E_INVALID;
  if (!ctx->dp.tm) return fail(ctx, POMCP_E_STATE, "set_type_policies: context is not type_based");
  const int A = ctx->dp.A, ne = tp->num_ego, no = tp->num_other;
  if (ne < 1 || ne > kTmMax || no < 1 || no > kTmMax)
    return fail(ctx, POMCP_E_INVALID, "set_type_policies: 1..8 ego and other-agent policies");
  TmTables t{};
  t.n_ego = ne;
  t.n_other = no;
  t.no_meta_draw = tp->no_meta_draw != 0;
  t.no_mixture_draw = tp->no_mixture_draw != 0;
  t.ego_uniform = tp->ego_uniform != 0;
  t.other_uniform = tp->other_uniform != 0;
  if (t.no_mixture_draw && no != 1)
    return fail(ctx, POMCP_E_INVALID, "set_type_policies: no_mixture_draw needs one other-agent policy");
  // random.choices' cumulative weights (itertools.accumulate) and total = cum[-1] + 0.0
  auto cum = [](const double* w, int n, double* c, double* total) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
      acc = i == 0 ? w[i] : acc + w[i];
      c[i] = acc;
    }
    *total = acc + 0.0;
  };
  for (int a = 0; a < A; ++a) t.prior[0][a] = tp->expected_prior[a];
  for (int k = 0; k < ne; ++k) {
    for (int a = 0; a < A; ++a) {
      if (!(tp->ego_pi[k][a] >= 0.0)) return fail(ctx, POMCP_E_INVALID, "set_type_policies: ego_pi < 0");
      t.prior[k + 1][a] = tp->ego_pi[k][a];
    }
    cum(tp->ego_pi[k], A, t.ego_cum[k], &t.ego_tot[k]);
    if (!(t.ego_tot[k] > 0.0)) return fail(ctx, POMCP_E_INVALID, "set_type_policies: ego_pi sums to 0");
  }
  for (int j = 0; j < no; ++j) {
    for (int a = 0; a < A; ++a)
      if (!(tp->other_pi[j][a] >= 0.0)) return fail(ctx, POMCP_E_INVALID, "set_type_policies: other_pi < 0");
    cum(tp->other_pi[j], A, t.oth_cum[j], &t.oth_tot[j]);
    if (!(t.oth_tot[j] > 0.0)) return fail(ctx, POMCP_E_INVALID, "set_type_policies: other_pi sums to 0");
    const int m = tp->meta_len[j];
    if (m < 1 || m > kTmMax) return fail(ctx, POMCP_E_INVALID, "set_type_policies: meta_len 1..8");
    t.meta_len[j] = m;
    for (int i = 0; i < m; ++i) {
      const int k = tp->meta_policy[j][i];
      if (k < 0 || k >= ne) return fail(ctx, POMCP_E_INVALID, "set_type_policies: meta_policy index");
      t.meta_idx[j][i] = k;
    }
    cum(tp->meta_weight[j], m, t.meta_cum[j], &t.meta_tot[j]);
  }
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  ctx->host_tm = t;
  HIP_TRY(ctx, hipMemcpyAsync(const_cast<TmTables*>(ctx->dp.tmt), &ctx->host_tm, sizeof(TmTables),
                              hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  ctx->tm_set = true;
  return POMCP_OK;
}

int pomcp_get_root_prior(pomcp_ctx* ctx, int32_t tree, double* out) {
  if (!ctx || !out || tree < 0 || tree >= ctx->dp.B) return POMCP_E_INVALID;
  if (!ctx->dp.tm) return fail(ctx, POMCP_E_STATE, "get_root_prior: context is not type_based");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  TreeHdr h;
  HIP_TRY(ctx, hipMemcpyAsync(&h, ctx->dp.hdr + tree, sizeof(TreeHdr), hipMemcpyDeviceToHost,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  const int A = ctx->dp.A;
  if (h.root_blk < 0) {   // no block yet: the prior its code names
    const int code = h.root_code >= 0 && h.root_code <= kTmMax ? h.root_code : 0;
    for (int a = 0; a < A; ++a) out[a] = ctx->host_tm.prior[code][a];
    return POMCP_OK;
  }
  const Line* blk = ctx->dp.an + tree_base_lines(tree, ctx->dp.Nb, ctx->dp.lines) +
                    (int64_t)h.root_blk * blk_stride_lines(ctx->dp.lines);
  HIP_TRY(ctx, hipMemcpyAsync(out, reinterpret_cast<const uint4*>(blk) + part_prior(A),
                              sizeof(double) * A, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

int pomcp_get_root_policies(pomcp_ctx* ctx, int32_t tree, int32_t* out, int32_t capacity,
                            int32_t* count) {
  if (!ctx || !count || tree < 0 || tree >= ctx->dp.B) return POMCP_E_INVALID;
  if (!ctx->dp.tm) return fail(ctx, POMCP_E_STATE, "get_root_policies: context is not type_based");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  TreeHdr h;
  HIP_TRY(ctx, hipMemcpyAsync(&h, ctx->dp.hdr + tree, sizeof(TreeHdr), hipMemcpyDeviceToHost,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  *count = h.belief_size;
  if (!out || capacity <= 0) return POMCP_OK;
  const int n = h.belief_size < capacity ? h.belief_size : capacity;
  std::vector<uint4> tmp((size_t)n);
  if (n > 0) {
    int rc = read_root_belief(ctx, tree, h, n, tmp.data());
    if (rc != POMCP_OK) return rc;
  }
  for (int i = 0; i < n; ++i) out[i] = (int32_t)tmp[i].w;
  return POMCP_OK;
}

int pomcp_arena_usage(pomcp_ctx* ctx, int32_t* max_blocks_used, int32_t* max_log_used) {
  if (!ctx || !max_blocks_used || !max_log_used) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  std::vector<TreeHdr> h((size_t)ctx->dp.B);
  HIP_TRY(ctx, hipMemcpyAsync(h.data(), ctx->dp.hdr, sizeof(TreeHdr) * h.size(),
                              hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  int32_t nb = 0, nl = 0;
  for (const auto& x : h) {
    nb = x.n_blocks > nb ? x.n_blocks : nb;
    nl = x.n_log > nl ? x.n_log : nl;
  }
  *max_blocks_used = nb;
  *max_log_used = nl;
  return POMCP_OK;
}

int pomcp_rekey(pomcp_ctx* ctx, uint64_t seed) {
  if (!ctx) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  std::vector<TreeHdr> h((size_t)ctx->dp.B);
  HIP_TRY(ctx, hipMemcpyAsync(h.data(), ctx->dp.hdr, sizeof(TreeHdr) * h.size(),
                              hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (auto& x : h) x.seed = seed;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->dp.hdr, h.data(), sizeof(TreeHdr) * h.size(),
                              hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

int pomcp_root_merge_buffer(pomcp_ctx* ctx, void** device_ptr) {
  if (!ctx || !device_ptr) return POMCP_E_INVALID;
  *device_ptr = ctx->dp.merge;
  return POMCP_OK;
}

int pomcp_root_gather_buffer(pomcp_ctx* ctx, int32_t world, void** device_ptr) {
  if (!ctx || !device_ptr || world < 1) return POMCP_E_INVALID;
  if (world > ctx->gather_world) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->gather) {
      for (auto& q : ctx->allocs)
        if (q == ctx->gather) q = nullptr;
      (void)hipFree(ctx->gather);
      ctx->gather = nullptr;
      ctx->gather_world = 0;
    }
    void* q = nullptr;
    const size_t bytes = sizeof(double) * (size_t)world * (size_t)ctx->dp.B * POMCP_XREC(ctx->dp.A);
    int rc = dev_alloc(ctx, &q, bytes);
    if (rc != POMCP_OK) return rc;
    HIP_TRY(ctx, hipMemsetAsync(q, 0, bytes, ctx->stream));
    ctx->gather = reinterpret_cast<double*>(q);
    ctx->gather_world = world;
  }
  *device_ptr = ctx->gather;
  return POMCP_OK;
}

// ncclAllGather of the RCCL copy already in this process (PyTorch's, or one
// the caller loaded; its soname is librccl.so.1): never a second copy, whose
// functions would be handed a communicator created by the first one.
typedef int (*pb_nccl_allgather_fn)(const void*, void*, size_t, int, void*, hipStream_t);
static pb_nccl_allgather_fn pb_rccl_allgather() {
  static pb_nccl_allgather_fn fn = nullptr;
  if (!fn) {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (h) fn = reinterpret_cast<pb_nccl_allgather_fn>(dlsym(h, "ncclAllGather"));
  }
  return fn;
}

int pomcp_allgather_root(pomcp_ctx* ctx, void* rccl_comm, int32_t world) {
  if (!ctx || !rccl_comm || world < 1) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const pb_nccl_allgather_fn allgather = pb_rccl_allgather();
  if (!allgather)
    return fail(ctx, POMCP_E_UNSUPPORTED,
                "allgather_root: no RCCL library is loaded in this process (load the one the "
                "communicator was created with first)");
  void* gbuf = nullptr;
  int rc = pomcp_root_gather_buffer(ctx, world, &gbuf);
  if (rc != POMCP_OK) return rc;
  constexpr int kNcclFloat64 = 8;   // rccl.h ncclDataType_t
  const size_t n = (size_t)ctx->dp.B * POMCP_XREC(ctx->dp.A);
  rc = allgather(ctx->dp.merge, gbuf, n, kNcclFloat64, rccl_comm, ctx->stream);
  if (rc != 0) return fail(ctx, POMCP_E_HIP, "allgather_root: ncclAllGather error " + std::to_string(rc));
  return POMCP_OK;
}

int pomcp_merge_roots(pomcp_ctx* ctx, int32_t group, int32_t world, pomcp_merged_root* out) {
  if (!ctx || group < 1 || ctx->dp.B % group != 0)
    return fail(ctx, POMCP_E_INVALID, "merge_roots: group must divide num_trees");
  if (world < 0 || (world > 0 && world > ctx->gather_world))
    return fail(ctx, POMCP_E_INVALID, "merge_roots: no gather buffer for that many ranks");
  if ((int64_t)(world > 0 ? world : 1) * group > INT32_MAX / 2)
    return fail(ctx, POMCP_E_INVALID, "merge_roots: too many replicas");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int G = ctx->dp.B / group;
  const double* src = world > 0 ? ctx->gather : ctx->dp.merge;
  hipLaunchKernelGGL(k_merge_roots, dim3((unsigned)G), dim3(kWave), 0, ctx->stream, src,
                     (int)ctx->dp.B, (int)ctx->dp.A, (int)ctx->dp.sel, (int)group,
                     world > 0 ? (int)world : 1, ctx->merged);
  HIP_TRY(ctx, hipGetLastError());
  if (!out) return POMCP_OK;
  HIP_TRY(ctx, hipMemcpyAsync(out, ctx->merged, sizeof(pomcp_merged_root) * (size_t)G,
                              hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (int g = 0; g < G; ++g)
    if (out[g].error != 0)
      return fail(ctx, out[g].error, "search: planner " + std::to_string(g) + ": replica error " +
                                         std::to_string(out[g].error));
  return POMCP_OK;
}

int pomcp_synthetic_obs(pomcp_ctx* ctx, uint64_t env_seed_base, uint64_t* obs_keys_out) {
  if (!ctx) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  PB_ENV_LAUNCH(ctx, k_synthetic_obs, dim3(grid_blocks(ctx->dp.B)), dim3(256), ctx->dp,
                env_seed_base);
  HIP_TRY(ctx, hipGetLastError());
  if (obs_keys_out) {
    HIP_TRY(ctx, hipMemcpyAsync(obs_keys_out, ctx->dp.out_obs, sizeof(uint64_t) * ctx->dp.B,
                                hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  }
  return POMCP_OK;
}

int pomcp_synthetic_step(pomcp_ctx* ctx, uint64_t env_seed_base, const int32_t* actions,
                         uint64_t* obs_keys_out) {
  if (!ctx || !actions) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int B = ctx->dp.B;
  HIP_TRY(ctx, hipMemcpyAsync((void*)ctx->dp.in_actions, actions, sizeof(int32_t) * B,
                              hipMemcpyHostToDevice, ctx->stream));
  PB_ENV_LAUNCH(ctx, k_synthetic_step, dim3(grid_blocks(B)), dim3(256), ctx->dp, env_seed_base);
  HIP_TRY(ctx, hipGetLastError());
  if (obs_keys_out) {
    HIP_TRY(ctx, hipMemcpyAsync(obs_keys_out, ctx->dp.out_obs, sizeof(uint64_t) * B,
                                hipMemcpyDeviceToHost, ctx->stream));
  }
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

int pomcp_snapshot(pomcp_ctx* ctx) {
  if (!ctx) return POMCP_E_INVALID;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int B = ctx->dp.B;
  std::vector<TreeHdr> h((size_t)B);
  HIP_TRY(ctx, hipMemcpyAsync(h.data(), ctx->dp.hdr, sizeof(TreeHdr) * B, hipMemcpyDeviceToHost,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (int t = 0; t < B; ++t) {
    // only the post-initial-update state (no blocks, no log, empty overflow map)
    // is restorable by resetting the header and bumping the map generation
    if (h[t].root_t != 1 || h[t].n_blocks != 0 || h[t].n_log != 0 || h[t].error != 0)
      return fail(ctx, POMCP_E_STATE, "snapshot: every tree must be right after its initial update");
  }
  if (!ctx->snap_hdr) HIP_TRY(ctx, hipMalloc(&ctx->snap_hdr, sizeof(TreeHdr) * B));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->snap_hdr, h.data(), sizeof(TreeHdr) * B, hipMemcpyHostToDevice,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  ctx->have_snapshot = true;
  return POMCP_OK;
}

int pomcp_restore(pomcp_ctx* ctx) {
  if (!ctx) return POMCP_E_INVALID;
  if (!ctx->have_snapshot) return fail(ctx, POMCP_E_STATE, "restore without snapshot");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_restore, dim3(grid_blocks(ctx->dp.B)), dim3(256), 0, ctx->stream, ctx->dp,
                     ctx->snap_hdr);
  HIP_TRY(ctx, hipGetLastError());
  ctx->defer_pending = false;   // back to the post-update roots: no records left
  return POMCP_OK;
}

// Debug: FP64 sqrt / div / add-mul on the device, for bit-exactness checks
// against the host (include/pomcp_debug.h).
int pomcp_debug_fp_selftest(const double* a, const double* b, int32_t n, double* out) {
  if (!a || !b || !out || n <= 0) return POMCP_E_INVALID;
  double *da = nullptr, *db = nullptr, *dout = nullptr;
  if (hipMalloc(&da, sizeof(double) * n) != hipSuccess) return POMCP_E_HIP;
  (void)hipMalloc(&db, sizeof(double) * n);
  (void)hipMalloc(&dout, sizeof(double) * 4 * n);
  (void)hipMemcpy(da, a, sizeof(double) * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, sizeof(double) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_fp_selftest, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, n, dout);
  hipError_t e = hipMemcpy(out, dout, sizeof(double) * 4 * n, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return e == hipSuccess ? POMCP_OK : POMCP_E_HIP;
}

// Debug: rcp_nr / rsq_nr (the fast UCB scores' 1/x and 1/sqrt(x)) on the
// device, for the error bound their exact fallback relies on.
int pomcp_debug_fast_recip(const double* x, int32_t n, double* out) {
  if (!x || !out || n <= 0) return POMCP_E_INVALID;
  double *dx = nullptr, *dout = nullptr;
  if (hipMalloc(&dx, sizeof(double) * n) != hipSuccess) return POMCP_E_HIP;
  if (hipMalloc(&dout, sizeof(double) * 2 * n) != hipSuccess) {
    (void)hipFree(dx);
    return POMCP_E_HIP;
  }
  (void)hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_fast_recip, dim3((n + 255) / 256), dim3(256), 0, 0, dx, n, dout);
  hipError_t e = hipMemcpy(out, dout, sizeof(double) * 2 * n, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(dout);
  return e == hipSuccess ? POMCP_OK : POMCP_E_HIP;
}

// Debug: device exp (the I-NTMCP softmax, intmcp.py:784-786) for comparison
// with the host's math.exp.
int pomcp_debug_exp(const double* x, int32_t n, double* out) {
  if (!x || !out || n <= 0) return POMCP_E_INVALID;
  double *dx = nullptr, *dout = nullptr;
  if (hipMalloc(&dx, sizeof(double) * n) != hipSuccess) return POMCP_E_HIP;
  (void)hipMalloc(&dout, sizeof(double) * n);
  (void)hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_exp_selftest, dim3((n + 255) / 256), dim3(256), 0, 0, dx, n, dout);
  hipError_t e = hipMemcpy(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(dout);
  return e == hipSuccess ? POMCP_OK : POMCP_E_HIP;
}


// Debug: k_search's fast-selection margin (pomcp_debug.h); >= 1e-12 keeps
// results exact, larger sends more selections to the exact FP64 scores
// (counted in pomcp_root_stats.n_exact_selects).
int pomcp_debug_set_select_margin(pomcp_ctx* ctx, double rel) {
  if (!ctx || !(rel >= 1e-12) || !(rel <= 1.0)) return POMCP_E_INVALID;
  ctx->dp.sel_margin = rel;
  return POMCP_OK;
}

// Debug: use only the first n (1..6) inline obs slots of every action node, so
// the overflow map serves the rest (tests of that path: the models here rarely
// give an action node more than 6 obs children).  Before the first search.
int pomcp_debug_set_inline_slots(pomcp_ctx* ctx, int32_t n) {
  if (!ctx || n < 1 || n > kSlots) return POMCP_E_INVALID;
  ctx->dp.islots = n;
  return POMCP_OK;
}

// Debug: k_search_lds's bound on waiting for a step-tree hand-off (polls; 0 =
// the default), so a test can make every hand-off late.
int pomcp_debug_set_spin_limit(pomcp_ctx* ctx, int32_t polls) {
  if (!ctx || polls < 0) return POMCP_E_INVALID;
  ctx->dp.spin_max = polls;
  return POMCP_OK;
}

// Debug: per-wave phase cycles of k_search (diagnostics build only).
int pomcp_debug_phase_timing(pomcp_ctx* ctx, uint64_t* out, int32_t capacity, int32_t* count) {
  if (!ctx || !count) return POMCP_E_INVALID;
#if !defined(POMCP_PHASE_TIMING) && !defined(PB_CLOG_TIMING)
  (void)out;
  (void)capacity;
  *count = 0;
  return POMCP_E_UNSUPPORTED;
#else
  const int64_t waves = search_waves(ctx->dp.B);
  if (ctx->dp.timing == nullptr) {   // first call: allocate; the next search fills it
    void* p = nullptr;
    if (dev_alloc(ctx, &p, sizeof(uint64_t) * 16 * (size_t)waves) != POMCP_OK) return POMCP_E_HIP;
    HIP_TRY(ctx, hipMemset(p, 0, sizeof(uint64_t) * 16 * (size_t)waves));
    ctx->dp.timing = reinterpret_cast<uint64_t*>(p);
    *count = 0;
    return POMCP_OK;
  }
  *count = (int32_t)(16 * waves);
  if (out && capacity >= *count) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipMemcpy(out, ctx->dp.timing, sizeof(uint64_t) * 16 * (size_t)waves,
                           hipMemcpyDeviceToHost));
  }
  return POMCP_OK;
#endif
}

}  // extern "C"

// I-NTMCP (include/intmcp.h)
#include "intmcp_capi.hip"
