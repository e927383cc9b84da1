// C-ABI host side of the I-NTMCP engine (include/intmcp.h).  Part of the
// single translation unit of pomcp_capi.hip.
#include <type_traits>

#include "../../include/intmcp.h"

struct intmcp_ctx {
  intmcp_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  ImParams ip{};
  std::vector<void*> allocs;
  std::string err;
  DrvModel host_drv;
  PeModel host_pe;
  const void* host_model = nullptr;
  size_t model_bytes = 0;
  std::vector<int32_t> host_out;
  std::vector<IHdr> host_hdr;
  intmcp_root_stats* dev_rstats = nullptr;   // device staging of intmcp_get_root_stats
};

// intmcp_root_stats of every pair's planner root (the level-1 root; at nesting
// level 0 the root of tree 1) (was a host loop with two synchronous copies per
// pair: seconds at 65,536 pairs)
__global__ __launch_bounds__(64) void k_im_root_stats(ImParams d, intmcp_root_stats* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= d.B) return;
  const IHdr h = d.hdr[t];
  const int T = d.nest0 ? 1 : 0;
  const char* const blk = d.nodes + im_node_off(d.Nn, d.B, t, T, h.cur, d.nt);
  const INode node = *reinterpret_cast<const INode*>(blk);
  intmcp_root_stats o;
  memset(&o, 0, sizeof(o));
  o.action = h.last_action;
  o.num_sims = h.num_sims;
  o.search_depth = h.search_depth;
  o.root_visits = node.visits;
  o.root_absorbing = im_absorbing(node.info) ? 1 : 0;
  o.belief_size = h.root_size;
  o.error = h.err;
  const int nr = im_nreg(node.info);
  o.num_children = nr;
  if (im_has_stats(node.info)) {
    const char* rv = blk + im_rec_delta(d.B, t);                   // its action records
    for (int i = 0; i < nr && i < POMCP_MAX_ACTIONS; ++i) {
      const int a = im_order(node.info, i);
      o.child_action[i] = a;
      if (a < d.A) {
        const uint32_t* hv = reinterpret_cast<const uint32_t*>(blk + kImHeads + 12 * a);   // node line
        const uint2 tot = *reinterpret_cast<const uint2*>(rv + kImRec * a);
        o.child_visits[i] = (int)hv[0];
        o.child_values[i] = hilo_d(hv[1], hv[2]);
        o.child_totals[i] = hilo_d(tot.x, tot.y);
      }
    }
  }
  o.min_value = h.mm_min[T];
  o.max_value = h.mm_max[T];
  for (int k = 0; k < 2; ++k) {   // (the first two trees; intmcp_get_tree_counts has them all)
    o.n_nodes[k] = h.n_nodes[k];
    o.n_log[k] = h.n_log[k];
    o.n_stats[k] = h.n_stats[k];
  }
  o.n_support = h.n_sup;
  out[t] = o;
}

#define IM_TRY(ctx, expr)                                                           \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return POMCP_E_HIP;                                                           \
    }                                                                               \
  } while (0)

#define IM_LAUNCH(ctx, KERNEL, grid, block, ...)                                              \
  do {                                                                                         \
    if ((ctx)->cfg.base.env_id == POMCP_ENV_PURSUIT_EVASION)                                   \
      hipLaunchKernelGGL(KERNEL<EnvPursuitEvasion>, grid, block, 0, (ctx)->stream, __VA_ARGS__); \
    else                                                                                       \
      hipLaunchKernelGGL(KERNEL<EnvDriving>, grid, block, 0, (ctx)->stream, __VA_ARGS__);    \
  } while (0)

static unsigned im_blocks(int B) { return (unsigned)((B + 63) / 64); }

static int im_alloc(intmcp_ctx* ctx, void** out, size_t bytes) {
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

template <class T>
static int im_copy(intmcp_ctx* ctx, T* dst, const T* src, size_t n) {
  if (n == 0) return POMCP_OK;
  IM_TRY(ctx, hipMemcpyAsync(dst, src, sizeof(T) * n, hipMemcpyDeviceToHost, ctx->stream));
  IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

// nodes 0..n-1 of one tree of one pair, packed as [n][kImBlock] (line, then
// the action records; the device layout interleaves them by wave:
// im_node_off, im_rec_delta)
static int im_copy_blocks(intmcp_ctx* ctx, std::vector<char>& out, int pair, int tree, int n) {
  out.resize((size_t)n * kImBlock);
  if (n == 0) return POMCP_OK;
  const char* line0 = ctx->ip.nodes + im_node_off(ctx->ip.Nn, ctx->ip.B, pair, tree, 0, ctx->ip.nt);
  const size_t ns = (size_t)im_node_stride(ctx->ip.B, pair);
  IM_TRY(ctx, hipMemcpy2DAsync(out.data(), kImBlock, line0, ns, kImLine, n, hipMemcpyDeviceToHost,
                               ctx->stream));
  IM_TRY(ctx, hipMemcpy2DAsync(out.data() + kImLine, kImBlock, line0 + im_rec_delta(ctx->ip.B, pair),
                               ns, kImRecs, n, hipMemcpyDeviceToHost, ctx->stream));
  IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

extern "C" {

// ctx == NULL: why the last intmcp_create of this thread failed
static thread_local std::string g_create_err;
const char* intmcp_last_error(const intmcp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

void intmcp_destroy(intmcp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (void* p : ctx->allocs) (void)hipFree(p);
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int intmcp_create(const intmcp_config* cfg, int32_t device, void* hip_stream, intmcp_ctx** out) {
  if (!cfg || !out) return POMCP_E_INVALID;
  *out = nullptr;
  const pomcp_config& c = cfg->base;
  auto* ctx = new intmcp_ctx();
  ctx->cfg = *cfg;
  g_create_err.clear();
  auto bad = [&](int code, const char* m) {
    g_create_err = m;
    int rc = code;
    delete ctx;
    return rc;
  };
  if (c.abi_version != POMCP_ABI_VERSION) return bad(POMCP_E_INVALID, "ABI version mismatch");
  if (c.env_id != POMCP_ENV_DRIVING && c.env_id != POMCP_ENV_PURSUIT_EVASION)
    return bad(POMCP_E_UNSUPPORTED, "env_id");
  if (c.num_agents != 2) return bad(POMCP_E_UNSUPPORTED, "2 agents");
  if (c.num_actions != (c.env_id == POMCP_ENV_DRIVING ? 5 : 4)) return bad(POMCP_E_INVALID, "num_actions");
  if (c.action_selection != POMCP_SEL_UCB && c.action_selection != POMCP_SEL_UNIFORM)
    return bad(POMCP_E_UNSUPPORTED, "I-NTMCP pucb reads self.action_space (intmcp.py:645): ucb / uniform only");
  if (c.ego_agent < 0 || c.ego_agent > 1 || c.num_trees < 1) return bad(POMCP_E_INVALID, "ego / pairs");
  if (cfg->nesting_level < 0 || cfg->nesting_level > kImMaxT - 1)
    return bad(POMCP_E_UNSUPPORTED, "nesting levels 0 to INTMCP_MAX_TREES - 1 (5)");
  if (c.depth_limit < 0 || c.step_limit < 0 || c.num_particles < 1) return bad(POMCP_E_INVALID, "limits");
  if (cfg->max_nodes < 2 || cfg->max_nodes >= (1ll << 28) || cfg->max_stats < c.num_actions ||
      cfg->max_log < 1 || cfg->hash_slots < 16 || (cfg->hash_slots & (cfg->hash_slots - 1)) ||
      cfg->hash_slots > (1ll << 31) || cfg->max_root_belief < 2 * (c.num_particles + c.extra_particles) ||
      cfg->max_support_particles < 1)
    return bad(POMCP_E_INVALID, "capacities");
  if (!c.log_table || c.log_table_size < 2 || !c.discount_pow || c.discount_pow_size < 1)
    return bad(POMCP_E_INVALID, "tables");
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
  if (c.env_id == POMCP_ENV_PURSUIT_EVASION) {
    build_pe_model(c.pe_grid, &ctx->host_pe);
    ctx->host_model = &ctx->host_pe;
    ctx->model_bytes = sizeof(PeModel);
  } else {
    std::memcpy(&ctx->host_drv.g, &c.grid, sizeof(DrvGrid));
    build_model_tables(ctx->host_drv.g, &ctx->host_drv);
    ctx->host_model = &ctx->host_drv;
    ctx->model_bytes = sizeof(DrvModel);
  }
  ImParams& d = ctx->ip;
  d.fast_slack = IM_FAST_SLACK;
  d.B = c.num_trees;
  d.A = c.num_actions;
  // nesting level 0: the planner's tree is tree 1, whose agent is p.other
  d.nest0 = cfg->nesting_level == 0 ? 1 : 0;
  d.nt = cfg->nesting_level >= 2 ? cfg->nesting_level + 1 : 2;   // a tree per level (nesting 0: 2)
  d.ego = d.nest0 ? 1 - c.ego_agent : c.ego_agent;
  d.other = 1 - d.ego;
  d.sel = c.action_selection;
  d.depth_limit = c.depth_limit;
  d.step_limit = c.step_limit;
  d.n_target = c.num_particles + c.extra_particles;
  d.extra = c.extra_particles;
  d.has_kb = c.has_known_bounds;
  d.state_belief_only = cfg->state_belief_only;
  d.discount = c.discount;
  d.c = c.c;
  d.limit_factor = c.reinvigoration_sample_limit_factor;
  d.kb_min = c.known_min;
  d.kb_max = c.known_max;
  d.Nn = cfg->max_nodes;
  d.Ns = cfg->max_stats;
  d.Nl = cfg->max_log;
  d.H = cfg->hash_slots;
  d.Nr = cfg->max_root_belief;
  d.Nsp = cfg->max_support_particles;
  const int64_t B = c.num_trees;
  int rc;
  void* p;
#define IM_ALLOC(field, type, count)                                            \
  do {                                                                          \
    if ((rc = im_alloc(ctx, &p, sizeof(type) * (size_t)(count))) != POMCP_OK) {\
      g_create_err = ctx->err;                                                  \
      intmcp_destroy(ctx);                                                      \
      return rc;                                                                \
    }                                                                           \
    d.field = reinterpret_cast<std::remove_reference_t<decltype(d.field)>>(p);  \
  } while (0)
  IM_ALLOC(hdr, IHdr, B);
  d.nstride = kImBlock;   // node blocks (intmcp.hip), interleaved by wave: im_node_off
  IM_ALLOC(nodes, char, B * d.nt * d.Nn * d.nstride);
  IM_ALLOC(hash, IHash, B * d.nt * d.H);
  IM_ALLOC(log, IRec, B * d.nt * d.Nl);
  IM_ALLOC(root, uint4, B * 2 * d.Nr);
  IM_ALLOC(sup, ISup, B * 2 * d.Nr);
  IM_ALLOC(supp, uint2, B * 2 * d.Nsp);
  for (int m = 0; m < kImMaxMid; ++m) {   // the middle planners' beliefs and distributions
    const bool mid = m < d.nt - 2;
    IM_ALLOC(msup[m], ISup, mid ? B * 2 * d.Nr : 1);
    IM_ALLOC(msupp[m], uint4, mid ? B * 2 * d.Nsp : 1);
    IM_ALLOC(mprob[m], double, mid ? B * d.Nr : 1);
  }
  IM_ALLOC(path, int4, B * kImPath * 3);
  IM_ALLOC(prob, double, B * d.Nr);
  IM_ALLOC(logtab, double, c.log_table_size);
  IM_ALLOC(dpow, double, c.discount_pow_size);
  IM_ALLOC(model, uint8_t, ctx->model_bytes);
  IM_ALLOC(in_actions, int32_t, B);
  IM_ALLOC(in_obs, uint64_t, B);
  IM_ALLOC(out, int32_t, B * 2);
  IM_ALLOC(out_obs, uint64_t, B);
#undef IM_ALLOC
  d.logtab_n = c.log_table_size;
  d.dpow_n = (int32_t)(c.discount_pow_size > INT32_MAX ? INT32_MAX : c.discount_pow_size);
  std::vector<IHdr> h((size_t)B);
  for (int64_t t = 0; t < B; ++t) {
    std::memset(&h[t], 0, sizeof(IHdr));
    h[t].seed = c.seed;
    h[t].tree_key = c.tree_key_base + (uint32_t)t;
  }
  hipStream_t s = ctx->stream;
  if (hipMemcpyAsync((void*)d.logtab, c.log_table, sizeof(double) * c.log_table_size,
                     hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync((void*)d.dpow, c.discount_pow, sizeof(double) * c.discount_pow_size,
                     hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync((void*)d.model, ctx->host_model, ctx->model_bytes, hipMemcpyHostToDevice,
                     s) != hipSuccess ||
      hipMemcpyAsync(d.hdr, h.data(), sizeof(IHdr) * (size_t)B, hipMemcpyHostToDevice, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    g_create_err = "initial upload failed";
    intmcp_destroy(ctx);
    return POMCP_E_HIP;
  }
  ctx->host_out.resize((size_t)(2 * B));
  ctx->host_hdr.resize((size_t)B);
  rc = intmcp_reset(ctx);
  if (rc != POMCP_OK) {
    g_create_err = "reset: " + ctx->err;
    intmcp_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return POMCP_OK;
}

int intmcp_reset(intmcp_ctx* ctx) {
  if (!ctx) return POMCP_E_INVALID;
  IM_TRY(ctx, hipSetDevice(ctx->device));
  // node lines and records start zeroed: statistics and inline child slots
  // need no initialising writes (intmcp.hip, kImBlock)
  IM_TRY(ctx, hipMemsetAsync(ctx->ip.nodes, 0, (size_t)ctx->ip.B * ctx->ip.nt * ctx->ip.Nn * kImBlock,
                             ctx->stream));
  const int64_t slots = (int64_t)ctx->ip.B * ctx->ip.nt * ctx->ip.H;
  const int64_t cblocks = std::min<int64_t>((slots + 255) / 256, 256 * 64);
  hipLaunchKernelGGL(k_im_clear_hash, dim3((unsigned)cblocks), dim3(256), 0, ctx->stream, ctx->ip.hash,
                     slots);
  IM_LAUNCH(ctx, k_im_reset, dim3(im_blocks(ctx->ip.B)), dim3(64), ctx->ip);
  IM_TRY(ctx, hipGetLastError());
  IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

static int im_first_error(intmcp_ctx* ctx, const char* what) {
  for (int t = 0; t < ctx->ip.B; ++t) {
    const int e = ctx->host_out[2 * t + 1];
    if (e != 0) {
      ctx->err = std::string(what) + ": pair " + std::to_string(t) + ": status " + std::to_string(e);
      return e;
    }
  }
  return POMCP_OK;
}

int intmcp_update(intmcp_ctx* ctx, const int32_t* actions, const uint64_t* obs_keys,
                  int32_t* root_absorbing_out) {
  if (!ctx || !obs_keys) return POMCP_E_INVALID;
  IM_TRY(ctx, hipSetDevice(ctx->device));
  const int B = ctx->ip.B;
  std::vector<int32_t> acts((size_t)B, -1);
  if (actions) std::memcpy(acts.data(), actions, sizeof(int32_t) * (size_t)B);
  IM_TRY(ctx, hipMemcpyAsync((void*)ctx->ip.in_actions, acts.data(), sizeof(int32_t) * B,
                             hipMemcpyHostToDevice, ctx->stream));
  IM_TRY(ctx, hipMemcpyAsync((void*)ctx->ip.in_obs, obs_keys, sizeof(uint64_t) * B,
                             hipMemcpyHostToDevice, ctx->stream));
  // a wave per pair for few pairs (the drop-in): the update's log scans are
  // shared by the wave's lanes (k_im_update kWave); a lane per pair otherwise
  const bool wave = B <= 1024;
  const dim3 ugrid(wave ? (unsigned)B : (unsigned)im_blocks(B));
#define IM_UPDATE_N(NT)                                                                                     \
  do {                                                                                                      \
    if (ctx->cfg.base.env_id == POMCP_ENV_PURSUIT_EVASION) {                                                \
      if (wave) hipLaunchKernelGGL((k_im_updateN<EnvPursuitEvasion, NT, true>), ugrid, dim3(64), 0, ctx->stream, ctx->ip); \
      else hipLaunchKernelGGL((k_im_updateN<EnvPursuitEvasion, NT, false>), ugrid, dim3(64), 0, ctx->stream, ctx->ip); \
    } else {                                                                                                \
      if (wave) hipLaunchKernelGGL((k_im_updateN<EnvDriving, NT, true>), ugrid, dim3(64), 0, ctx->stream, ctx->ip); \
      else hipLaunchKernelGGL((k_im_updateN<EnvDriving, NT, false>), ugrid, dim3(64), 0, ctx->stream, ctx->ip); \
    }                                                                                                       \
  } while (0)
  if (ctx->ip.nt == 6) {   // nesting level 5
    IM_UPDATE_N(6);
  } else if (ctx->ip.nt == 5) {   // nesting level 4
    IM_UPDATE_N(5);
  } else if (ctx->ip.nt == 4) {   // nesting level 3
    IM_UPDATE_N(4);
  } else if (ctx->ip.nt == 3) {   // nesting level 2
    IM_UPDATE_N(3);
  } else if (ctx->cfg.base.env_id == POMCP_ENV_PURSUIT_EVASION) {
    if (wave) hipLaunchKernelGGL((k_im_update<EnvPursuitEvasion, true>), ugrid, dim3(64), 0, ctx->stream, ctx->ip);
    else hipLaunchKernelGGL((k_im_update<EnvPursuitEvasion, false>), ugrid, dim3(64), 0, ctx->stream, ctx->ip);
  } else {
    if (wave) hipLaunchKernelGGL((k_im_update<EnvDriving, true>), ugrid, dim3(64), 0, ctx->stream, ctx->ip);
    else hipLaunchKernelGGL((k_im_update<EnvDriving, false>), ugrid, dim3(64), 0, ctx->stream, ctx->ip);
  }
  IM_TRY(ctx, hipGetLastError());
  IM_TRY(ctx, hipMemcpyAsync(ctx->host_out.data(), ctx->ip.out, sizeof(int32_t) * 2 * B,
                             hipMemcpyDeviceToHost, ctx->stream));
  IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (root_absorbing_out)
    for (int t = 0; t < B; ++t) root_absorbing_out[t] = ctx->host_out[2 * t];
  return im_first_error(ctx, "update");
}

static int im_fetch_hdr(intmcp_ctx* ctx) {
  IM_TRY(ctx, hipMemcpyAsync(ctx->host_hdr.data(), ctx->ip.hdr, sizeof(IHdr) * ctx->ip.B,
                             hipMemcpyDeviceToHost, ctx->stream));
  IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

// one launch of sims[l] simulations at level l (l = 0 .. nt - 1 in turn; nt >= 3)
static int im_searchN(intmcp_ctx* ctx, const int32_t sims[kImMaxT], int32_t flags, int32_t* actions_out);

int intmcp_search_levels(intmcp_ctx* ctx, int32_t level0_sims, int32_t level1_sims,
                         int32_t flags, int32_t* actions_out) {
  if (!ctx || level0_sims < 0 || level1_sims < 0 || (flags & ~(kImBegin | kImFinal)))
    return POMCP_E_INVALID;
  if (ctx->ip.nest0 && level1_sims > 0) {
    ctx->err = "search_levels: nesting level 0 has no level-1 simulations";
    return POMCP_E_INVALID;
  }
  if (ctx->ip.nt >= 3) {
    int32_t sims[kImMaxT] = {};
    sims[0] = level0_sims;
    sims[1] = level1_sims;
    return im_searchN(ctx, sims, flags, actions_out);
  }
  IM_TRY(ctx, hipSetDevice(ctx->device));
  IM_LAUNCH(ctx, k_im_search, dim3(im_blocks(ctx->ip.B)), dim3(64), ctx->ip, (int)level0_sims,
            (int)level1_sims, (int)flags);
  IM_TRY(ctx, hipGetLastError());
  if (!actions_out) return POMCP_OK;
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  for (int t = 0; t < ctx->ip.B; ++t) {
    if (ctx->host_hdr[t].err != 0) {
      ctx->err = "search: pair " + std::to_string(t) + ": status " + std::to_string(ctx->host_hdr[t].err);
      return ctx->host_hdr[t].err;
    }
    actions_out[t] = ctx->host_hdr[t].last_action;
  }
  return POMCP_OK;
}

static int im_searchN(intmcp_ctx* ctx, const int32_t sims[kImMaxT], int32_t flags, int32_t* actions_out) {
  IM_TRY(ctx, hipSetDevice(ctx->device));
  const dim3 grid(im_blocks(ctx->ip.B));
  const bool pe = ctx->cfg.base.env_id == POMCP_ENV_PURSUIT_EVASION;
  ImSims s{};
  for (int l = 0; l < ctx->ip.nt; ++l) s.s[l] = sims[l];
#define IM_SEARCH_N(NT)                                                                                      \
  do {                                                                                                       \
    if (pe) hipLaunchKernelGGL((k_im_searchN<EnvPursuitEvasion, NT>), grid, dim3(64), 0, ctx->stream, ctx->ip, s, (int)flags); \
    else hipLaunchKernelGGL((k_im_searchN<EnvDriving, NT>), grid, dim3(64), 0, ctx->stream, ctx->ip, s, (int)flags); \
  } while (0)
  switch (ctx->ip.nt) {   // a tree per nesting level
    case 6: IM_SEARCH_N(6); break;
    case 5: IM_SEARCH_N(5); break;
    case 4: IM_SEARCH_N(4); break;
    default: IM_SEARCH_N(3); break;
  }
#undef IM_SEARCH_N
  IM_TRY(ctx, hipGetLastError());
  if (!actions_out) return POMCP_OK;
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  for (int t = 0; t < ctx->ip.B; ++t) {
    if (ctx->host_hdr[t].err != 0) {
      ctx->err = "search: pair " + std::to_string(t) + ": status " + std::to_string(ctx->host_hdr[t].err);
      return ctx->host_hdr[t].err;
    }
    actions_out[t] = ctx->host_hdr[t].last_action;
  }
  return POMCP_OK;
}

int intmcp_search(intmcp_ctx* ctx, int32_t num_sims, int32_t* actions_out) {
  if (!ctx || num_sims < 0) return POMCP_E_INVALID;
  if (ctx->ip.nt >= 3) {
    int32_t sims[kImMaxT] = {};
    for (int l = 0; l < ctx->ip.nt; ++l) sims[l] = num_sims;
    return im_searchN(ctx, sims, kImBegin | kImFinal, actions_out);
  }
  return intmcp_search_levels(ctx, num_sims, ctx->ip.nest0 ? 0 : num_sims, kImBegin | kImFinal,
                              actions_out);
}

int intmcp_search_level(intmcp_ctx* ctx, int32_t level, int32_t sims, int32_t flags,
                        int32_t* actions_out) {
  if (!ctx || sims < 0 || (flags & ~(kImBegin | kImFinal))) return POMCP_E_INVALID;
  const int top = ctx->ip.nest0 ? 0 : ctx->ip.nt - 1;   // the planner's nesting level
  if (level < 0 || level > top) {
    ctx->err = "search_level: no level " + std::to_string(level);
    return POMCP_E_INVALID;
  }
  if (ctx->ip.nt >= 3) {
    int32_t s[kImMaxT] = {};
    s[level] = sims;
    return im_searchN(ctx, s, flags, actions_out);
  }
  return intmcp_search_levels(ctx, level == 0 ? sims : 0, level == 1 ? sims : 0, flags, actions_out);
}

int intmcp_get_root_stats(intmcp_ctx* ctx, intmcp_root_stats* out) {
  if (!ctx || !out) return POMCP_E_INVALID;
  IM_TRY(ctx, hipSetDevice(ctx->device));
  const int B = ctx->ip.B;
  if (!ctx->dev_rstats) {
    void* p = nullptr;
    const int rc = im_alloc(ctx, &p, sizeof(intmcp_root_stats) * (size_t)B);
    if (rc != POMCP_OK) return rc;
    ctx->dev_rstats = reinterpret_cast<intmcp_root_stats*>(p);
  }
  // one lane per pair gathers its root's record, then a single copy
  hipLaunchKernelGGL(k_im_root_stats, dim3(im_blocks(B)), dim3(64), 0, ctx->stream, ctx->ip,
                     ctx->dev_rstats);
  IM_TRY(ctx, hipGetLastError());
  const int rc = im_copy(ctx, out, ctx->dev_rstats, (size_t)B);
  if (rc != POMCP_OK) return rc;
  // a failed search (arena, depleted root, ...) is reported here, as
  // pomcp_get_root_stats does: its partial tree's action must not be used
  for (int t = 0; t < B; ++t) {
    if (out[t].error != 0) {
      ctx->err = "search: pair " + std::to_string(t) + ": status " + std::to_string(out[t].error);
      return out[t].error;
    }
  }
  return POMCP_OK;
}

int intmcp_get_root_belief(intmcp_ctx* ctx, int32_t pair, uint32_t* out, int32_t capacity,
                           int32_t* count) {
  if (!ctx || !count || pair < 0 || pair >= ctx->ip.B) return POMCP_E_INVALID;
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  const IHdr& h = ctx->host_hdr[pair];
  *count = h.root_size;
  if (!out || capacity < h.root_size) return POMCP_OK;
  std::vector<uint4> buf((size_t)h.root_size);
  rc = im_copy(ctx, buf.data(), ctx->ip.root + ((int64_t)pair * 2 + h.root_sel) * ctx->ip.Nr,
               (size_t)h.root_size);
  if (rc != POMCP_OK) return rc;
  for (int i = 0; i < h.root_size; ++i) {
    out[3 * i] = buf[i].x;
    out[3 * i + 1] = buf[i].y;
    out[3 * i + 2] = buf[i].z;
  }
  return POMCP_OK;
}

int intmcp_get_nodes(intmcp_ctx* ctx, int32_t pair, int32_t tree, void* out, int32_t capacity,
                     int32_t* count) {
  if (!ctx || !count || pair < 0 || pair >= ctx->ip.B || tree < 0 || tree >= ctx->ip.nt)
    return POMCP_E_INVALID;
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  const int n = ctx->host_hdr[pair].n_nodes[tree];
  *count = n;
  if (!out || capacity < n) return POMCP_OK;
  // the 32 B record of include/intmcp.h from each node's INode and ICold
  // (layout: intmcp.hip ImPair::N, ImPair::C)
  const int64_t ns = kImBlock;
  std::vector<char> blocks;
  rc = im_copy_blocks(ctx, blocks, pair, tree, n);
  if (rc != POMCP_OK) return rc;
  struct NodeRec {
    int32_t parent;
    uint32_t info;
    int32_t visits, t, stats;
    uint32_t support;
    uint64_t okey;
  };
  NodeRec* o = reinterpret_cast<NodeRec*>(out);
  for (int i = 0; i < n; ++i) {
    INode x;
    ICold c;
    std::memcpy(&x, blocks.data() + (size_t)i * ns, sizeof(INode));
    std::memcpy(&c, blocks.data() + (size_t)i * ns + kImCold, sizeof(ICold));
    o[i] = NodeRec{x.parent, x.info & ~kImStatsBit, x.visits, x.t, c.stats, c.support, c.okey};
  }
  return POMCP_OK;
}

int intmcp_get_stats(intmcp_ctx* ctx, int32_t pair, int32_t tree, void* out, int32_t capacity,
                     int32_t* count) {
  if (!ctx || !count || pair < 0 || pair >= ctx->ip.B || tree < 0 || tree >= ctx->ip.nt)
    return POMCP_E_INVALID;
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  const int n = ctx->host_hdr[pair].n_stats[tree];
  *count = n;
  if (!out || capacity < n) return POMCP_OK;
  // statistics in allocation order (INode.stats = their first index), gathered
  // from the node blocks
  const int nn = ctx->host_hdr[pair].n_nodes[tree];
  const int64_t ns = kImBlock;
  std::vector<char> blocks;
  rc = im_copy_blocks(ctx, blocks, pair, tree, nn);
  if (rc != POMCP_OK) return rc;
  IStat* o = reinterpret_cast<IStat*>(out);
  for (int i = 0; i < nn; ++i) {
    const char* bk = blocks.data() + (size_t)i * ns;   // head {visits, value}; record {total, ...}
    ICold c;
    std::memcpy(&c, bk + kImCold, sizeof(ICold));
    if (c.stats < 0) continue;
    for (int a = 0; a < ctx->ip.A && c.stats + a < n; ++a) {
      IStat st;
      std::memcpy(&st.visits, bk + kImHeads + 12 * (size_t)a, 4);
      st.pad = 0;
      std::memcpy(&st.value, bk + kImHeads + 12 * (size_t)a + 4, 8);
      std::memcpy(&st.total, bk + kImLine + kImRec * (size_t)a, 8);
      st.agg = 0.0;   // not kept
      o[c.stats + a] = st;
    }
  }
  return POMCP_OK;
}

// Debug: per-pair phase cycles of k_im_search (diagnostics build only): the
// first call allocates and zeroes the counters; later searches add to them.
int intmcp_debug_phase_timing(intmcp_ctx* ctx, uint64_t* out, int32_t capacity, int32_t* count) {
  if (!ctx || !count) return POMCP_E_INVALID;
#ifndef POMCP_PHASE_TIMING
  (void)out;
  (void)capacity;
  *count = 0;
  return POMCP_E_UNSUPPORTED;
#else
  const size_t n = (size_t)kImPhases * (size_t)ctx->ip.B;
  if (ctx->ip.timing == nullptr) {
    void* p = nullptr;
    if (im_alloc(ctx, &p, sizeof(uint64_t) * n) != POMCP_OK) return POMCP_E_HIP;
    IM_TRY(ctx, hipMemset(p, 0, sizeof(uint64_t) * n));
    ctx->ip.timing = reinterpret_cast<uint64_t*>(p);
    *count = 0;
    return POMCP_OK;
  }
  *count = (int32_t)n;
  if (out && capacity >= *count) {
    IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
    IM_TRY(ctx, hipMemcpy(out, ctx->ip.timing, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
  }
  return POMCP_OK;
#endif
}

// Debug: the other agent's softmax fast path (ImPair::sample_action) with its
// bound widened `slack` times (>= 1 keeps results exact; a large slack sends
// most draws to the exact FP64 path); from this call on, exact-path draws are
// counted (intmcp_debug_exact_draws).
int intmcp_debug_set_softmax_slack(intmcp_ctx* ctx, float slack) {
  if (!ctx || !(slack >= 1.0f)) return POMCP_E_INVALID;
  if (ctx->ip.exact_draws == nullptr) {
    void* p = nullptr;
    if (im_alloc(ctx, &p, sizeof(unsigned long long)) != POMCP_OK) return POMCP_E_HIP;
    IM_TRY(ctx, hipMemsetAsync(p, 0, sizeof(unsigned long long), ctx->stream));
    ctx->ip.exact_draws = reinterpret_cast<unsigned long long*>(p);
  }
  ctx->ip.fast_slack = slack;
  return POMCP_OK;
}

int intmcp_set_search_policy(intmcp_ctx* ctx, int32_t level, int32_t agent, const double* probs) {
  if (!ctx || agent < 0 || agent > 1) return POMCP_E_INVALID;
  const int top = ctx->ip.nest0 ? 0 : ctx->ip.nt - 1;   // the planner's nesting level
  if (level < 0 || level > top) {
    ctx->err = "set_search_policy: no planner at level " + std::to_string(level);
    return POMCP_E_INVALID;
  }
  const int k = top - level;               // tree 0 = the top level; the level-0 planner's is the last
  const int tree = ctx->ip.nest0 ? 1 : k;
  ImParams& d = ctx->ip;
  if (probs == nullptr) {
    d.sp_fixed[tree][agent] = 0;
  } else {
    // random.choices' cumulative weights, summed left to right as
    // itertools.accumulate does, and total = cum[-1] + 0.0
    double acc = 0.0;
    for (int a = 0; a < d.A; ++a) {
      if (!(probs[a] >= 0.0)) {
        ctx->err = "set_search_policy: negative or NaN weight";
        return POMCP_E_INVALID;
      }
      acc = a == 0 ? probs[0] : acc + probs[a];
      d.sp_cum[tree][agent][a] = acc;
    }
    if (!(acc > 0.0)) {
      ctx->err = "set_search_policy: weights sum to zero";
      return POMCP_E_INVALID;
    }
    d.sp_tot[tree][agent] = acc + 0.0;
    d.sp_fixed[tree][agent] = 1;
  }
  d.sp_any = 0;
  for (int t = 0; t < kImMaxT; ++t)
    for (int i = 0; i < 2; ++i) d.sp_any |= d.sp_fixed[t][i];
  return POMCP_OK;
}

int intmcp_debug_exact_draws(intmcp_ctx* ctx, uint64_t* count) {
  if (!ctx || !count) return POMCP_E_INVALID;
  *count = 0;
  if (ctx->ip.exact_draws == nullptr) return POMCP_OK;
  IM_TRY(ctx, hipMemcpyAsync(count, ctx->ip.exact_draws, sizeof(uint64_t), hipMemcpyDeviceToHost,
                             ctx->stream));
  IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

int intmcp_get_support(intmcp_ctx* ctx, int32_t pair, int32_t* entries, int32_t capacity_entries,
                       int32_t* n_entries, uint32_t* particles, int32_t capacity_particles,
                       int32_t* n_particles) {
  if (!ctx || !n_entries || !n_particles || pair < 0 || pair >= ctx->ip.B) return POMCP_E_INVALID;
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  const IHdr& h = ctx->host_hdr[pair];
  *n_entries = h.n_sup;
  *n_particles = h.sup_used;
  if (entries && capacity_entries >= h.n_sup) {
    rc = im_copy(ctx, reinterpret_cast<ISup*>(entries),
                 ctx->ip.sup + ((int64_t)pair * 2 + h.sup_sel) * ctx->ip.Nr, (size_t)h.n_sup);
    if (rc != POMCP_OK) return rc;
  }
  if (particles && capacity_particles >= h.sup_used) {
    rc = im_copy(ctx, reinterpret_cast<uint2*>(particles),
                 ctx->ip.supp + ((int64_t)pair * 2 + h.sup_sel) * ctx->ip.Nsp, (size_t)h.sup_used);
    if (rc != POMCP_OK) return rc;
  }
  return POMCP_OK;
}

int intmcp_get_middle_support(intmcp_ctx* ctx, int32_t pair, int32_t tree, int32_t* entries,
                              int32_t capacity_entries, int32_t* n_entries, uint32_t* particles,
                              int32_t capacity_particles, int32_t* n_particles) {
  if (!ctx || !n_entries || !n_particles || pair < 0 || pair >= ctx->ip.B) return POMCP_E_INVALID;
  if (tree < 1 || tree > ctx->ip.nt - 2) {
    ctx->err = "get_middle_support: no middle tree " + std::to_string(tree) + " (nesting levels >= 2)";
    return POMCP_E_INVALID;
  }
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  const IHdr& h = ctx->host_hdr[pair];
  const int m = tree - 1;
  *n_entries = h.n_msup[m];
  *n_particles = h.msup_used[m];
  if (entries && capacity_entries >= h.n_msup[m]) {
    rc = im_copy(ctx, reinterpret_cast<ISup*>(entries),
                 ctx->ip.msup[m] + ((int64_t)pair * 2 + h.msel[m]) * ctx->ip.Nr, (size_t)h.n_msup[m]);
    if (rc != POMCP_OK) return rc;
  }
  if (particles && capacity_particles >= h.msup_used[m]) {
    std::vector<uint4> buf((size_t)h.msup_used[m]);
    rc = im_copy(ctx, buf.data(), ctx->ip.msupp[m] + ((int64_t)pair * 2 + h.msel[m]) * ctx->ip.Nsp,
                 (size_t)h.msup_used[m]);
    if (rc != POMCP_OK) return rc;
    for (int i = 0; i < h.msup_used[m]; ++i) {
      particles[3 * i] = buf[i].x;
      particles[3 * i + 1] = buf[i].y;
      particles[3 * i + 2] = buf[i].z;
    }
  }
  return POMCP_OK;
}

int intmcp_get_mid_support(intmcp_ctx* ctx, int32_t pair, int32_t* entries, int32_t capacity_entries,
                           int32_t* n_entries, uint32_t* particles, int32_t capacity_particles,
                           int32_t* n_particles) {
  return intmcp_get_middle_support(ctx, pair, 1, entries, capacity_entries, n_entries, particles,
                                   capacity_particles, n_particles);
}

int intmcp_get_tree_counts(intmcp_ctx* ctx, int32_t* out) {
  if (!ctx || !out) return POMCP_E_INVALID;
  int rc = im_fetch_hdr(ctx);
  if (rc != POMCP_OK) return rc;
  for (int t = 0; t < ctx->ip.B; ++t) {
    const IHdr& h = ctx->host_hdr[t];
    for (int k = 0; k < kImMaxT; ++k) {
      const bool on = k < ctx->ip.nt;
      out[3 * kImMaxT * t + 3 * k] = on ? h.n_nodes[k] : 0;
      out[3 * kImMaxT * t + 3 * k + 1] = on ? h.n_log[k] : 0;
      out[3 * kImMaxT * t + 3 * k + 2] = on ? h.n_stats[k] : 0;
    }
  }
  return POMCP_OK;
}

int intmcp_synthetic_obs(intmcp_ctx* ctx, uint64_t env_seed_base, uint64_t* obs_keys_out) {
  if (!ctx) return POMCP_E_INVALID;
  IM_TRY(ctx, hipSetDevice(ctx->device));
  IM_LAUNCH(ctx, k_im_synthetic, dim3(im_blocks(ctx->ip.B)), dim3(64), ctx->ip, env_seed_base);
  IM_TRY(ctx, hipGetLastError());
  if (obs_keys_out) {
    IM_TRY(ctx, hipMemcpyAsync(obs_keys_out, ctx->ip.out_obs, sizeof(uint64_t) * ctx->ip.B,
                               hipMemcpyDeviceToHost, ctx->stream));
  }
  IM_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return POMCP_OK;
}

}  // extern "C"
