/* pomcp.h — C ABI of the MI355X-native POMCP engine (libpomcp_hip.so).
 *
 * Drop-in boundary for the hot path of posggym_baselines.planning
 * (SURVEY §8(b)).  Plain pointers and sizes only; no torch types.  Every entry
 * point replaces a piece of the reference planner, cited per function below
 * (paths relative to posggym_baselines/planning/ in the reference).
 *
 * Threading: a context is not thread-safe (the reference planner objects are
 * single-threaded).  Host buffers are copied synchronously unless noted.
 * Return codes: POMCP_OK (0) or a negative pomcp_status; pomcp_last_error()
 * gives the message.
 */
#ifndef POMCP_H_
#define POMCP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POMCP_ABI_VERSION 7
#define POMCP_MAX_ACTIONS 8
#define POMCP_MAX_TYPE_POLICIES 8

typedef enum pomcp_status {
  POMCP_OK = 0,
  POMCP_E_INVALID = -1,      /* bad argument / config (MCTSConfig.__post_init__ asserts) */
  POMCP_E_HIP = -2,          /* HIP runtime error */
  POMCP_E_ARENA = -3,        /* per-tree arena capacity exceeded */
  POMCP_E_STATE = -4,        /* call out of order (e.g. search before update) */
  POMCP_E_UNSUPPORTED = -5,  /* model / option not implemented on the GPU */
  POMCP_E_NOT_FOUND = -6,    /* node.py:58-63 AssertionError: root has no child for action */
  POMCP_E_NO_DEVICE = -7
} pomcp_status;

typedef enum pomcp_selection {
  POMCP_SEL_PUCB = 0,     /* mcts.py:492-527 + max_visit final (565-581) */
  POMCP_SEL_UCB = 1,      /* mcts.py:529-546 + max_value final (583-600) */
  POMCP_SEL_UNIFORM = 2   /* mcts.py:548-563 + max_value final */
} pomcp_selection;

typedef enum pomcp_env {
  POMCP_ENV_DRIVING = 1,            /* Driving-v1: pomcp_config.grid */
  POMCP_ENV_PURSUIT_EVASION = 2     /* PursuitEvasion-v1: pomcp_config.pe_grid */
} pomcp_env;

/* Driving-v1 grid tables (16-wide row stride). */
typedef struct pomcp_grid {
  uint8_t wall[256];
  uint8_t dist[8][256];
  uint8_t loc_x[8], loc_y[8], loc_dir[8];
  int32_t width, height, num_locs;
  int32_t obs_front, obs_back, obs_side;
  int32_t pad[2];
} pomcp_grid;

/* PursuitEvasion-v1 grid (16-wide row stride; coordinates are (x, y)). */
typedef struct pomcp_pe_grid {
  uint8_t wall[256];
  uint8_t goal_dist[4][256];      /* BFS distance to goal k (127 = unreachable) */
  uint8_t evader_start[4][2], pursuer_start[4][2], goal[4][2];
  int32_t width, height, n_evader_start, n_pursuer_start, n_goal, max_obs_distance;
  int32_t use_progress_reward, pad;
  double reward_norm;             /* R_MAX + R_PROGRESS * longest start-goal path */
} pomcp_pe_grid;

/* MCTSConfig (config.py:8-55) after __post_init__, plus engine sizing. */
typedef struct pomcp_config {
  int32_t abi_version;          /* = POMCP_ABI_VERSION */
  int32_t env_id;               /* pomcp_env */
  int32_t num_agents;           /* model.possible_agents (2) */
  int32_t ego_agent;            /* index of agent_id in possible_agents */
  int32_t num_actions;          /* model.action_spaces[agent_id].n */
  int32_t action_selection;     /* pomcp_selection */
  int32_t depth_limit;          /* config.py:50-55 */
  int32_t step_limit;           /* mcts.py:53-58; INT32_MAX = unbounded */
  int32_t num_particles;        /* config.py:47 */
  int32_t extra_particles;      /* config.py:48 */
  int32_t has_known_bounds;
  int32_t num_trees;            /* independent planners (batched roots) */
  double discount;
  double c;
  double pucb_exploration_fraction;
  double reinvigoration_sample_limit_factor;
  double known_min, known_max;
  uint64_t seed;                /* MCTSConfig.seed -> stream key (seed, tree) */
  uint32_t tree_key_base;       /* tree t uses key tree_key_base + t */
  int32_t type_based;           /* 1: POTMMCP's type-based search (pomcp_set_type_policies) */
  /* per-tree arena capacities */
  int64_t max_blocks;           /* expanded obs nodes: A x 128 B action nodes each */
  int64_t max_particles;        /* particle log records (16 B) */
  int64_t max_belief;           /* root belief region (16 B records): the root belief and
                                   the one a re-root builds, one from each end (ABI 7;
                                   was one of two ping-pong buffers); < 2^31 */
  int64_t overflow_slots;       /* children beyond 6 per action node; power of two >= 16 */
  /* host-computed FP64 tables (Python's own math.log / float.__pow__) */
  const double* log_table;      /* log_table[n] = math.log(n), n >= 1 */
  int64_t log_table_size;
  const double* discount_pow;   /* discount ** k */
  int64_t discount_pow_size;
  pomcp_grid grid;              /* env_id == POMCP_ENV_DRIVING */
  pomcp_pe_grid pe_grid;        /* env_id == POMCP_ENV_PURSUIT_EVASION */
} pomcp_config;

/* Per-tree result of the last search (MCTS.step_statistics + root children). */
typedef struct pomcp_root_stats {
  int32_t action;               /* _final_action_selection(root) */
  int32_t num_sims;
  int32_t search_depth;
  int32_t root_visits;
  int32_t root_absorbing;
  int32_t belief_size;
  int32_t error;                /* pomcp_status of this tree */
  int32_t num_children;
  int32_t child_visits[POMCP_MAX_ACTIONS];
  double child_values[POMCP_MAX_ACTIONS];
  double child_totals[POMCP_MAX_ACTIONS];
  double min_value, max_value;  /* MinMaxStats (utils.py:15-42) */
  /* work counters (algorithmic-byte accounting) */
  int64_t n_levels;             /* tree levels stepped (mcts.py:330-381) */
  int64_t n_expansions;         /* leaf expansions (mcts.py:318-321) */
  int64_t n_new_nodes;          /* obs nodes created (mcts.py:369); with deferred cut-off
                                   records (pomcp_set_defer_cutoff) the children first
                                   reached by those records are not included -- they are
                                   created at the next re-root, if they survive it */
  int64_t n_rollout_steps;      /* model steps in _rollout (mcts.py:414-450) */
  int64_t n_probes;             /* obs-child hash bucket probes */
  int32_t n_obs_nodes, n_blocks, n_log;
  int32_t n_deferred;           /* levels whose child (beyond the depth / step limits) was
                                   not looked up: deferred records */
  int32_t n_cutoff;             /* levels below the root whose child lies beyond the depth /
                                   step limits (mcts.py:315), deferred or looked up; their
                                   child slot is not rewritten (0: the wave kernel) */
  int32_t n_exact_selects;      /* UCB / PUCB selections decided by the exact FP64 scores
                                   (near-ties of the fast scores, DESIGN.md §4 "Fast
                                   selection"; pomcp_debug_set_select_margin widens it) */
} pomcp_root_stats;

typedef struct pomcp_ctx pomcp_ctx;

/* Library / ABI identity. */
int32_t pomcp_abi_version(void);

/* MCTS.__init__ (mcts.py:29-91): allocate all per-tree device state.
 * `hip_stream` is a hipStream_t (NULL = the library's own stream). */
int pomcp_create(const pomcp_config* cfg, int32_t device, void* hip_stream, pomcp_ctx** out);
void pomcp_destroy(pomcp_ctx* ctx);
const char* pomcp_last_error(const pomcp_ctx* ctx);
int pomcp_set_stream(pomcp_ctx* ctx, void* hip_stream);

/* MCTS.reset (mcts.py:123-138) for every tree: fresh root, t=0; RNG
 * counters persist (the reference's generators are not reseeded). */
int pomcp_reset(pomcp_ctx* ctx);

/* MCTS.update (mcts.py:159-263) for every tree: at t == 0 the initial
 * belief (_initial_update, mcts.py:175-227), else re-root to child
 * (action, obs) and reinvigorate (mcts.py:651-700, belief.py:145-194).
 * obs_keys: packed ego observations (driving.h).  root_absorbing_out may be NULL. */
int pomcp_update(pomcp_ctx* ctx, const int32_t* actions, const uint64_t* obs_keys,
                 int32_t* root_absorbing_out);

/* MCTS.get_action (mcts.py:269-306) for every tree with exactly num_sims
 * simulations each (the time-bounded loop of mcts.py:285 becomes a count).
 * actions_out (host, [num_trees]) may be NULL: results stay on device. */
int pomcp_search(pomcp_ctx* ctx, int32_t num_sims, int32_t* actions_out);
/* num_sims more simulations WITHOUT the final action choice (mcts.py:299-306):
 * a get_action split over several launches -- the wall-clock loop of
 * mcts.py:285 -- is pomcp_search_continue(n1), ..., (nk) then
 * pomcp_search(ctx, 0, ...), and consumes exactly the draws of one
 * pomcp_search(n1 + ... + nk).  Root stats' action is -1 after it. */
int pomcp_search_continue(pomcp_ctx* ctx, int32_t num_sims);

/* Search kernel of pomcp_search / pomcp_search_continue (results are the same
 * bit for bit; only the speed differs):
 *   POMCP_SEARCH_AUTO  (default) wave-per-tree for small batches whose
 *                      scratch fits, tree-per-lane otherwise;
 *   POMCP_SEARCH_LANE  one tree per lane, tree in HBM (k_search: the
 *                      throughput kernel for thousands of trees);
 *   POMCP_SEARCH_WAVE  one wave per tree, tree blocks in LDS (k_search_lds: a
 *                      lone planner's latency, mcts.py:285's loop as fast as one
 *                      tree allows); for depth limits <= 8 the tree's workgroup
 *                      adds step-tree producer waves that evaluate the first
 *                      three levels' generative steps ahead of the search
 *                      (environment POMCP_STEP_TREE=0 / 1 forces them off / on). */
typedef enum pomcp_search_kernel {
  POMCP_SEARCH_AUTO = 0,
  POMCP_SEARCH_LANE = 1,
  POMCP_SEARCH_WAVE = 2
} pomcp_search_kernel;
int pomcp_set_search_kernel(pomcp_ctx* ctx, int32_t kind);
/* The kernel the next search will use (POMCP_SEARCH_LANE or _WAVE). */
int32_t pomcp_search_kernel_used(const pomcp_ctx* ctx);
/* Cut-off children in the lane kernel (k_search): on = 1 (the default) a
 * simulation's arrival at a child beyond the depth / step limits
 * (mcts.py:315) is recorded against its action node and the child is
 * materialised at the next re-root (pomcp_update) -- one slot line less per
 * simulation, the cheaper choice when a tree is searched several times per
 * re-root (batched search throughput); on = 0 looks the child up during the
 * search (as the wave kernel always does) -- the cheaper choice when every
 * search is followed by a re-root (an episode planner).  Same results either
 * way (only node labels differ). */
int pomcp_set_defer_cutoff(pomcp_ctx* ctx, int32_t on);

/* Copy every tree's pomcp_root_stats of the last search to host. */
int pomcp_get_root_stats(pomcp_ctx* ctx, pomcp_root_stats* out);

/* Host particles as the root belief of one FRESH tree (after pomcp_reset,
 * before its first update): `particles` = count (t, v0, v1) u32 triples in
 * insertion order (ParticleBelief, belief.py:47-64), all with the same t >= 1.
 * The root becomes an unexpanded obs node at time t holding them -- what
 * _initial_update builds (mcts.py:175-227), from the caller's particles
 * instead of b0 samples (no RNG draws).  Searches and updates follow as usual. */
int pomcp_set_root_belief(pomcp_ctx* ctx, int32_t tree, const uint32_t* particles, int32_t count);

/* Root belief particles of one tree as (t, v0, v1) u32 triples (belief.py:47-64). */
int pomcp_get_root_belief(pomcp_ctx* ctx, int32_t tree, uint32_t* out, int32_t capacity,
                          int32_t* count);

/* POTMMCP (potmmcp.py:18-301) with non-neural policies: a context created with
 * pomcp_config.type_based = 1 searches with a meta-policy over the ego's
 * policies and a mixture over the other agent's policies, every policy a fixed
 * action distribution (planning/policies.py FixedDistributionPolicy):
 *   - the root belief's particles carry the other agent's policy, drawn by
 *     OtherAgentMixturePolicy.sample_initial_state (other_policy.py:178-183);
 *   - every simulation draws an ego policy from the meta-policy row of its
 *     particle's other-agent policy (POTMMCPMetaPolicy.sample_policy,
 *     potmmcp.py:381-389); the ego rolls out with it (potmmcp.py:221-229) and
 *     the other agent acts by its particle's policy;
 *   - every obs node keeps ObsNode.action_probs, PUCB's prior (mcts.py:492-527):
 *     a child created by a simulation starts with that simulation's ego policy
 *     distribution, a root made by update with `expected_prior`
 *     (get_expected_action_probs(None, ...), potmmcp.py:391-431), and a node's
 *     priors move towards the simulation's policy on every arrival at an
 *     existing child (potmmcp.py:255-264).
 * Draws follow CPython's random.choices (cumulative weights, bisection).  Must
 * be called after pomcp_create and before the first update. */
typedef struct pomcp_type_policies {
  int32_t num_ego;                 /* POTMMCPMetaPolicy.policies, 1..8 */
  int32_t num_other;               /* OtherAgentMixturePolicy.policies, 1..8 (dict order) */
  double ego_pi[POMCP_MAX_TYPE_POLICIES][POMCP_MAX_ACTIONS];     /* get_pi, action order */
  double other_pi[POMCP_MAX_TYPE_POLICIES][POMCP_MAX_ACTIONS];
  /* meta_policy[other policy j]: its keys (ego policy indices) and weights in the dict's order */
  int32_t meta_len[POMCP_MAX_TYPE_POLICIES];
  int32_t meta_policy[POMCP_MAX_TYPE_POLICIES][POMCP_MAX_TYPE_POLICIES];
  double meta_weight[POMCP_MAX_TYPE_POLICIES][POMCP_MAX_TYPE_POLICIES];
  double expected_prior[POMCP_MAX_ACTIONS];
  /* The base planner (MCTS / IPOMCP / POMCP, mcts.py:22-739) with fixed-
   * distribution policies runs on the same machinery; zeros = POTMMCP:
   *   no_meta_draw     no sample_policy draw per simulation (ego policy 0 = the
   *                    search policy, potmmcp.py:381-389 is POTMMCP's only);
   *   no_mixture_draw  no policy draw per initial particle (the other agent is
   *                    one stateless policy, index 0: state_belief_only=True);
   *   ego_uniform      the ego's rollout draws Discrete.sample() (RandomSearchPolicy,
   *                    search_policy.py:170) instead of random.choices over ego_pi;
   *   other_uniform    the other agent draws Discrete.sample()
   *                    (RandomOtherAgentPolicy, other_policy.py:151). */
  int32_t no_meta_draw, no_mixture_draw, ego_uniform, other_uniform;
} pomcp_type_policies;
int pomcp_set_type_policies(pomcp_ctx* ctx, const pomcp_type_policies* tp);

/* Type-based contexts: the root's ObsNode.action_probs (num_actions doubles) and
 * its particles' other-agent policy indices (belief order). */
int pomcp_get_root_prior(pomcp_ctx* ctx, int32_t tree, double* out);
int pomcp_get_root_policies(pomcp_ctx* ctx, int32_t tree, int32_t* out, int32_t capacity,
                            int32_t* count);

/* Arena use: the largest block count and particle-log record count over the
 * trees (after the last update's subtree compaction / the last search).  The
 * wall-clock loop sizes its chunks from it (never overflowing the arenas). */
int pomcp_arena_usage(pomcp_ctx* ctx, int32_t* max_blocks_used, int32_t* max_log_used);

/* Root-parallel search: re-key every tree's streams to `seed`
 * keeping counters (rank g uses seed ^ (g << 32)). */
int pomcp_rekey(pomcp_ctx* ctx, uint64_t seed);

/* Exchange record of one tree, written by pomcp_search (the operand of the
 * root-parallel exchange at action-selection time): POMCP_XREC(A) doubles =
 *   [2a] child visits, [2a + 1] child total value    (a < num_actions)
 *   [2A + 0] num_sims, [2A + 1] root visits, [2A + 2] search depth,
 *   [2A + 3] error (pomcp_status), [2A + 4] min value, [2A + 5] max value
 * (integers are exact in a double). */
#define POMCP_XREC_STATS 6
#define POMCP_XREC(num_actions) (2 * (num_actions) + POMCP_XREC_STATS)

/* Device pointer of the merge buffer: double[num_trees][POMCP_XREC(A)], this
 * GPU's exchange records. */
int pomcp_root_merge_buffer(pomcp_ctx* ctx, void** device_ptr);

/* Device pointer of the gather buffer: double[world][num_trees][POMCP_XREC(A)],
 * every rank's merge buffer in rank order (allocated on the first call for a
 * given world size; a larger world re-allocates).  The caller may fill it with
 * its own all-gather (e.g. torch.distributed.all_gather_into_tensor) instead
 * of pomcp_allgather_root. */
int pomcp_root_gather_buffer(pomcp_ctx* ctx, int32_t world, void** device_ptr);

/* The root-parallel exchange of SURVEY §8(b)/(e) (mcts.py:269-306 run as
 * root-parallel trees on several GPUs): ncclAllGather(merge buffer -> gather
 * buffer, num_trees * POMCP_XREC(A) doubles per rank, comm, context stream),
 * before pomcp_merge_roots(..., world, ...).  An all-gather, not an
 * all-reduce: the merge then sums the replicas in one fixed order on every
 * rank (a ring all-reduce's summation order depends on the algorithm and the
 * rank count, so its FP64 sums could not be restated).  rccl_comm: an
 * ncclComm_t of `world` ranks, one per GPU, created by the RCCL library that
 * is already loaded in this process (PyTorch's, or one the caller loaded): the
 * library never loads a second RCCL copy; POMCP_E_UNSUPPORTED if none is loaded. */
int pomcp_allgather_root(pomcp_ctx* ctx, void* rccl_comm, int32_t world);

/* Root-parallel decision of one planner. */
typedef struct pomcp_merged_root {
  int32_t action;               /* merged final action (see pomcp_merge_roots) */
  int32_t num_trees;            /* replicas merged */
  int32_t search_depth;         /* max over the replicas */
  int32_t error;                /* first non-zero replica error, in replica order */
  int64_t num_sims;             /* summed over the replicas */
  int64_t root_visits;          /* summed */
  double min_value, max_value;  /* min / max over the replicas' MinMaxStats */
  double visits[POMCP_MAX_ACTIONS];   /* summed root child visits */
  double totals[POMCP_MAX_ACTIONS];   /* summed root child total values */
} pomcp_merged_root;

/* Root-parallel merge on the device: trees [g*group, (g+1)*group) are the
 * replicas of planner g on every rank (num_trees % group == 0).
 *   world == 0: this GPU's merge buffer alone (replicas k = 0..group-1);
 *   world >= 1: the gather buffer of `world` ranks (pomcp_allgather_root):
 *               replica j = r * group + k is tree g*group + k of rank r.
 * Replica records are summed in one fixed order -- lane l of a 64-lane wave
 * sums replicas [l*c, (l+1)*c), c = ceil(N / 64), N = max(world,1) * group, in
 * replica order from 0.0, then the 64 partials in lane order from 0.0
 * (restated by oracle/root_parallel.py) -- so every rank takes the same
 * decision, bit-identical to one GPU merging all N replicas:
 *   PUCB: argmax summed visits (the merged max_visit_action_selection,
 *         mcts.py:565-581);  UCB / uniform: argmax summed total / summed visits
 *         over visited actions (max_value_action_selection, mcts.py:583-600);
 * lowest action on ties, 0 if nothing was visited.  Replaces the reference's
 * single-tree _final_action_selection when one planner runs many trees.
 * out (host, [num_trees / group]) may be NULL: the result stays on device. */
int pomcp_merge_roots(pomcp_ctx* ctx, int32_t group, int32_t world, pomcp_merged_root* out);

/* Bench / batch helpers: synthetic roots (the configured environment).  Tree b samples s0 from
 * the model's b0 under env key (env_seed_base + b, 0x40000000) and the ego's
 * initial obs is written to obs_keys_out (host, [num_trees], may be NULL). */
int pomcp_synthetic_obs(pomcp_ctx* ctx, uint64_t env_seed_base, uint64_t* obs_keys_out);
/* The environment's answer to the planners' actions (env.step of the episode
 * loop, exp_utils.py:481-505, for the synthetic roots): tree b's true initial
 * state (as pomcp_synthetic_obs) stepped with actions[b] (host, [num_trees]) and
 * the other agent's uniformly drawn action (env key's action stream); the ego's
 * next observation -> obs_keys_out (host, may be NULL).  For update()-inclusive
 * benchmark steps. */
int pomcp_synthetic_step(pomcp_ctx* ctx, uint64_t env_seed_base, const int32_t* actions,
                         uint64_t* obs_keys_out);
/* Save / restore the complete post-update root state (headers, root nodes,
 * root belief, RNG counters) so a timed loop can re-search the same roots. */
int pomcp_snapshot(pomcp_ctx* ctx);
int pomcp_restore(pomcp_ctx* ctx);

/* ---- Host (CPU) Driving-v1 model from the same header (driving.h) -------
 * The environment side of the episode loop (env.step in
 * tests/planning/test_pomcp.py:23-29); not on the planner's hot path. */
int pomcp_driving_sample_initial_state(const pomcp_grid* g, uint64_t seed, uint32_t tree,
                                       uint32_t* model_ctr, uint32_t state_out[2]);
/* One joint step; draws the execution-order shuffle from the model stream
 * (seed, tree) at counter *model_ctr (advanced). */
int pomcp_driving_step(const pomcp_grid* g, uint64_t seed, uint32_t tree, uint32_t* model_ctr,
                       const uint32_t state[2], const int32_t actions[2], uint32_t next_out[2],
                       double rewards_out[2], int32_t terminated_out[2],
                       uint64_t obs_keys_out[2]);
int pomcp_driving_obs(const pomcp_grid* g, const uint32_t state[2], uint64_t obs_keys_out[2]);

/* ---- Host (CPU) PursuitEvasion-v1 model from csrc/pursuit_evasion.h ----- */
int pomcp_pe_sample_initial_state(const pomcp_pe_grid* g, uint64_t seed, uint32_t tree,
                                  uint32_t* model_ctr, uint32_t state_out[2]);
/* One joint step (deterministic: no model draw). */
int pomcp_pe_step(const pomcp_pe_grid* g, const uint32_t state[2], const int32_t actions[2],
                  uint32_t next_out[2], double rewards_out[2], int32_t terminated_out[2],
                  uint64_t obs_keys_out[2]);
int pomcp_pe_obs(const pomcp_pe_grid* g, const uint32_t state[2], uint64_t obs_keys_out[2]);

/* ---- Host RNG streams (csrc/philox.h) -----------------------------------
 * out[k] = word (first + k) of Philox stream `stream` under key (seed, tree):
 * the draws of the episode loop's non-planning agents (the reference's
 * UniformOtherAgentFn / Random-v0 policies, baseline_exps/exp_utils.py:481). */
int pomcp_philox_words(uint64_t seed, uint32_t tree, uint32_t stream, uint32_t first, int32_t n,
                       uint32_t* out);

/* ---- Host math.log table -------------------------------------------------
 * out[k] = log(first + k) with the host C library's log (the function
 * Python's math.log calls: mcts.py:534's log(N) bit for bit), 0.0 for 0; the
 * planner's pomcp_config.log_table at C speed (wall-clock arenas ask for tens
 * of millions of entries). */
int pomcp_host_log_table(int64_t first, int64_t n, double* out);

#ifdef __cplusplus
}
#endif

#endif /* POMCP_H_ */
