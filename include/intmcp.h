/* intmcp.h — C ABI of the I-NTMCP engine in libpomcp_hip.so (BASELINE config 5).
 *
 * Drop-in boundary for posggym_baselines.planning.intmcp.INTMCP at nesting
 * level 1 with two agents, as built by
 * INTMCP.initialize(model, ego, config, nesting_level=1, search_policies=None)
 * (intmcp.py:949-994): the ego's level-1 tree and the other agent's level-0
 * tree, random search policies.  One planner pair per "tree" index; many
 * pairs per call (a batched launch).  nesting_level = 0: one level-0 planner
 * per index (its tree is tree 1 of the diagnostics below; the other agent acts
 * by the planner's own random choice, intmcp.py:750-753).  nesting_level = 2:
 * three trees per index -- tree 0 the planner's (level 2), tree 1 the other
 * agent's level-1 planner, tree 2 the level-0 planner of the planner's agent
 * (INTMCP.initialize's recursion, intmcp.py:950-994); nesting_level = 3:
 * four trees -- tree 0 the planner's (level 3), trees 1 and 2 the level-2 and
 * level-1 planners of the other agent and the planner's agent, tree 3 the
 * other agent's level-0 planner; in general nesting_level = L >= 2 keeps L + 1
 * trees, tree k the level-(L - k) planner (of the planner's agent if k is
 * even), up to INTMCP_MAX_TREES.  Paths relative to
 * posggym_baselines/planning/ in the reference.
 *
 * Same conventions as pomcp.h (plain pointers, POMCP_* status codes, a
 * context is not thread-safe).
 */
#ifndef INTMCP_H_
#define INTMCP_H_

#include <stdint.h>

#include "pomcp.h"

#ifdef __cplusplus
extern "C" {
#endif

#define INTMCP_MAX_TREES 6        /* nesting levels 0 .. 5: a tree per level */

typedef struct intmcp_config {
  pomcp_config base;              /* MCTSConfig + model + tables (num_trees = planner pairs) */
  int32_t state_belief_only;      /* MCTSConfig.state_belief_only (test config: 0) */
  int32_t nesting_level;          /* 0 to INTMCP_MAX_TREES - 1 (INTMCP.initialize's nesting_level) */
  int64_t max_nodes;              /* obs nodes per tree */
  int64_t max_stats;              /* action-node statistics entries per tree (A per expanded node) */
  int64_t max_log;                /* particle log records per tree (16 B) */
  int64_t hash_slots;             /* obs-child map slots per tree, power of two */
  int64_t max_root_belief;        /* level-1 root particles (and level-0 support entries) */
  int64_t max_support_particles;  /* materialised level-0 particles per pair */
} intmcp_config;

typedef struct intmcp_root_stats {
  int32_t action;                 /* _final_action_selection of the level-1 root */
  int32_t num_sims;               /* simulations over both levels */
  int32_t search_depth;
  int32_t root_visits;
  int32_t root_absorbing;
  int32_t belief_size;
  int32_t error;
  int32_t num_children;           /* registered children of the root, registration order: */
  int32_t child_action[POMCP_MAX_ACTIONS];
  int32_t child_visits[POMCP_MAX_ACTIONS];
  double child_values[POMCP_MAX_ACTIONS];
  double child_totals[POMCP_MAX_ACTIONS];
  double min_value, max_value;    /* the level-1 planner's MinMaxStats */
  int32_t n_nodes[2], n_log[2], n_stats[2];
  int32_t n_support, pad;
} intmcp_root_stats;

typedef struct intmcp_ctx intmcp_ctx;

/* INTMCP.initialize (intmcp.py:949-994) for every pair. */
int intmcp_create(const intmcp_config* cfg, int32_t device, void* hip_stream, intmcp_ctx** out);
void intmcp_destroy(intmcp_ctx* ctx);
/* ctx == NULL: the reason the calling thread's last intmcp_create failed. */
const char* intmcp_last_error(const intmcp_ctx* ctx);
/* INTMCP.reset (intmcp.py:154-176). */
int intmcp_reset(intmcp_ctx* ctx);
/* INTMCP.update (intmcp.py:198-300): t == 0 -> _initial_nested_update, else
 * _nested_update (re-root, reinvigoration, the level-0 update of every
 * other-agent history in the new root belief). */
int intmcp_update(intmcp_ctx* ctx, const int32_t* actions, const uint64_t* obs_keys,
                  int32_t* root_absorbing_out);
/* intmcp_update action of a pair to leave untouched (its episode has ended). */
#define INTMCP_SKIP (-2)
/* INTMCP.get_action (intmcp.py:368-408) with num_sims simulations per nesting level
 * (nesting level 0: num_sims at level 0). */
int intmcp_search(intmcp_ctx* ctx, int32_t num_sims_per_level, int32_t* actions_out);
/* One chunk of get_action: level0_sims simulations at level 0 then
 * level1_sims at level 1.  flags: INTMCP_BEGIN resets the step's counters,
 * INTMCP_FINAL runs _final_action_selection (actions_out is then valid).  The
 * reference's wall-clock loop (per-level time budget) is a sequence of chunks;
 * intmcp_search(n) == intmcp_search_levels(n, n, BEGIN | FINAL) (nesting level 0:
 * (n, 0); level1_sims > 0 is POMCP_E_INVALID there). */
#define INTMCP_BEGIN 1
#define INTMCP_FINAL 2
int intmcp_search_levels(intmcp_ctx* ctx, int32_t level0_sims, int32_t level1_sims, int32_t flags,
                         int32_t* actions_out);
int intmcp_get_root_stats(intmcp_ctx* ctx, intmcp_root_stats* out);
/* Level-1 root particles of one pair as (v0, v1, level-0 node id) u32 triples. */
int intmcp_get_root_belief(intmcp_ctx* ctx, int32_t pair, uint32_t* out, int32_t capacity,
                           int32_t* count);
/* Diagnostics: one tree's node records (32 B each: parent i32, info u32,
 * visits i32, t i32, stats i32, -, obs key u64; info = parent action:3 |
 * absorbing:1 | path_ok:1 | registered:3 | registration order 6 x 3 bits) and
 * statistics entries (32 B: visits i32, -, value f64, total f64, agg f64 = 0: not kept);
 * tree 0 = the planner's (top) level, tree k the level k below it (the last
 * tree level 0). */
int intmcp_get_nodes(intmcp_ctx* ctx, int32_t pair, int32_t tree, void* out, int32_t capacity,
                     int32_t* count);
int intmcp_get_stats(intmcp_ctx* ctx, int32_t pair, int32_t tree, void* out, int32_t capacity,
                     int32_t* count);
/* The materialised level-0 beliefs: entries (node, offset, size, capacity) and
 * their (v0, v1) particles. */
int intmcp_get_support(intmcp_ctx* ctx, int32_t pair, int32_t* entries, int32_t capacity_entries,
                       int32_t* n_entries, uint32_t* particles, int32_t capacity_particles,
                       int32_t* n_particles);
/* Nesting levels 2, 3: middle tree `tree`'s (1 <= tree <= nesting level - 1)
 * materialised beliefs of the histories in the belief distribution above it
 * (tree 1: the top root belief's): entries (node, offset, size, capacity) and
 * their (v0, v1, next tree's node id) particles.  POMCP_E_INVALID for any other
 * tree.  (intmcp_get_support is always the level-0 tree's.) */
int intmcp_get_middle_support(intmcp_ctx* ctx, int32_t pair, int32_t tree, int32_t* entries,
                              int32_t capacity_entries, int32_t* n_entries, uint32_t* particles,
                              int32_t capacity_particles, int32_t* n_particles);
/* intmcp_get_middle_support of tree 1. */
int intmcp_get_mid_support(intmcp_ctx* ctx, int32_t pair, int32_t* entries, int32_t capacity_entries,
                           int32_t* n_entries, uint32_t* particles, int32_t capacity_particles,
                           int32_t* n_particles);
/* One chunk of get_action at one nesting level (level <= the planner's):
 * `sims` simulations at `level` (intmcp.py:385-392; the wall-clock loop of a
 * nesting-level-2 planner is a sequence of these).  flags as
 * intmcp_search_levels. */
int intmcp_search_level(intmcp_ctx* ctx, int32_t level, int32_t sims, int32_t flags,
                        int32_t* actions_out);
/* Arena counters of every pair: out[pair][tree][{nodes, log records, stats}]
 * for trees 0 .. INTMCP_MAX_TREES - 1 (zeros for a tree the nesting level does
 * not have), B x INTMCP_MAX_TREES x 3. */
int intmcp_get_tree_counts(intmcp_ctx* ctx, int32_t* out);
/* INTMCP.initialize's search_policies (intmcp.py:956-971): the search policy of
 * agent `agent` at nesting level `level` -- NULL: RandomSearchPolicy
 * (Discrete.sample(), the default), else the num_actions probabilities of a
 * SearchPolicyWrapper(FixedDistributionPolicy), drawn as random.choices on the
 * agent's action stream.  It draws the rollout actions of that level's planner
 * (intmcp.py:547-593) and, at level 1, the other agent's action at a history
 * its level-0 tree has not visited (intmcp.py:778-780).  Takes effect at the
 * next search; every pair of the context. */
int intmcp_set_search_policy(intmcp_ctx* ctx, int32_t level, int32_t agent, const double* probs);
/* Synthetic roots (as pomcp_synthetic_obs). */
int intmcp_synthetic_obs(intmcp_ctx* ctx, uint64_t env_seed_base, uint64_t* obs_keys_out);

#ifdef __cplusplus
}
#endif

#endif /* INTMCP_H_ */
