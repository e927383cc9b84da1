/* pomcp_debug.h — diagnostics of libpomcp_hip.so (not part of the drop-in ABI). */
#ifndef POMCP_DEBUG_H_
#define POMCP_DEBUG_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* out[4*i + k] = {sqrt(a), a / b, a + 0.95 * b, (a - b) / (a + b)} computed on
 * device 0 in FP64 (checks the device FP64 path is correctly rounded). */
int pomcp_debug_fp_selftest(const double* a, const double* b, int32_t n, double* out);
/* out[2i] = rcp_nr(x[i]), out[2i + 1] = rsq_nr(x[i]) on device 0: the FP64
 * 1/x and 1/sqrt(x) of k_search's fast UCB scores (hardware estimate + two
 * Newton steps), whose error bound decides when the exact scores are needed. */
int pomcp_debug_fast_recip(const double* x, int32_t n, double* out);
/* out[i] = host_exp(x[i]) on device 0 (FP64): the I-NTMCP softmax's exp, a
 * bit-exact restatement of the host libm's exp (csrc/host_exp.h). */
int pomcp_debug_exp(const double* x, int32_t n, double* out);
/* The same function evaluated on the host CPU (no GPU needed). */
int pomcp_debug_host_exp(const double* x, int32_t n, double* out);
/* k_search phase cycles per wave, [waves][16] (libpomcp_hip built with
 * -DPOMCP_PHASE_TIMING; POMCP_E_UNSUPPORTED otherwise).  The first call
 * enables collection (count = 0); later calls copy the last search's values
 * when capacity >= count. */
typedef struct pomcp_ctx pomcp_ctx;
int pomcp_debug_phase_timing(pomcp_ctx* ctx, uint64_t* out, int32_t capacity, int32_t* count);
/* k_im_search phase cycles per wave (libpomcp_hip built with
 * -DPOMCP_PHASE_TIMING; POMCP_E_UNSUPPORTED otherwise), same protocol as
 * pomcp_debug_phase_timing (tools/phase_timing_im.py). */
typedef struct intmcp_ctx intmcp_ctx;
int intmcp_debug_phase_timing(intmcp_ctx* ctx, uint64_t* out, int32_t capacity, int32_t* count);
/* k_search_lds (the wave-per-tree kernel): polls of a late step-tree hand-off
 * before the search wave stops its producer waves and computes the rest of the
 * launch itself (0 = the default, ~0.1 s); results are the same either way. */
int pomcp_debug_set_spin_limit(pomcp_ctx* ctx, int32_t polls);
/* I-NTMCP: the other agent's softmax (sample_action, intmcp.py:763-791) takes
 * its choice from bounded FP32 weights and falls back to the exact FP64 path
 * near a cumulative weight; `slack` (>= 1, default 1) widens that bound, so a
 * large value sends most draws down the exact path (results stay exact).  From
 * this call on the exact-path draws are counted: intmcp_debug_exact_draws. */
int intmcp_debug_set_softmax_slack(intmcp_ctx* ctx, float slack);
int intmcp_debug_exact_draws(intmcp_ctx* ctx, uint64_t* count);
/* k_search's fast UCB / PUCB selection (DESIGN.md §4 "Fast selection") takes
 * the fast scores' leader unless an action with different statistics scores
 * within `rel` of it relative to their magnitudes, and then decides with the
 * exact FP64 scores (mcts.py:502-546).  rel >= 1e-12 (the default, above the
 * fast scores' proven error) keeps results exact; a large rel (e.g. 1e-4)
 * sends most selections down the exact path.  pomcp_root_stats.n_exact_selects
 * counts them per tree and search. */
int pomcp_debug_set_select_margin(pomcp_ctx* ctx, double rel);
/* Only the first n (1..6) inline obs-child slots of each action node are used,
 * the overflow map holds the rest (tests of that path).  Before the first search. */
int pomcp_debug_set_inline_slots(pomcp_ctx* ctx, int32_t n);
#ifdef __cplusplus
}
#endif
#endif
