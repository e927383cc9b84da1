// Host-only entry points of libpomcp_hip.so (include/pomcp.h, pomcp_debug.h):
// the environment side of the episode loop (Driving-v1 / PursuitEvasion-v1
// from the same driving.h / pursuit_evasion.h the kernels use), the host RNG
// words and the host log / exp tables -- the reference's step / obs / RNG
// contract (mcts.py:181-198, 333, 418; exp_utils.py:481).
//
// Plain C++ with no HIP dependency: pomcp_capi.hip includes it into the
// product library, and tests/test_host_sanitize.py compiles it on its own
// with -fsanitize=address,undefined into an executable that serves the same
// calls (tests/native/host_rpc.cpp), so the host code runs under the
// sanitizers through the same Python tests.
#if !defined(__HIPCC__) && !defined(__HIP__)
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif
#include <stdint.h>

#include <cmath>
#include <cstring>

#include "driving.h"
#include "host_exp.h"
#include "philox.h"
#include "pursuit_evasion.h"
#include "../../include/pomcp.h"
#include "../../include/pomcp_debug.h"

using namespace pb;

namespace {
void make_model(const pomcp_grid* g, DrvModel* m) {
  std::memcpy(&m->g, g, sizeof(DrvGrid));
  build_model_tables(m->g, m);
}
}  // namespace

extern "C" {

// ---------------------------------------------------------------- host model

int pomcp_driving_sample_initial_state(const pomcp_grid* g, uint64_t seed, uint32_t tree,
                                       uint32_t* model_ctr, uint32_t state_out[2]) {
  if (!g || !model_ctr || !state_out) return POMCP_E_INVALID;
  const DrvGrid& gg = *reinterpret_cast<const DrvGrid*>(g);
  Streams s;
  s.seed = seed;
  s.tree = tree;
  for (int k = 0; k < 5; ++k) s.ctr[k] = 0;
  s.ctr[2] = *model_ctr;
  drv_sample_initial_state2(gg, [&](uint32_t n) { return s.model(n); }, &state_out[0],
                            &state_out[1]);
  *model_ctr = s.ctr[2];
  return POMCP_OK;
}

int pomcp_driving_step(const pomcp_grid* g, uint64_t seed, uint32_t tree, uint32_t* model_ctr,
                       const uint32_t state[2], const int32_t actions[2], uint32_t next_out[2],
                       double rewards_out[2], int32_t terminated_out[2],
                       uint64_t obs_keys_out[2]) {
  if (!g || !model_ctr || !state || !actions || !next_out) return POMCP_E_INVALID;
  DrvModel m;
  make_model(g, &m);
  Streams s;
  s.seed = seed;
  s.tree = tree;
  for (int k = 0; k < 5; ++k) s.ctr[k] = 0;
  s.ctr[2] = *model_ctr;
  const uint32_t j = s.model(2);   // execution-order shuffle
  *model_ctr = s.ctr[2];
  drv_step2_fast(m, state[0], state[1], actions[0], actions[1], j, &next_out[0], &next_out[1]);
  for (int i = 0; i < 2; ++i) {
    if (rewards_out) rewards_out[i] = drv_reward_fast(m, state[i], next_out[i]);
    if (terminated_out) terminated_out[i] = veh_done(next_out[i]) ? 1 : 0;
  }
  if (obs_keys_out) {
    obs_keys_out[0] = obs_key_fast(m, next_out[0], next_out[1]);
    obs_keys_out[1] = obs_key_fast(m, next_out[1], next_out[0]);
  }
  return POMCP_OK;
}

int pomcp_driving_obs(const pomcp_grid* g, const uint32_t state[2], uint64_t obs_keys_out[2]) {
  if (!g || !state || !obs_keys_out) return POMCP_E_INVALID;
  DrvModel m;
  make_model(g, &m);
  obs_keys_out[0] = obs_key_fast(m, state[0], state[1]);
  obs_keys_out[1] = obs_key_fast(m, state[1], state[0]);
  return POMCP_OK;
}

// ---------------------------------------------------------- host RNG streams

int pomcp_philox_words(uint64_t seed, uint32_t tree, uint32_t stream, uint32_t first, int32_t n,
                       uint32_t* out) {
  if (n < 0 || (n > 0 && !out)) return POMCP_E_INVALID;
  for (int32_t k = 0; k < n; ++k) out[k] = philox_word(seed, tree, stream, first + (uint32_t)k);
  return POMCP_OK;
}

// ---------------------------------------------------------- host log(N) table

// out[i] = log((double)i) for i in [first, first + n), out[0] of i = 0 is 0.0:
// the host C library's log, the function Python's math.log calls for a float
// (Modules/mathmodule.c), so the table is math.log's bit for bit at C speed
// (tests/test_host_exp.py checks it against math.log).
int pomcp_host_log_table(int64_t first, int64_t n, double* out) {
  if (first < 0 || n < 0 || (n > 0 && !out)) return POMCP_E_INVALID;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = first + k;
    out[k] = i == 0 ? 0.0 : std::log((double)i);
  }
  return POMCP_OK;
}

// ---------------------------------------------------------- host PursuitEvasion

int pomcp_pe_sample_initial_state(const pomcp_pe_grid* g, uint64_t seed, uint32_t tree,
                                  uint32_t* model_ctr, uint32_t state_out[2]) {
  if (!g || !model_ctr || !state_out) return POMCP_E_INVALID;
  PeModel m;
  build_pe_model(*g, &m);
  Streams s;
  s.seed = seed;
  s.tree = tree;
  for (int k = 0; k < 5; ++k) s.ctr[k] = 0;
  s.ctr[2] = *model_ctr;
  pe_sample_initial_state(m, [&](uint32_t n) { return s.model(n); }, &state_out[0], &state_out[1]);
  *model_ctr = s.ctr[2];
  return POMCP_OK;
}

int pomcp_pe_step(const pomcp_pe_grid* g, const uint32_t state[2], const int32_t actions[2],
                  uint32_t next_out[2], double rewards_out[2], int32_t terminated_out[2],
                  uint64_t obs_keys_out[2]) {
  if (!g || !state || !actions || !next_out || !rewards_out || !terminated_out || !obs_keys_out)
    return POMCP_E_INVALID;
  for (int i = 0; i < 2; ++i)
    if (actions[i] < 0 || actions[i] > 3) return POMCP_E_INVALID;
  PeModel m;
  build_pe_model(*g, &m);
  uint32_t prog, outcome;
  pe_step(m, state[0], state[1], (uint32_t)actions[0], (uint32_t)actions[1], &next_out[0],
          &next_out[1], &prog, &outcome);
  for (int i = 0; i < 2; ++i) {
    rewards_out[i] = pe_reward(m, i, state[0], prog, outcome);
    terminated_out[i] = pe_done(next_out[0]) ? 1 : 0;
    obs_keys_out[i] = pe_obs_key(m, i, next_out[0], next_out[1]);
  }
  return POMCP_OK;
}

int pomcp_pe_obs(const pomcp_pe_grid* g, const uint32_t state[2], uint64_t obs_keys_out[2]) {
  if (!g || !state || !obs_keys_out) return POMCP_E_INVALID;
  PeModel m;
  build_pe_model(*g, &m);
  for (int i = 0; i < 2; ++i) obs_keys_out[i] = pe_obs_key(m, i, state[0], state[1]);
  return POMCP_OK;
}


// Debug: the same host_exp on the host CPU (tests/test_host_exp.py compares it
// with math.exp without a GPU).
int pomcp_debug_host_exp(const double* x, int32_t n, double* out) {
  if (!x || !out || n < 0) return POMCP_E_INVALID;
  for (int32_t i = 0; i < n; ++i) out[i] = host_exp(x[i]);
  return POMCP_OK;
}

}  // extern "C"
