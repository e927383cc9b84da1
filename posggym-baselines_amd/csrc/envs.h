// The generative models the engine runs, behind one static interface.
//
// Every kernel is templated on an Env:
//   Model                      device tables (staged in LDS)
//   kStepDraws                 model-stream draws per joint step (Driving's
//                              execution-order shuffle: 1; PursuitEvasion: 0)
//   step(m, ego, s0, s1, a_ego, a_oth, j, &n0, &n1, &r, &done)
//                              joint step + the ego's reward and
//                              terminated-or-all-done flag (mcts.py:333-344)
//   obs_key(m, ego, n0, n1)    the ego's packed observation
//   done_of(ego, n0, n1)       step's done flag, from the next state alone
//   sample_initial(m, draw, &s0, &s1)             model.sample_initial_state
//   sample_agent_initial(m, ego, obs, draw, &s0, &s1)
//                              model.sample_agent_initial_state (false: obs
//                              inconsistent with the model)
// step/obs_key work per lane (the search kernel: one tree per lane) and in
// the wave-per-tree kernels (every lane computes the tree's uniform value).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "driving.h"
#include "driving_vec.h"
#include "pursuit_evasion.h"

namespace pb {

struct EnvDriving {
  using Model = DrvModel;
  static constexpr int kStepDraws = 1;
  static constexpr int kEnvId = POMCP_ENV_DRIVING;
  static constexpr int kA = 5;   // actions per agent

  __device__ static __forceinline__ void step(const Model& m, int ego, uint32_t s0, uint32_t s1,
                                              uint32_t a_ego, uint32_t a_oth, uint32_t j,
                                              uint32_t* n0, uint32_t* n1, double* r, int* done) {
    drv_step2_vec(m, s0, s1, ego == 0 ? a_ego : a_oth, ego == 0 ? a_oth : a_ego, j, n0, n1);
    const uint32_t e0 = ego == 0 ? s0 : s1, e1 = ego == 0 ? *n0 : *n1;
    *r = drv_reward_vec(m, e0, e1);
    *done = done_of(ego, *n0, *n1);
  }
  // the ego's terminated-or-all-done flag of a next state (mcts.py:340-344):
  // a function of the state alone (deferred records, pomcp_device.h)
  __device__ static __forceinline__ int done_of(int ego, uint32_t n0, uint32_t n1) {
    const uint32_t e1 = ego == 0 ? n0 : n1;
    return (((e1 >> 15) & 3u) != 0u || (((n0 >> 15) & 3u) != 0u && ((n1 >> 15) & 3u) != 0u)) ? 1 : 0;
  }
  __device__ static __forceinline__ uint64_t obs_key(const Model& m, int ego, uint32_t n0,
                                                     uint32_t n1) {
    return obs_key_vec(m, ego == 0 ? n0 : n1, ego == 0 ? n1 : n0);
  }
  template <class Draw>
  __device__ static void sample_initial(const Model& m, Draw draw, uint32_t* s0, uint32_t* s1) {
    drv_sample_initial_state2(m.g, draw, s0, s1);
  }
  // oracle/driving.py sample_agent_initial_state: ego from its obs, the other
  // vehicle rejected until the ego window matches (<= 64 tries).
  template <class Draw>
  __device__ static bool sample_agent_initial(const Model& m, int ego, uint64_t obs, Draw draw,
                                              uint32_t* s0, uint32_t* s1) {
    const DrvGrid& g = m.g;
    const int eloc = loc_index(g, (int)((obs >> 32) & 15), (int)((obs >> 36) & 15));
    const int edest = loc_index(g, (int)((obs >> 40) & 15), (int)((obs >> 44) & 15));
    if (eloc < 0 || edest < 0) return false;
    const uint32_t all = (1u << g.num_locs) - 1u;
    const uint32_t ev = make_vehicle(g, eloc, edest);
    uint32_t ov = 0;
    for (int tr = 0; tr < 64; ++tr) {
      const uint32_t av = all & ~(1u << eloc);
      const int s = kth_bit(av, draw((uint32_t)popc8(av)));
      const uint32_t avd = all & ~(1u << edest) & ~(1u << s);
      const int d = kth_bit(avd, draw((uint32_t)popc8(avd)));
      ov = make_vehicle(g, s, d);
      if (obs_key_fast(m, ev, ov) == obs) break;
    }
    *s0 = ego == 0 ? ev : ov;
    *s1 = ego == 0 ? ov : ev;
    return true;
  }
};

struct EnvPursuitEvasion {
  using Model = PeModel;
  static constexpr int kStepDraws = 0;
  static constexpr int kEnvId = POMCP_ENV_PURSUIT_EVASION;
  static constexpr int kA = 4;   // actions per agent

  __device__ static __forceinline__ void step(const Model& m, int ego, uint32_t s0, uint32_t s1,
                                              uint32_t a_ego, uint32_t a_oth, uint32_t /*j*/,
                                              uint32_t* n0, uint32_t* n1, double* r, int* done) {
    uint32_t prog, outcome;
    pe_step(m, s0, s1, ego == 0 ? a_ego : a_oth, ego == 0 ? a_oth : a_ego, n0, n1, &prog,
            &outcome);
    *r = pe_reward(m, ego, s0, prog, outcome);
    *done = done_of(ego, *n0, *n1);
  }
  __device__ static __forceinline__ int done_of(int /*ego*/, uint32_t n0, uint32_t /*n1*/) {
    return pe_done(n0) ? 1 : 0;   // both agents terminate together
  }
  __device__ static __forceinline__ uint64_t obs_key(const Model& m, int ego, uint32_t n0,
                                                     uint32_t n1) {
    return pe_obs_key(m, ego, n0, n1);
  }
  template <class Draw>
  __device__ static void sample_initial(const Model& m, Draw draw, uint32_t* s0, uint32_t* s1) {
    pe_sample_initial_state(m, draw, s0, s1);
  }
  template <class Draw>
  __device__ static bool sample_agent_initial(const Model& m, int ego, uint64_t obs, Draw draw,
                                              uint32_t* s0, uint32_t* s1) {
    return pe_sample_agent_initial(m, ego, obs, draw, s0, s1);
  }
};

template <class Model>
__device__ __forceinline__ void stage_model(const void* src, Model& dst) {
  static_assert(sizeof(Model) % 4 == 0, "model size");
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(&dst);
  for (int i = threadIdx.x; i < (int)(sizeof(Model) / 4); i += blockDim.x) d[i] = s[i];
  __syncthreads();
}

}  // namespace pb
