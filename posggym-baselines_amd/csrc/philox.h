// Philox4x32-7 counter-based RNG streams (host + device).
//
// Draw j of stream s under key (seed, tree) is word (j & 3) of
// philox4x32(ctr = {j >> 2, 0, s, seed >> 32}, key = {seed & 0xffffffff, tree}),
// Random123's Philox4x32 with 7 rounds (round 6 of the build; rounds 1-5 used
// 10).  Random123 (Salmon et al., SC'11) reports Philox4x32-7 passing TestU01's
// BigCrush with no failures ("Crush-resistant": 7 is the fewest rounds that
// do) and recommends 10 only as a safety margin; a planner's draws are
// simulation noise, not cryptography.  7 rounds are 30% less Philox work in
// k_search (10% of a simulation by phase timing: +3% measured); the Random123
// known answers for 7 and 10 rounds pin the function (tests/test_oracle.py).
// uniform int in [0, n) = (u32 * n) >> 32; uniform float = u32 * 2^-32.
// This is the build's definition of "the reference's RNG" (SURVEY Appendix B):
// every random draw on the hot path (planner Random(seed), global `random`,
// Discrete.sample() per agent, model RNG) is one stream.  Restated by
// oracle/rng.py for the CPU oracle; parity between the two is bit-exact.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PB_HD __host__ __device__ __forceinline__
#else
#define PB_HD inline
#endif

namespace pb {

enum Stream : uint32_t {
  S_BELIEF = 0,   // planner random.Random(seed): belief.sample(), rejection sampling
  S_SELECT = 1,   // global `random`: UCB/PUCB N==0, final tie-breaks
  S_MODEL = 2,    // model RNG: initial state sampling, execution-order shuffle
  S_BELIEF_NESTED = 3,  // I-NTMCP level-0 planner's random.Random(seed) (intmcp.py:66)
  S_MIXTURE = 4,  // other_policy.py `random`: OtherAgentMixturePolicy's policy draw (POTMMCP)
  S_BELIEF_MID = 5,  // I-NTMCP middle planners' random.Random(seed): level l on 5 + l - 1
                     // (5 at nesting level 2; 5, 6 at level 3)
  S_ACT_BASE = 8, // Discrete.sample() of agent i: 8 + i
  S_ENV_MODEL = 32,
  S_ENV_POLICY_BASE = 40,
};

// I-NTMCP: the middle planner of level l (1 <= l < the nesting level) draws its
// random.Random(seed) on S_BELIEF_MID + l - 1 for levels 1-3 (5, 6, 7) and on
// 16 + l beyond (20, 21: clear of the agents' action streams 8 + i); the
// oracle's belief_stream (oracle/intmcp.py) is the same map.
PB_HD constexpr uint32_t belief_mid_stream(int level) {
  return level <= 3 ? (uint32_t)S_BELIEF_MID + (uint32_t)level - 1u : 16u + (uint32_t)level;
}

// PB_PHILOX_ROUNDS: ablation builds only (tools/ablate.sh measures the RNG's
// share of k_search); any other value breaks parity with oracle/rng.py.
#ifndef PB_PHILOX_ROUNDS
#define PB_PHILOX_ROUNDS 7
#endif
PB_HD void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < PB_PHILOX_ROUNDS; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// Word j of stream s (stateless form).
PB_HD uint32_t philox_word(uint64_t seed, uint32_t tree, uint32_t s, uint32_t j) {
  uint32_t c[4] = {j >> 2, 0u, s, (uint32_t)(seed >> 32)};
  philox4x32(c, (uint32_t)seed, tree);
  return c[j & 3];
}

PB_HD uint32_t uniform_int(uint32_t u, uint32_t n) {
  return (uint32_t)(((uint64_t)u * (uint64_t)n) >> 32);
}

PB_HD double uniform_float(uint32_t u) { return (double)u * (1.0 / 4294967296.0); }

// One tree's key + per-stream counters.  Counter slots: 0 belief, 1 select,
// 2 model, 3 + i agent i's action space (2 agents).
struct Streams {
  uint64_t seed;
  uint32_t tree;
  uint32_t ctr[5];

  PB_HD uint32_t next(uint32_t slot, uint32_t stream) {
    const uint32_t j = ctr[slot]++;
    return philox_word(seed, tree, stream, j);
  }
  PB_HD uint32_t belief(uint32_t n) { return uniform_int(next(0, S_BELIEF), n); }
  PB_HD uint32_t select(uint32_t n) { return uniform_int(next(1, S_SELECT), n); }
  PB_HD double select_float() { return uniform_float(next(1, S_SELECT)); }
  PB_HD uint32_t model(uint32_t n) { return uniform_int(next(2, S_MODEL), n); }
  PB_HD uint32_t act(int agent, uint32_t n) {
    return uniform_int(agent == 0 ? next(3, S_ACT_BASE) : next(4, S_ACT_BASE + 1), n);
  }
};

}  // namespace pb
