// host_exp(x): bit-identical restatement of the exp() that Python's math.exp
// calls on this image -- glibc 2.35's table-driven exp (since glibc 2.28), in
// its x86-64 FMA variant, which the libm ifunc selects on every CPU with FMA
// and AVX2 (the container's Xeon and the GPU box's host alike).
//
// Why: I-NTMCP's other-agent policy is a softmax over math.exp(visits / sqrt(N))
// (intmcp.py:782-790); the device's own exp is not glibc's and differs by 1 ulp
// on ~6% of arguments, and one flipped random.choices bisection diverges a
// whole episode.  Parity needs exactly glibc's rounding.
//
// Algorithm (published glibc design, restated): x = k ln2/128 + r with
// k = round(x * 128/ln2), exp(x) = 2^(k/128) * exp(r); 2^(k/128) from a 128-entry
// table (host_exp_table.h: computed from its definition, checked equal to the
// host libm's), exp(r) - 1 by a degree-5 polynomial.  The operation order --
// which products are fused into FMAs -- is the one the x86-64 FMA build
// executes (read off its machine code): kd = fma(x, N/ln2, shift);
// r = fma(kd', -ln2lo/N, fma(kd', -ln2hi/N, x)); tmp = fma(r2 * r2,
// fma(r, C5, C4), fma(fma(r, C3, C2), r2, r + tail)); result =
// fma(scale, tmp, scale).  Special cases (|x| < 2^-54, |x| >= 512, inf/nan)
// follow the same code.  Checked against math.exp over millions of arguments
// on the host (tests/test_host_exp.py) and on the GPU (tests/test_gpu_intmcp.py).
#pragma once
#include <stdint.h>
#include <string.h>

#include "host_exp_table.h"

namespace pb {

__host__ __device__ inline uint64_t hx_bits(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
__host__ __device__ inline double hx_dbl(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}
__host__ __device__ inline double hx_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// |x| >= 512: the scale's exponent is adjusted to stay representable.
__host__ __device__ inline double host_exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {                       // k > 0
    sbits -= 1009ull << 52;
    const double scale = hx_dbl(sbits);
    return hx_fma(scale, tmp, scale) * 0x1p1009;
  }
  sbits += 1022ull << 52;                                // k < 0 (subnormal range)
  const double scale = hx_dbl(sbits);
  const double st = scale * tmp;                         // not fused in this branch
  double y = scale + st;
  if (y < 1.0) {
    double lo = (scale - y) + st;
    const double hi = 1.0 + y;
    lo = ((1.0 - hi) + y) + lo;
    y = (lo + hi) - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return y * 0x1p-1022;
}

// tab: kHostExpTab or a copy of it (a kernel may stage it in LDS: the
// lookup is otherwise a dependent global load per exp)
__host__ __device__ inline double host_exp_tab(double x, const uint64_t* tab) {
  constexpr double kInvLn2N = 0x1.71547652b82fep7;    // 128 / ln 2
  constexpr double kShift = 0x1.8p52;
  constexpr double kNegLn2hiN = -0x1.62e42fefa0000p-8;
  constexpr double kNegLn2loN = -0x1.cf79abc9e3b3ap-47;
  constexpr double kC2 = 0x1.ffffffffffdbdp-2;
  constexpr double kC3 = 0x1.555555555543cp-3;
  constexpr double kC4 = 0x1.55555cf172b91p-5;
  constexpr double kC5 = 0x1.1111167a4d017p-7;
  const uint64_t ux = hx_bits(x);
  uint32_t abstop = (uint32_t)(ux >> 52) & 0x7ffu;
  if (abstop - 0x3c9u >= 0x3fu) {                        // |x| < 2^-54 or |x| >= 512
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;
    if (abstop >= 0x409u) {                              // |x| >= 1024
      if (ux == 0xfff0000000000000ull) return 0.0;
      if (abstop >= 0x7ffu) return 1.0 + x;
      return (ux >> 63) ? 0.0 : __builtin_inf();
    }
    abstop = 0;                                          // 512 <= |x| < 1024
  }
  const double kraw = hx_fma(x, kInvLn2N, kShift);
  const uint64_t ki = hx_bits(kraw);
  const double kd = kraw - kShift;
  const double r = hx_fma(kd, kNegLn2loN, hx_fma(kd, kNegLn2hiN, x));
  const uint32_t idx = 2u * (uint32_t)(ki & 127u);
  const uint64_t top = ki << 45;
  const double tail = hx_dbl(tab[idx]);
  const uint64_t sbits = tab[idx + 1] + top;
  const double r2 = r * r;
  const double p23 = hx_fma(r, kC3, kC2);
  const double p45 = hx_fma(r, kC5, kC4);
  const double tmp = hx_fma(r2 * r2, p45, hx_fma(p23, r2, r + tail));
  if (abstop == 0) return host_exp_special(tmp, sbits, ki);
  const double scale = hx_dbl(sbits);
  return hx_fma(scale, tmp, scale);
}

__host__ __device__ inline double host_exp(double x) { return host_exp_tab(x, kHostExpTab); }

}  // namespace pb
