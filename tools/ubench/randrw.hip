// Random-line read-modify-write latency/throughput (diagnostic microbenchmark
// for the k_search tree layout).  One dependent chain per lane: every lane
// repeatedly picks a pseudo-random 128 B line, reads PARTS x 16 B of it (one
// dwordx4 per part, like k_search's per-lane block accesses), optionally
// writes it back, and derives the next address from the data.
//
// Address modes (buffer = 2^lg lines of 128 B, 65536 lanes):
//   0 "global":      any line of the buffer
//   1 "per-lane":    a lane's lines form its own contiguous region (k_search's
//                    [tree][block] arena layout)
//   2 "interleaved": line i of lane l of wave w at ((w * R + i) * 64 + l): the
//                    64 lanes of a wave share pages ([wave][block][lane])
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

template <int PARTS, int WPARTS, int MODE>
__global__ __launch_bounds__(256) void k_rw(uint4* buf, int lg, int lg_region, int iters, uint32_t* sink) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = gid & 63u, wave = gid >> 6;
  uint32_t x = gid * 0x9E3779B9u + 0x7F4A7C15u;
  uint32_t acc = 0;
  const uint64_t rmask = (1ull << lg_region) - 1;
  for (int i = 0; i < iters; ++i) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    uint64_t line;
    if (MODE == 0) line = ((uint64_t)x * 0x9E3779B1u) >> (64 - lg);
    else if (MODE == 1) line = ((uint64_t)gid << lg_region) | (x & rmask);
    else line = ((((uint64_t)wave << lg_region) | (x & rmask)) << 6) | lane;
    uint4* p = buf + line * 8;
    uint4 v[PARTS];
#pragma unroll
    for (int q = 0; q < PARTS; ++q) v[q] = p[q];
#pragma unroll
    for (int q = 0; q < PARTS; ++q) { v[q].x += 1; acc += v[q].y; }
#pragma unroll
    for (int q = 0; q < WPARTS; ++q) p[q] = v[q];   // write back the first WPARTS parts
    x += acc & 1;   // next address depends on the data: one chain per lane
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// Reads PARTS x 16 B and writes back 16 B to each of NW different 32 B
// sectors (parts 0, 2, 4, ..): partial-sector writes.
template <int PARTS, int NW>
__global__ __launch_bounds__(256) void k_rw_split(uint4* buf, int lg, int lg_region, int iters, uint32_t* sink) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = gid & 63u, wave = gid >> 6;
  uint32_t x = gid * 0x9E3779B9u + 0x7F4A7C15u;
  uint32_t acc = 0;
  const uint64_t rmask = (1ull << lg_region) - 1;
  for (int i = 0; i < iters; ++i) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const uint64_t line = ((((uint64_t)wave << lg_region) | (x & rmask)) << 6) | lane;
    uint4* p = buf + line * 8;
    uint4 v[PARTS];
#pragma unroll
    for (int q = 0; q < PARTS; ++q) v[q] = p[q];
#pragma unroll
    for (int q = 0; q < PARTS; ++q) { v[q].x += 1; acc += v[q].y; }
#pragma unroll
    for (int q = 0; q < NW; ++q) p[2 * q] = v[q];
    x += acc & 1;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// As k_rw, but each access's write-back is issued after the NEXT access's
// loads: on gfx9 (CDNA) stores count in vmcnt, so a wait for a load issued
// after a store also waits for the store's acknowledgement; deferring the
// store keeps it off the dependent chain.
template <int PARTS, int WPARTS, int MODE>
__global__ __launch_bounds__(256) void k_rw_defer(uint4* buf, int lg, int lg_region, int iters, uint32_t* sink) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = gid & 63u, wave = gid >> 6;
  uint32_t x = gid * 0x9E3779B9u + 0x7F4A7C15u;
  uint32_t acc = 0;
  const uint64_t rmask = (1ull << lg_region) - 1;
  auto addr = [&]() {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    uint64_t line;
    if (MODE == 0) line = ((uint64_t)x * 0x9E3779B1u) >> (64 - lg);
    else if (MODE == 1) line = ((uint64_t)gid << lg_region) | (x & rmask);
    else line = ((((uint64_t)wave << lg_region) | (x & rmask)) << 6) | lane;
    return buf + line * 8;
  };
  uint4* p = addr();
  uint4 v[PARTS];
#pragma unroll
  for (int q = 0; q < PARTS; ++q) v[q] = p[q];
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int q = 0; q < PARTS; ++q) { v[q].x += 1; acc += v[q].y; }
    x += acc & 1;
    uint4* const pn = addr();
    uint4 vn[PARTS];
#pragma unroll
    for (int q = 0; q < PARTS; ++q) vn[q] = pn[q];
#pragma unroll
    for (int q = 0; q < WPARTS; ++q) p[q] = v[q];   // the previous access's write-back
#pragma unroll
    for (int q = 0; q < PARTS; ++q) v[q] = vn[q];
    p = pn;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// Cooperative line load: the 64 lanes of a wave fetch the 64 lanes' 128 B
// lines 8 at a time -- in load j lane l reads 16 B part (l % 8) of the line of
// lane 8 j + l / 8 -- so each load instruction touches 8 lines instead of 64;
// the parts are regrouped per lane through LDS.  Same bytes, 8x fewer lines per
// instruction (address processing, translation).
template <int MODE>
__global__ __launch_bounds__(256) void k_coop(uint4* buf, int lg, int lg_region, int iters, uint32_t* sink) {
  __shared__ uint4 lds[4][64][9];   // [wave in block][lane][part] (+1: bank spread)
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = gid & 63u, wave = gid >> 6, wib = threadIdx.x >> 6;
  uint32_t x = gid * 0x9E3779B9u + 0x7F4A7C15u;
  uint32_t acc = 0;
  const uint64_t rmask = (1ull << lg_region) - 1;
  for (int i = 0; i < iters; ++i) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    uint64_t line;
    if (MODE == 0) line = ((uint64_t)x * 0x9E3779B1u) >> (64 - lg);
    else if (MODE == 1) line = ((uint64_t)gid << lg_region) | (x & rmask);
    else line = ((((uint64_t)wave << lg_region) | (x & rmask)) << 6) | lane;
    const int lo = (int)(uint32_t)line, hi = (int)(uint32_t)(line >> 32);
    uint4 got[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int src = 8 * j + (int)(lane >> 3);
      const uint64_t l2 = (uint64_t)(uint32_t)__shfl(lo, src) | ((uint64_t)(uint32_t)__shfl(hi, src) << 32);
      got[j] = buf[l2 * 8 + (lane & 7u)];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[wib][8 * j + (lane >> 3)][lane & 7u] = got[j];
    __builtin_amdgcn_wave_barrier();
    uint4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = lds[wib][lane][q];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 8; ++q) { v[q].x += 1; acc += v[q].y; }
    x += acc & 1;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int lg_region = argc > 1 ? atoi(argv[1]) : 10;   // lines per lane region (log2)
  uint4* buf; uint32_t* sink;
  const int lanes = 65536;
  const int lg = 16 + lg_region;   // total lines
  const uint64_t nlines = 1ull << lg;
  if (hipMalloc(&buf, nlines * 128) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMalloc(&sink, 4);
  hipMemset(buf, 0, nlines * 128);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 2000;
  printf("buffer %.2f GB, %d lanes, region %d lines (%d KB) per lane\n", nlines * 128 / 1e9, lanes,
         1 << lg_region, (1 << lg_region) * 128 / 1024);
  auto run = [&](const char* name, void (*k)(uint4*, int, int, int, uint32_t*), int bytes, int rw) {
    hipLaunchKernelGGL(k, dim3(lanes / 256), dim3(256), 0, 0, buf, lg, lg_region, 50, sink);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(lanes / 256), dim3(256), 0, 0, buf, lg, lg_region, iters, sink);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    const double acc = (double)lanes * iters;
    printf("%-22s %6.2f G acc/s  %6.2f us/access/lane  useful %7.1f GB/s\n", name, acc / ms / 1e6,
           ms * 1e3 / iters, acc * bytes * rw / ms / 1e6);
  };
  // bytes column: bytes read + written per access (useful bytes)
  run("global r16", k_rw<1, 0, 0>, 16, 1);
  run("global r128(8x16B)", k_rw<8, 0, 0>, 128, 1);
  run("global rw112(7x16B)", k_rw<7, 7, 0>, 112, 2);
  run("per-lane r16", k_rw<1, 0, 1>, 16, 1);
  run("per-lane r128", k_rw<8, 0, 1>, 128, 1);
  run("per-lane rw112", k_rw<7, 7, 1>, 112, 2);
  run("interleaved r16", k_rw<1, 0, 2>, 16, 1);
  run("interleaved r128", k_rw<8, 0, 2>, 128, 1);
  run("interleaved rw112", k_rw<7, 7, 2>, 112, 2);
  // k_search's own shapes (FETCH_SIZE / WRITE_SIZE calibration, tools/calib_fetch.sh):
  // the node statistics line (5 x 16 B), the chosen action's line (7 x 16 B),
  // and a line read then one 16 B part written back (the backup)
  run("interleaved r80", k_rw<5, 0, 2>, 80, 1);
  run("interleaved r112", k_rw<7, 0, 2>, 112, 1);
  run("interleaved r112w16", k_rw<7, 1, 2>, 128, 1);
  run("interleaved r112w16 defer", k_rw_defer<7, 1, 2>, 128, 1);
  run("interleaved r112w32", k_rw<7, 2, 2>, 144, 1);       // one full 32 B sector
  run("interleaved r112w16x2", k_rw_split<7, 2>, 144, 1);  // two half sectors
  run("interleaved r112w64", k_rw<7, 4, 2>, 176, 1);
  run("interleaved rw112 defer", k_rw_defer<7, 7, 2>, 112, 2);
  run("global r128 coop", k_coop<0>, 128, 1);
  run("per-lane r128 coop", k_coop<1>, 128, 1);
  run("interleaved r128 coop", k_coop<2>, 128, 1);
  return 0;
}
