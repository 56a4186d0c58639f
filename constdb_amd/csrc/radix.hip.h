// Stable LSD radix sort of (u64 key, u32 value) pairs for gfx950, 8-bit digits, one pass per digit:
//   radix_hist_kernel:    per tile of kRadixTile pairs, the 256-bin digit histogram, stored
//                         digit-major (hist[d * tiles + t]) so that one exclusive scan over the
//                         whole array gives every (digit, tile) its first output slot;
//   radix_scatter_kernel: each tile ranks its pairs stably (wave ballots find the lanes holding
//                         the same digit; a per-digit running count in LDS carries the order from
//                         one 256-pair round to the next) and writes them to their slots.
// Used by the over-capacity bucket path (hot.hip.h), where a few keys own millions of children.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cdb {

constexpr int kRadixThreads = 256;
constexpr int kRadixRounds = 16;
constexpr int kRadixTile = kRadixThreads * kRadixRounds;  // 4096 pairs per tile

__global__ void __launch_bounds__(kRadixThreads) radix_hist_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                                   int shift, uint32_t* __restrict__ hist,
                                                                   uint32_t tiles) {
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kRadixTile;
  for (int r = 0; r < kRadixRounds; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kRadixThreads + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(uint32_t)(keys[i] >> shift) & 0xFF], 1u);
  }
  __syncthreads();
  hist[(uint64_t)threadIdx.x * tiles + blockIdx.x] = cnt[threadIdx.x];
}

// Lanes of the calling wave whose digit equals mine (8 ballots over the digit's bits).
__device__ __forceinline__ uint64_t radix_match(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t bb = __ballot(valid && ((d >> b) & 1));
    m &= ((d >> b) & 1) ? bb : ~bb;
  }
  return m;
}

__global__ void __launch_bounds__(kRadixThreads) radix_scatter_kernel(const uint64_t* __restrict__ kin,
                                                                      const uint32_t* __restrict__ vin, uint64_t n,
                                                                      int shift, const uint32_t* __restrict__ base,
                                                                      uint32_t tiles, uint64_t* __restrict__ kout,
                                                                      uint32_t* __restrict__ vout) {
  constexpr int W = kRadixThreads / 64;
  __shared__ uint32_t run[256];      // pairs of each digit placed by earlier rounds of this tile
  __shared__ uint32_t wcnt[W][256];  // this round: pairs of each digit per wave
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  run[threadIdx.x] = base[(uint64_t)threadIdx.x * tiles + blockIdx.x];
  const uint64_t t0 = (uint64_t)blockIdx.x * kRadixTile;
  const uint64_t lt = lane ? ((~0ull) >> (64 - lane)) : 0ull;
  for (int r = 0; r < kRadixRounds; ++r) {
    for (int w = 0; w < W; ++w) wcnt[w][threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i = t0 + (uint64_t)r * kRadixThreads + threadIdx.x;
    const bool valid = i < n;
    const uint64_t k = valid ? kin[i] : 0;
    const uint32_t v = valid ? vin[i] : 0;
    const uint32_t d = (uint32_t)(k >> shift) & 0xFF;
    const uint64_t m = radix_match(d, valid);
    const uint32_t below = (uint32_t)__popcll(m & lt);
    if (valid && below == 0) wcnt[wv][d] = (uint32_t)__popcll(m);  // the digit's first lane
    __syncthreads();
    if (valid) {
      uint32_t off = run[d] + below;
      for (int w = 0; w < wv; ++w) off += wcnt[w][d];
      kout[off] = k;
      vout[off] = v;
    }
    __syncthreads();
    uint32_t tot = 0;
    for (int w = 0; w < W; ++w) tot += wcnt[w][threadIdx.x];
    run[threadIdx.x] += tot;
    __syncthreads();
  }
}

}  // namespace cdb
