// Stable LSD radix sort of (u64 key, u32 value) pairs for gfx950, 8-bit digits, one pass per digit:
//   radix_hist_kernel:    per tile of kRadixTile pairs, the 256-bin digit histogram, stored
//                         digit-major (hist[d * tiles + t]) so that one exclusive scan over the
//                         whole array gives every (digit, tile) its first output slot;
//   radix_scatter_kernel: each tile loads its pairs at once (every load in flight), ranks them
//                         stably (wave ballots find the lanes holding the same digit; per-digit
//                         running counts in LDS carry the order from one 256-pair round to the
//                         next) into an LDS copy of the tile in digit order, and writes each
//                         digit's run to its slots contiguously.
// Used by the over-capacity bucket path (hot.hip.h), where a few keys own millions of children.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cdb {

constexpr int kRadixThreads = 512;
constexpr int kRadixRounds = 8;
constexpr int kRadixTile = kRadixThreads * kRadixRounds;  // 4096 pairs per tile

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

// (Prefetching the tile's digits, wave-aggregated atomics and 16 tiles per block with runs of
// adjacent counts all measured slower on C5's 52M tags: 164-190 against 139 us.)
__global__ void __launch_bounds__(kRadixThreads) radix_hist_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                                   int shift, uint32_t* __restrict__ hist,
                                                                   uint32_t tiles) {
  __shared__ uint32_t cnt[256];
  if (threadIdx.x < 256) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kRadixTile;
  for (int r = 0; r < kRadixRounds; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kRadixThreads + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(uint32_t)(keys[i] >> shift) & 0xFF], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 256) hist[(uint64_t)threadIdx.x * tiles + blockIdx.x] = cnt[threadIdx.x];
}

__global__ void __launch_bounds__(kRadixThreads) radix_scatter_kernel(const uint64_t* __restrict__ kin,
                                                                      const uint32_t* __restrict__ vin, uint64_t n,
                                                                      int shift, const uint32_t* __restrict__ base,
                                                                      uint32_t tiles, uint64_t* __restrict__ kout,
                                                                      uint32_t* __restrict__ vout) {
  constexpr int W = kRadixThreads / 64;
  __shared__ uint64_t sk[kRadixTile];  // the tile in digit order
  __shared__ uint32_t sv[kRadixTile];
  __shared__ uint32_t run[256];        // next tile slot of each digit
  __shared__ uint32_t lbase[256];      // first tile slot of each digit
  __shared__ uint32_t gbase[256];      // first output slot of the tile's pairs of each digit
  __shared__ uint32_t wcnt[W][256];    // this round: pairs of each digit per wave
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t t0 = (uint64_t)blockIdx.x * kRadixTile;
  const uint32_t cnt = (uint32_t)(n - t0 < (uint64_t)kRadixTile ? n - t0 : (uint64_t)kRadixTile);
  uint64_t kr[kRadixRounds];
  uint32_t vr[kRadixRounds];
#pragma unroll
  for (int r = 0; r < kRadixRounds; ++r) {  // every load of the tile in flight at once
    const uint32_t i = r * kRadixThreads + tid;
    kr[r] = i < cnt ? kin[t0 + i] : 0;
    vr[r] = i < cnt ? vin[t0 + i] : 0;
  }
  // this tile's pairs of digit tid (the scanned histogram's step to the next (digit, tile) slot),
  // scanned over the digits into first tile slots
  uint32_t c = 0, inc = 0;
  if (tid < 256) {
    const uint64_t idx = (uint64_t)tid * tiles + blockIdx.x;
    const uint32_t g = base[idx];
    c = (idx + 1 < 256ull * tiles ? base[idx + 1] : (uint32_t)n) - g;
    gbase[tid] = g;
    run[tid] = 0;
    inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, d);
      if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) wcnt[0][wv] = inc;
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t pre = inc - c;
    for (uint32_t k = 0; k < wv; ++k) pre += wcnt[0][k];
    lbase[tid] = pre;
  }
  const uint64_t lt = lane ? ((~0ull) >> (64 - lane)) : 0ull;
#pragma unroll
  for (int r = 0; r < kRadixRounds; ++r) {
    __syncthreads();
    for (uint32_t k = tid; k < W * 256; k += kRadixThreads) (&wcnt[0][0])[k] = 0;
    __syncthreads();
    const uint32_t i = r * kRadixThreads + tid;
    const bool valid = i < cnt;
    const uint32_t d = (uint32_t)(kr[r] >> shift) & 0xFF;
    const uint64_t m = radix_match(d, valid);
    const uint32_t below = (uint32_t)__popcll(m & lt);
    if (valid && below == 0) wcnt[wv][d] = (uint32_t)__popcll(m);  // the digit's first lane
    __syncthreads();
    if (valid) {
      uint32_t off = lbase[d] + run[d] + below;
      for (uint32_t w = 0; w < wv; ++w) off += wcnt[w][d];
      sk[off] = kr[r];
      sv[off] = vr[r];
    }
    __syncthreads();
    if (tid < 256) {
      uint32_t tot = 0;
      for (int w = 0; w < W; ++w) tot += wcnt[w][tid];
      run[tid] += tot;
    }
  }
  __syncthreads();
  for (uint32_t p = tid; p < cnt; p += kRadixThreads) {  // each digit's run written contiguously
    const uint64_t k = sk[p];
    const uint32_t d = (uint32_t)(k >> shift) & 0xFF;
    const uint32_t dst = gbase[d] + (p - lbase[d]);
    kout[dst] = k;
    vout[dst] = sv[p];
  }
}

}  // namespace cdb
