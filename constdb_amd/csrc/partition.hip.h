// Bucket partition (MSD multisplit) and device-wide scans for gfx950.
//
// A row family (key rows, node rows, member rows — each a set of u64 SoA columns) is
// split into NB buckets by floor(h * NB / 2^64) of column 0 (the key hash kh, or the parent
// key hash pkh for children), so a key and all its children share a bucket. NB is a
// product of per-level digit counts <= 512: each level is one streaming pass (histogram pass over col 0,
// then a scatter pass that stages every column through LDS so that writes leave the CU
// as contiguous per-digit runs). The last level moves only a u32 row index (a
// permutation): its segments are ~1000 rows, so the bucket kernels' gathers through the
// permutation hit rows that are L2/MALL resident instead of re-streaming every column. Rows inside a bucket end up in arbitrary order; the
// bucket kernel sorts them by full identity, so results stay deterministic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cdb {
namespace {  // internal linkage: included by several translation units

constexpr int kPartThreads = 1024;
constexpr int kPartTile = 8192;       // rows staged through LDS at once (one sub-tile)
constexpr int kPartRowsPerThread = kPartTile / kPartThreads;
constexpr int kPartLocalMax = 2048;   // local (tile) bucket slots held in LDS
constexpr int kPF = 2;                // partition scatter: columns prefetched ahead

// 16 bytes at an 8-byte aligned address (records rows)
typedef unsigned long long ul2a8 __attribute__((ext_vector_type(2), aligned(8)));

template <int NC>
struct ColSet {
  uint64_t* c[NC];
  uint32_t s[NC];  // row stride of column k in words (0 = 1: a plain column; records layout, common.h)
  __device__ __forceinline__ uint64_t at(int k, uint64_t i) const { return c[k][s[k] ? i * s[k] : i]; }
  __device__ __forceinline__ const uint64_t* ptr(int k, uint64_t i) const { return &c[k][s[k] ? i * s[k] : i]; }
  __device__ __forceinline__ uint64_t& ref(int k, uint64_t i) const { return c[k][s[k] ? i * s[k] : i]; }
  // a streamed read of column k: non-temporal for a plain column (each line is read once); a
  // records field shares its line with the record's other fields, read by the next loads, so that
  // line must stay cached
  __device__ __forceinline__ uint64_t stream(int k, uint64_t i) const {
    return s[k] > 1 ? *ptr(k, i) : __builtin_nontemporal_load(ptr(k, i));
  }
};

// Bucket index of hash h among `nb` buckets: floor(h * nb / 2^64). Monotone in h, so for
// N_{l+1} = N_l * d the level-(l+1) buckets refine the level-l ones (MSD partition with
// bucket counts that need not be powers of two).
__device__ __forceinline__ uint64_t bucket_of_n(uint64_t h, uint64_t nb) { return __umul64hi(h, nb); }

// ---------------------------------------------------------------- histogram
// hist[gb] += number of rows in bucket gb. Rows arrive grouped by their previous-level
// bucket, so a workgroup's kPartTile rows span few parents and count in LDS; one global
// atomic per (workgroup, touched bucket).
__global__ void __launch_bounds__(kPartThreads) part_hist_kernel(const uint64_t* __restrict__ col0, uint64_t n,
                                                                 uint64_t nprev, uint32_t d, int shift,
                                                                 uint32_t* __restrict__ hist) {
  __shared__ uint32_t cnt[kPartLocalMax];
  const uint64_t tile0 = (uint64_t)blockIdx.x * kPartTile;
  if (tile0 >= n) return;
  const uint64_t tile1 = tile0 + kPartTile < n ? tile0 + kPartTile : n;
  const uint64_t ncur = nprev * d;
  const uint64_t plo = bucket_of_n(col0[tile0] << shift, nprev);
  const uint64_t phi = bucket_of_n(col0[tile1 - 1] << shift, nprev);
  const uint64_t glo = plo * d;
  const uint64_t span = (phi - plo + 1) * d;
  const bool local = span <= (uint64_t)kPartLocalMax;
  for (int i = threadIdx.x; i < kPartLocalMax; i += kPartThreads) cnt[i] = 0;
  __syncthreads();
  for (uint64_t r = tile0 + threadIdx.x; r < tile1; r += kPartThreads) {
    const uint64_t gb = bucket_of_n(col0[r] << shift, ncur);
    if (local) atomicAdd(&cnt[gb - glo], 1u);
    else atomicAdd(&hist[gb], 1u);
  }
  __syncthreads();
  if (local)
    for (int i = threadIdx.x; i < (int)span; i += kPartThreads)
      if (cnt[i]) atomicAdd(&hist[glo + i], cnt[i]);
}

// Exclusive scan of a[0..span) in place by the first wave; returns nothing (LDS result).
__device__ __forceinline__ void wave0_exclusive_scan(uint32_t* a, int span) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int per = (span + 63) / 64;
    uint32_t s = 0;
    for (int j = 0; j < per; ++j) {
      const int i = lane * per + j;
      if (i < span) s += a[i];
    }
    uint32_t incl = s;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    uint32_t run = incl - s;
    for (int j = 0; j < per; ++j) {
      const int i = lane * per + j;
      if (i < span) {
        const uint32_t c = a[i];
        a[i] = run;
        run += c;
      }
    }
  }
}

// ---------------------------------------------------------------- scatter
// Moves every column of every row of a kPartTile tile to its bucket's range (one global
// atomic per (tile, touched bucket) reserves it). Columns are staged through LDS in bucket
// order so that each wave's stores are contiguous runs; column c + kPF is requested before
// column c is staged. IDX: index-only final level — writes the u32 row index (to perm)
// instead of moving the NC columns.
template <int NC, bool IDX = false>
__global__ void __launch_bounds__(kPartThreads) part_scatter_kernel(ColSet<NC> in, ColSet<NC> out, uint64_t n,
                                                                    uint64_t nprev, uint32_t d, int shift,
                                                                    uint32_t* __restrict__ cursor,
                                                                    uint32_t* __restrict__ perm = nullptr) {
  __shared__ uint32_t cnt[kPartLocalMax];   // per local bucket: count, then its exclusive scan
  __shared__ uint32_t delta[kPartLocalMax]; // global row of staged slot j = delta[bucket] + j
  __shared__ uint16_t slot_lb[kPartTile];   // local bucket of each staged slot
  __shared__ uint64_t stage[kPartTile];
  const uint64_t tile0 = (uint64_t)blockIdx.x * kPartTile;
  if (tile0 >= n) return;
  const uint64_t tile1 = tile0 + kPartTile < n ? tile0 + kPartTile : n;
  const int rows = (int)(tile1 - tile0);
  const uint64_t ncur = nprev * d;
  const uint64_t plo = bucket_of_n(in.at(0, tile0) << shift, nprev);
  const uint64_t phi = bucket_of_n(in.at(0, tile1 - 1) << shift, nprev);
  const uint64_t glo = plo * d;
  const uint64_t span64 = (phi - plo + 1) * d;

  if (span64 > (uint64_t)kPartLocalMax) {  // wide tile: per-row global reservation
    for (int r = threadIdx.x; r < rows; r += kPartThreads) {
      const uint64_t gb = bucket_of_n(in.at(0, tile0 + r) << shift, ncur);
      const uint32_t p = atomicAdd(&cursor[gb], 1u);
      if (IDX) {
        perm[p] = (uint32_t)(tile0 + r);
      } else {
#pragma unroll
        for (int c = 0; c < NC; ++c) out.ref(c, p) = in.at(c, tile0 + r);
      }
    }
    return;
  }
  const int span = (int)span64;
  for (int i = threadIdx.x; i < span; i += kPartThreads) cnt[i] = 0;
  constexpr int NV = IDX ? 1 : NC;
  uint64_t v[NV][kPartRowsPerThread];
  auto load_col = [&](int c) {
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      const int r = threadIdx.x + k * kPartThreads;
      v[c][k] = r < rows ? in.stream(c, tile0 + r) : 0;
    }
  };
#pragma unroll
  for (int c = 0; c < (NV < kPF ? NV : kPF); ++c) load_col(c);
  __syncthreads();
  uint16_t lb[kPartRowsPerThread];
  uint32_t rk[kPartRowsPerThread];
#pragma unroll
  for (int k = 0; k < kPartRowsPerThread; ++k) {
    const int r = threadIdx.x + k * kPartThreads;
    if (r < rows) {
      lb[k] = (uint16_t)(bucket_of_n(v[0][k] << shift, ncur) - glo);
      rk[k] = atomicAdd(&cnt[lb[k]], 1u);
    }
  }
  __syncthreads();
  // reserve each touched bucket's range, then scan the counts
  for (int i = threadIdx.x; i < span; i += kPartThreads) delta[i] = cnt[i] ? atomicAdd(&cursor[glo + i], cnt[i]) : 0;
  __syncthreads();
  wave0_exclusive_scan(cnt, span);
  __syncthreads();
  for (int i = threadIdx.x; i < span; i += kPartThreads) delta[i] -= cnt[i];
  uint32_t slot[kPartRowsPerThread];
#pragma unroll
  for (int k = 0; k < kPartRowsPerThread; ++k) {
    const int r = threadIdx.x + k * kPartThreads;
    if (r < rows) {
      slot[k] = cnt[lb[k]] + rk[k];
      slot_lb[slot[k]] = lb[k];
    }
  }
  __syncthreads();
  if (IDX) {
    uint32_t* st32 = reinterpret_cast<uint32_t*>(stage);
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      const int r = threadIdx.x + k * kPartThreads;
      if (r < rows) st32[slot[k]] = (uint32_t)(tile0 + r);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < rows; j += kPartThreads) perm[delta[slot_lb[j]] + j] = st32[j];
    return;
  }
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    if (c + kPF < NV) load_col(c + kPF < NV ? c + kPF : 0);
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      const int r = threadIdx.x + k * kPartThreads;
      if (r < rows) stage[slot[k]] = v[c][k];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < rows; j += kPartThreads) out.ref(c, delta[slot_lb[j]] + j) = stage[j];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- scatter to rows (AoS)
// The last column-moving level: the same multisplit, but each row leaves as one W-word record
// (W = 8 for key rows, whose 8th word is zero padding: one aligned 64-B line per row; W = 6 for
// child rows) and column 0 also goes to `khcol` for the index level. The bucket kernels then
// fetch a row with 16-B loads from one or two lines instead of one gathered line per column.
// Rows are staged whole through LDS (2048-row tiles) and leave as 16-B pieces, W/2 lanes per
// row, so each store instruction writes whole rows of one digit run.
// TILE = 1024 (two workgroups per CU, so one's barriers and scan overlap the other's memory
// traffic) or 2048 (one workgroup per CU, longer per-digit runs); LMAX = local digit slots.
template <int NC, int W, int TILE = 1024, int LMAX = 1024>
__global__ void __launch_bounds__(kPartThreads) part_scatter_aos_kernel(ColSet<NC> in, uint64_t* __restrict__ aos,
                                                                        uint64_t* __restrict__ khcol, uint64_t n,
                                                                        uint64_t nprev, uint32_t d, int shift,
                                                                        uint32_t* __restrict__ cursor,
                                                                        uint16_t* __restrict__ dig = nullptr,
                                                                        uint32_t d1 = 0) {
  // dig != nullptr (a per-segment final level follows): instead of the key-hash column, each
  // row's digit inside its segment, floor(h * ncur * d1 / 2^64) - segment * d1, as a u16.
  static_assert(W % 2 == 0 && W >= NC, "rows leave as 16-B pieces");
  constexpr int kAosTile = TILE;
  constexpr int kLocal = LMAX;
  constexpr int RPT = (kAosTile + kPartThreads - 1) / kPartThreads;
  __shared__ uint32_t cnt[kLocal];
  __shared__ uint32_t delta[kLocal];
  __shared__ uint16_t slot_lb[kAosTile];
  __shared__ __attribute__((aligned(16))) uint64_t stage[kAosTile * W];
  const uint64_t tile0 = (uint64_t)blockIdx.x * kAosTile;
  if (tile0 >= n) return;
  const uint64_t tile1 = tile0 + kAosTile < n ? tile0 + kAosTile : n;
  const int rows = (int)(tile1 - tile0);
  const uint64_t ncur = nprev * d;
  const uint64_t plo = bucket_of_n(in.at(0, tile0) << shift, nprev);
  const uint64_t phi = bucket_of_n(in.at(0, tile1 - 1) << shift, nprev);
  const uint64_t glo = plo * d;
  const uint64_t span64 = (phi - plo + 1) * d;

  if (span64 > (uint64_t)kLocal) {  // wide tile: per-row global reservation
    for (int r = threadIdx.x; r < rows; r += kPartThreads) {
      const uint64_t h = in.at(0, tile0 + r);
      const uint64_t gb = bucket_of_n(h << shift, ncur);
      const uint32_t p = atomicAdd(&cursor[gb], 1u);
#pragma unroll
      for (int c = 0; c < W; ++c) aos[(uint64_t)p * W + c] = c < NC ? in.at(c < NC ? c : 0, tile0 + r) : 0;
      if (dig) dig[p] = (uint16_t)(bucket_of_n(h << shift, ncur * d1) - gb * d1);
      else khcol[p] = h;
    }
    return;
  }
  const int span = (int)span64;
  for (int i = threadIdx.x; i < span; i += kPartThreads) cnt[i] = 0;
  uint64_t v0[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = threadIdx.x + k * kPartThreads;
    v0[k] = r < rows ? __builtin_nontemporal_load(in.ptr(0, tile0 + r)) : 0;
  }
  __syncthreads();
  uint16_t lb[RPT];
  uint32_t rk[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = threadIdx.x + k * kPartThreads;
    if (r < rows) {
      lb[k] = (uint16_t)(bucket_of_n(v0[k] << shift, ncur) - glo);
      rk[k] = atomicAdd(&cnt[lb[k]], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < span; i += kPartThreads) delta[i] = cnt[i] ? atomicAdd(&cursor[glo + i], cnt[i]) : 0;
  __syncthreads();
  wave0_exclusive_scan(cnt, span);
  __syncthreads();
  for (int i = threadIdx.x; i < span; i += kPartThreads) delta[i] -= cnt[i];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = threadIdx.x + k * kPartThreads;
    if (r < rows) {
      const uint32_t s = cnt[lb[k]] + rk[k];
      slot_lb[s] = lb[k];
      uint64_t* row = &stage[(uint32_t)s * W];
      row[0] = v0[k];
      if (in.s[1] > 1) {  // (uniform) records: the row's NC - 1 record words in 16-B pieces (8-B aligned)
        const uint64_t* rec = in.ptr(1, tile0 + r);
#pragma unroll
        for (int c = 1; c + 1 < NC; c += 2) {
          const ul2a8 q = *reinterpret_cast<const ul2a8*>(rec + (c - 1));
          row[c] = q.x;
          row[c + 1] = q.y;
        }
        if ((NC - 1) & 1) row[NC - 1] = rec[NC - 2];
#pragma unroll
        for (int c = NC; c < W; ++c) row[c] = 0;
      } else {
#pragma unroll
        for (int c = 1; c < W; ++c) row[c] = c < NC ? __builtin_nontemporal_load(in.ptr(c < NC ? c : 0, tile0 + r)) : 0;
      }
    }
  }
  __syncthreads();
  constexpr int Q = W / 2;  // 16-B pieces per row
  for (int i = threadIdx.x; i < rows * Q; i += kPartThreads) {
    const int j = i / Q, q = i - j * Q;
    const uint64_t dst = (uint64_t)(delta[slot_lb[j]] + (uint32_t)j) * W + 2 * q;
    *reinterpret_cast<ulonglong2*>(&aos[dst]) = *reinterpret_cast<const ulonglong2*>(&stage[j * W + 2 * q]);
  }
  if (dig) {
    for (int j = threadIdx.x; j < rows; j += kPartThreads) {
      const uint64_t gb = glo + slot_lb[j];
      dig[delta[slot_lb[j]] + j] = (uint16_t)(bucket_of_n(stage[j * W] << shift, ncur * d1) - gb * d1);
    }
  } else {
    for (int j = threadIdx.x; j < rows; j += kPartThreads) khcol[delta[slot_lb[j]] + j] = stage[j * W];
  }
}

// ---------------------------------------------------------------- final level, per segment
// The last (index-only) level when it follows a row level of large fan-out: segment s (the
// rows of row-level bucket s, contiguous in `khcol` order) is split into d1 buckets by ONE
// workgroup: an LDS histogram of the segment, its scan (the bucket directory of the segment,
// written straight to base_out / hist_out), and an LDS-cursor scatter of row indices into
// perm. No global histogram pass, no device-wide scan, no global atomics; the row level left
// each row's digit as a u16, read twice (2 B per row each time).
constexpr int kFinalThreads = 1024;
constexpr int kFinalMaxD = 16384;

__global__ void __launch_bounds__(kFinalThreads) part_final_kernel(const uint16_t* __restrict__ dig,
                                                                   const uint32_t* __restrict__ sbase,
                                                                   const uint32_t* __restrict__ scnt, uint64_t nseg,
                                                                   uint32_t d1,
                                                                   uint32_t* __restrict__ base_out,
                                                                   uint32_t* __restrict__ hist_out,
                                                                   uint32_t* __restrict__ perm) {
  __shared__ uint32_t cnt[kFinalMaxD];
  __shared__ uint32_t part[kFinalThreads / 64];
  const uint32_t s = blockIdx.x;
  const uint32_t b0 = sbase[s], n = scnt[s];
  const uint64_t g0 = (uint64_t)s * d1;
  for (uint32_t j = threadIdx.x; j < d1; j += kFinalThreads) cnt[j] = 0;
  __syncthreads();
  // 8 independent loads in flight per thread, then their LDS atomics
  constexpr int U = 8;
  for (uint32_t i0 = 0; i0 < n; i0 += U * kFinalThreads) {
    uint32_t h[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kFinalThreads + threadIdx.x;
      h[u] = i < n ? dig[b0 + i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * kFinalThreads + threadIdx.x < n) atomicAdd(&cnt[h[u]], 1u);
  }
  __syncthreads();
  // exclusive scan of cnt[0 .. d1): thread t owns a run of `per` consecutive entries
  const uint32_t per = (d1 + kFinalThreads - 1) / kFinalThreads;
  const uint32_t j0 = threadIdx.x * per, j1 = min(d1, j0 + per);
  uint32_t run = 0;
  for (uint32_t j = j0; j < j1; ++j) run += cnt[j];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = run;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) part[w] = incl;
  __syncthreads();
  uint32_t off = incl - run;
  for (int k = 0; k < w; ++k) off += part[k];
  for (uint32_t j = j0; j < j1; ++j) {
    const uint32_t c = cnt[j];
    hist_out[g0 + j] = c;
    base_out[g0 + j] = b0 + off;
    cnt[j] = off;  // becomes the bucket's cursor
    off += c;
  }
  __syncthreads();
  for (uint32_t i0 = 0; i0 < n; i0 += U * kFinalThreads) {
    uint32_t h[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kFinalThreads + threadIdx.x;
      h[u] = i < n ? dig[b0 + i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kFinalThreads + threadIdx.x;
      if (i < n) perm[b0 + atomicAdd(&cnt[h[u]], 1u)] = b0 + i;
    }
  }
}

// ---------------------------------------------------------------- scans
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;  // items per thread
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint64_t block_exclusive_scan_u64(uint64_t v, uint64_t* total) {
  __shared__ uint64_t warp_sums[kScanThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) warp_sums[w] = incl;
  __syncthreads();
  uint64_t off = 0, tot = 0;
  for (int i = 0; i < kScanThreads / 64; ++i) {
    if (i < w) off += warp_sums[i];
    tot += warp_sums[i];
  }
  __syncthreads();
  *total = tot;
  return off + incl - v;
}

// pass 1: per-tile sums
template <typename T>
__global__ void __launch_bounds__(kScanThreads) scan_reduce_kernel(const T* __restrict__ in, uint64_t n,
                                                                   uint64_t* __restrict__ sums) {
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint64_t s = 0;
  for (int k = 0; k < kScanItems; ++k) {
    const uint64_t i = base + (uint64_t)threadIdx.x * kScanItems + k;
    if (i < n) s += in[i];
  }
  uint64_t tot;
  block_exclusive_scan_u64(s, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// pass 2: exclusive scan of the tile sums (one workgroup, sequential over chunks)
__global__ void __launch_bounds__(kScanThreads) scan_sums_kernel(uint64_t* __restrict__ sums, uint64_t m,
                                                                 uint64_t* __restrict__ grand_total) {
  uint64_t carry = 0;
  for (uint64_t b = 0; b < m; b += kScanThreads) {
    const uint64_t i = b + threadIdx.x;
    const uint64_t v = i < m ? sums[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan_u64(v, &tot);
    if (i < m) sums[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && grand_total) *grand_total = carry;
}

// pass 3: out[i] = exclusive prefix (as OutT); optionally copies it to out2 as well
template <typename T, typename OutT>
__global__ void __launch_bounds__(kScanThreads) scan_apply_kernel(const T* __restrict__ in, uint64_t n,
                                                                  const uint64_t* __restrict__ sums,
                                                                  OutT* __restrict__ out, OutT* __restrict__ out2) {
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  T v[kScanItems];
  uint64_t s = 0;
  for (int k = 0; k < kScanItems; ++k) {
    const uint64_t i = base + (uint64_t)threadIdx.x * kScanItems + k;
    v[k] = i < n ? in[i] : 0;
    s += v[k];
  }
  uint64_t tot;
  uint64_t run = sums[blockIdx.x] + block_exclusive_scan_u64(s, &tot);
  for (int k = 0; k < kScanItems; ++k) {
    const uint64_t i = base + (uint64_t)threadIdx.x * kScanItems + k;
    if (i < n) {
      out[i] = (OutT)run;
      if (out2) out2[i] = (OutT)run;
    }
    run += v[k];
  }
}

}  // namespace
}  // namespace cdb
