// Sorted-run merge path (gfx950): inputs whose rows are already grouped into runs ordered by key
// hash -- one run per replica, as this engine's own merge output is (bucket order, then exact
// key-hash order inside a bucket) and as a snapshot written from it and decoded again is.
//
// The partition pass disappears: a bucket's rows are a few consecutive rows of every run.
//   1. run_mark_kernel: one streaming read of column 0 (the key hash; 8 B of each row) finds,
//      for every run and bucket, the run-relative first row of the bucket (the run directory,
//      run-major: rdir[r * (nb + 1) + b]), and verifies that every run is non-decreasing in
//      (hash << key_shift) -- a violation sends the merge to the partition path;
//   2. run_reduce_kernel: per bucket, the row count and the exclusive prefix over buckets (the
//      same bucket directory the partition path builds; the other tiers and the compaction
//      read it unchanged);
//   3. the wave / wide kernels read each bucket's rows straight from the caller's SoA columns,
//      lane by lane, consecutive rows of each run on consecutive lanes; buckets beyond a wave
//      are materialised as AoS rows + row indices (materialize_kernel), the layout the
//      workgroup tiers (bucket.hip.h) read.
// Bucket function, folds and outputs are those of the partition path, so both paths produce the
// same result row for row (tests/test_sorted_runs_gpu.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bucket_wave.hip.h"
#include "common.h"

namespace cdb {

// 16 bytes at an 8-byte aligned address (records rows): one 16-B load per piece
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2), aligned(8)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2), aligned(4)));


constexpr int kMaxRuns = 64;          // runs per family (cdb_dev_input.run_start rows)
constexpr uint32_t kGapInline = 32;  // longer directory gaps go to the gap list

struct RunMarkArgs {
  const uint64_t* kh;        // column 0 of the family
  const uint64_t* rs;        // device copy of run_start[f][0 .. nr]
  uint32_t nr;
  uint64_t nb;
  int shift;
  uint32_t* rdir;            // nr x (nb + 1)
  uint32_t* gaps;            // 4 u32 per entry: run, first bucket, last bucket, value
  uint32_t* gap_count;
  uint32_t gap_cap;
  uint32_t* err;             // bit 0: a run decreases; bit 1: gap list overflow
};

__device__ __forceinline__ void run_fill(const RunMarkArgs& a, uint32_t r, uint64_t c0, uint64_t c1, uint32_t v) {
  // buckets c0 .. c1 (inclusive) of run r start at run row v
  if (c0 > c1) return;
  if (c1 - c0 < kGapInline) {
    uint32_t* row = a.rdir + (uint64_t)r * (a.nb + 1);
    for (uint64_t c = c0; c <= c1; ++c) row[c] = v;
    return;
  }
  const uint32_t k = atomicAdd(a.gap_count, 1u);
  if (k >= a.gap_cap) {
    atomicOr(a.err, 2u);
    return;
  }
  uint4* g = reinterpret_cast<uint4*>(a.gaps) + k;
  *g = make_uint4(r, (uint32_t)c0, (uint32_t)c1, v);
}

// One thread per row: the first row of each (run, bucket) writes the directory entries of every
// bucket from its predecessor's bucket + 1 up to its own (empty buckets start where the next
// non-empty one does); the last row of a run closes the run's remaining buckets.
__global__ void __launch_bounds__(256) run_mark_kernel(RunMarkArgs a, uint64_t n) {
  __shared__ uint64_t rs[kMaxRuns + 1];
  for (uint32_t i = threadIdx.x; i <= a.nr; i += blockDim.x) rs[i] = a.rs[i];
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t lo = 0, hi = a.nr;  // run r: rs[r] <= i < rs[r + 1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (rs[mid] <= i) lo = mid;
      else hi = mid;
    }
    const uint32_t r = lo;
    const uint64_t rel = i - rs[r], len = rs[r + 1] - rs[r];
    const uint64_t h = a.kh[i] << a.shift;
    const uint64_t b = __umul64hi(h, a.nb);
    uint64_t c0 = 0;
    if (rel) {
      const uint64_t hp = a.kh[i - 1] << a.shift;
      if (hp > h) atomicOr(a.err, 1u);
      c0 = __umul64hi(hp, a.nb) + 1;
    }
    run_fill(a, r, c0, b, (uint32_t)i);
    if (rel + 1 == len) run_fill(a, r, b + 1, a.nb, (uint32_t)rs[r + 1]);
  }
}

// The same, four consecutive rows per thread read as two 16-B loads (the hash column must be
// 16-B aligned): fewer load instructions and one run lookup per four rows.
__global__ void __launch_bounds__(256) run_mark4_kernel(RunMarkArgs a, uint64_t n) {
  __shared__ uint64_t rs[kMaxRuns + 1];
  for (uint32_t i = threadIdx.x; i <= a.nr; i += blockDim.x) rs[i] = a.rs[i];
  __syncthreads();
  const uint64_t groups = (n + 3) / 4;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i0 = 4 * g;
    uint64_t h[4];
    if (i0 + 3 < n) {
      const ulonglong2 q0 = reinterpret_cast<const ulonglong2*>(a.kh)[2 * g];
      const ulonglong2 q1 = reinterpret_cast<const ulonglong2*>(a.kh)[2 * g + 1];
      h[0] = q0.x;
      h[1] = q0.y;
      h[2] = q1.x;
      h[3] = q1.y;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) h[k] = i0 + k < n ? a.kh[i0 + k] : 0;
    }
    uint64_t prev = i0 ? a.kh[i0 - 1] : 0;
    uint32_t lo = 0, hi = a.nr;  // run of row i0: rs[r] <= i0 < rs[r + 1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (rs[mid] <= i0) lo = mid;
      else hi = mid;
    }
    uint32_t r = lo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t i = i0 + k;
      if (i >= n) break;
      while (i >= rs[r + 1]) ++r;  // (empty runs in between are skipped too)
      const uint64_t rel = i - rs[r], len = rs[r + 1] - rs[r];
      const uint64_t hk = h[k] << a.shift;
      const uint64_t b = __umul64hi(hk, a.nb);
      uint64_t c0 = 0;
      if (rel) {
        const uint64_t hp = prev << a.shift;
        if (hp > hk) atomicOr(a.err, 1u);
        c0 = __umul64hi(hp, a.nb) + 1;
      }
      run_fill(a, r, c0, b, (uint32_t)i);
      if (rel + 1 == len) run_fill(a, r, b + 1, a.nb, (uint32_t)rs[r + 1]);
      prev = h[k];
    }
  }
}

// The long gaps, one workgroup per entry.
__global__ void __launch_bounds__(256) run_gap_kernel(const uint32_t* __restrict__ gaps, const uint32_t* gap_count,
                                                      uint32_t gap_cap, uint32_t* __restrict__ rdir, uint64_t nb) {
  const uint32_t n = min(*gap_count, gap_cap);
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint4 g = reinterpret_cast<const uint4*>(gaps)[k];
    uint32_t* row = rdir + (uint64_t)g.x * (nb + 1);
    for (uint64_t c = (uint64_t)g.y + threadIdx.x; c <= g.z; c += blockDim.x) row[c] = g.w;
  }
}

// Bucket directory of the family from its run directory: count[b] and the exclusive prefix
// base[b] = sum over runs of the run-relative first row of b (the directory holds absolute rows:
// rs_sum = the sum of the runs' first rows).
__global__ void __launch_bounds__(256) run_reduce_kernel(const uint32_t* __restrict__ rdir, uint32_t nr, uint64_t nb,
                                                         uint64_t rs_sum, uint32_t* __restrict__ base,
                                                         uint32_t* __restrict__ cnt) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t s0 = 0, s1 = 0;
    for (uint32_t r = 0; r < nr; ++r) {
      s0 += rdir[(uint64_t)r * (nb + 1) + b];
      s1 += rdir[(uint64_t)r * (nb + 1) + b + 1];
    }
    base[b] = (uint32_t)(s0 - rs_sum);
    cnt[b] = (uint32_t)(s1 - s0);
  }
}

// At most 8 runs per family: the three families' bucket directories in one pass, plus the
// bucket-major copy of the run directories that the persistent wave tier reads -- row b of bdir is
// 32 u32 (one 128-B line): key run r at slot r, node run r at 16 + r, member run r at 24 + r, the
// other slots 0. A wave streaming through consecutive buckets then reads one line per bucket
// instead of 3 nr lines of the run-major directories, lines that L2 no longer holds by the time
// the same wave reaches the neighbouring bucket (PMC: 68 GB fetched per C4 launch, not 28).
constexpr int kBdirRow = 32;
struct Reduce3Args {
  const uint32_t* rdir;  // the three families' run-major directories, one allocation
  uint32_t nr;
  uint64_t nb;
  uint32_t rs_sum[3];
  uint32_t* base[3];
  uint32_t* cnt[3];
  uint32_t* bdir;        // (nb + 1) x kBdirRow
};
__global__ void __launch_bounds__(256) run_reduce3_kernel(Reduce3Args a) {
  // the block's 256 bdir rows are staged in LDS (33-word pitch: no bank conflicts on the row writes)
  // and stored as contiguous 16-B pieces: one lane per row wrote 8 pieces 128 B apart before
  __shared__ uint32_t tile[256 * (kBdirRow + 1)];
  const uint64_t row = a.nb + 1, per_fam = (uint64_t)a.nr * row;
  for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 <= a.nb; b0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = b0 + threadIdx.x;
    uint32_t v[kBdirRow];
#pragma unroll
    for (int j = 0; j < kBdirRow; ++j) v[j] = 0;
    if (b <= a.nb) {
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        uint32_t s0 = 0, s1 = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if ((uint32_t)r < a.nr) {
            const uint32_t* d = a.rdir + f * per_fam + (uint64_t)r * row + b;
            const uint32_t x = d[0];
            v[f == 0 ? r : 8 + 8 * f + r] = x;
            s0 += x;
            if (b < a.nb) s1 += d[1];
          }
        }
        if (b < a.nb) {
          a.base[f][b] = s0 - a.rs_sum[f];
          a.cnt[f][b] = s1 - s0;
        }
      }
    }
    __syncthreads();  // (the previous round's readers are done with the tile)
#pragma unroll
    for (int j = 0; j < kBdirRow; ++j) tile[threadIdx.x * (kBdirRow + 1) + j] = v[j];
    __syncthreads();
    const uint64_t nrow = min((uint64_t)blockDim.x, a.nb + 1 - b0);  // rows of this round
    uint4* o = reinterpret_cast<uint4*>(a.bdir + b0 * kBdirRow);
    for (uint32_t q = threadIdx.x; q < nrow * (kBdirRow / 4); q += blockDim.x) {
      const uint32_t r = q / (kBdirRow / 4), c = 4 * (q % (kBdirRow / 4));
      const uint32_t* t = tile + r * (kBdirRow + 1) + c;
      o[q] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  }
}

// The persistent wave tier's units (bucket_wave_pipe_kernel): bit b of `units` is set where a unit
// starts. Consecutive buckets are packed greedily while together they hold at most 64 key rows,
// ccap child rows and gmax buckets (gmax: their hash span still fits the wave's sort word); a unit
// also starts at every multiple of 32 (so a chunk's last unit ends within the next 32 bits) and at
// every range start of a pipelined bucket phase, and a bucket beyond one wave (the wide tier's) or
// any bucket when gmax = 1 is a unit of its own. Bits past the last bucket are set. One wave per 64
// buckets: lane i finds how far a unit starting at its bucket would extend (window prefix sums of the
// row counts, compared up to kGroupMax buckets ahead), then the unit starts are the chain 0 ->
// next(0) -> ... -- the greedy packing, with one scalar step per unit instead of per bucket (a scalar
// loop over the buckets was SALU-bound: 0.46 ms per C4 step).
struct UnitArgs {
  const uint32_t *kcnt, *ncnt, *mcnt;
  uint64_t nb;
  uint32_t P;          // bucket-phase ranges: range p starts at bucket nb * p / P
  uint32_t gmax, ccap;
  uint32_t* units;     // (nb + 31) / 32 + 3 words
};
__global__ void __launch_bounds__(256) pipe_units_kernel(UnitArgs a) {
  const uint64_t words = (a.nb + 31) / 32 + 3, waves = (words + 1) / 2;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < waves;
       w += ((uint64_t)gridDim.x * blockDim.x) >> 6) {  // (wave-uniform)
    const uint64_t b = 64 * w + lane;
    uint32_t K = 0, C = 0;
    bool rstart = false;
    if (b < a.nb) {
      K = a.kcnt[b];
      C = min(a.ncnt[b] + a.mcnt[b], 0x7FFFFFFFu);
      if (a.P > 1) {  // (wave-uniform; 64-bit divisions only for a pipelined bucket phase)
        const uint64_t p = (b * a.P + a.nb - 1) / a.nb;  // the first range starting at or after b
        rstart = a.nb * p / a.P == b;
      }
    }
    const bool single = b >= a.nb || a.gmax <= 1 || K > (uint32_t)WaveLds<1>::KC || C > a.ccap;
    const uint64_t sgl = __ballot(single);
    // a unit starts here whatever precedes: the window's first bucket, each multiple of 32, a range
    // start, a bucket beyond one wave or past the end, and the bucket after one of those
    const uint64_t forced = 1ull | (1ull << 32) | __ballot(rstart) | sgl | (sgl << 1);
    uint32_t ek = min(K, 0xFFFFu), ec = min(C, 0xFFFFu);  // inclusive window prefixes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t tk = (uint32_t)__shfl_up((int)ek, o, 64), tc = (uint32_t)__shfl_up((int)ec, o, 64);
      if ((int)lane >= o) {
        ek += tk;
        ec += tc;
      }
    }
    const uint32_t sk = ek - min(K, 0xFFFFu), sc = ec - min(C, 0xFFFFu);  // exclusive
    uint32_t run = 1;  // buckets of a unit starting here
    bool alive = !single;
#pragma unroll
    for (uint32_t d = 1; d < 16; ++d) {
      const uint32_t j = lane + d;
      const uint32_t ekj = (uint32_t)__shfl_down((int)ek, d, 64), ecj = (uint32_t)__shfl_down((int)ec, d, 64);
      alive = alive && j < 64 && d < a.gmax && !((forced >> (j & 63)) & 1) && ekj - sk <= (uint32_t)WaveLds<1>::KC &&
              ecj - sc <= a.ccap;
      run += alive ? 1u : 0u;
    }
    const uint32_t nxt = lane + run;
    uint64_t m = 0;
    for (uint32_t st = 0; st < 64; st = (uint32_t)__builtin_amdgcn_readlane((int)nxt, (int)st))  // (scalar)
      m |= 1ull << st;
    m |= forced;  // (every forced start is on the chain already; past-the-end bits included)
    if (lane < 2 && 2 * w + lane < words) a.units[2 * w + lane] = (uint32_t)(m >> (32 * lane));
  }
}

// A bucket's slices of the runs, one per lane: lane j < L holds slice j of the family group --
// keys: the nr key runs; children: the nr node runs, then the nr member runs (child slots are
// node rows first, then member rows). incl = inclusive prefix of the slice lengths over lanes;
// off = absolute row of the slice's first row minus its first slot (row of slot c = off + c).
// (The run directory holds absolute rows, so no per-run base is loaded.)
struct RunMap {
  uint32_t incl, L;
  uint64_t off;
};

__device__ __forceinline__ RunMap run_map(const RunView& V, uint32_t b, int lane, bool children) {
  RunMap q;
  q.L = children ? 2 * V.nr : V.nr;
  uint32_t s = 0, n = 0;
  if ((uint32_t)lane < q.L) {
    const int f = children ? 1 + (lane >= (int)V.nr) : 0;
    const uint32_t r = (uint32_t)lane - (f == 2 ? V.nr : 0);
    const uint32_t* row = V.rdir[f] + (uint64_t)r * V.nbp1;
    const u32x2 se = *reinterpret_cast<const u32x2*>(row + b);  // row[b], row[b + 1]: one load
    s = se.x;
    n = se.y - s;
  }
  uint32_t incl = n;
  if (q.L <= 16) {  // (wave-uniform) the slices sit in lanes 0..15: a row scan by DPP, no LDS trips
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xF, 0xF, false);  // row_shr:1
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xF, 0xF, false);  // row_shr:2
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xF, 0xF, false);  // row_shr:4
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x118, 0xF, 0xF, false);  // row_shr:8
  } else {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
  }
  q.incl = incl;  // (lanes >= L: unused; lane_slice reads lanes < L only)
  q.off = (uint64_t)s - (incl - n);
  return q;
}

// The slice holding slot c: the number of slices that end at or before c (incl is
// non-decreasing over the lanes), found by a binary search over the lanes' incl.
__device__ __forceinline__ uint32_t lane_slice(uint32_t incl, uint32_t L, uint32_t c) {
  uint32_t r = 0;
  uint32_t k = 1;
  while (2 * k <= L) k <<= 1;
  for (; k; k >>= 1) {
    const uint32_t v = (uint32_t)__shfl((int)incl, (int)min(r + k - 1, L - 1), 64);
    if (r + k <= L && v <= c) r += k;
  }
  return min(r, L - 1);
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t x, uint32_t r) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, (int)r, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), (int)r, 64);
  return ((uint64_t)hi << 32) | lo;
}
// Absolute row of slot c.
__device__ __forceinline__ uint64_t run_row(const RunMap& q, uint32_t c) {
  return shfl_u64(q.off, lane_slice(q.incl, q.L, c)) + c;
}

// Key row `row` of the runs into key slot e (either input layout: a lane reads its row's fields
// with one 8-B load each, or the record as 16-B pieces).
// (REC: the records layout is known at compile time -- the column pointers stay out of registers)
template <bool REC = false, int KE, int CE>
__device__ __forceinline__ void load_key_row(const RunView& V, uint64_t row, int e, WaveIn<KE, CE>& in) {
  in.kh[e] = V.kin[K_KH][row];
  // aux (a counter's load-time total) is read only by a counter key no other replica holds:
  // the fold fetches it then, by the row index kept in its place (wave_bucket, RunView)
  in.kaux[e] = row;
  if (REC || V.ks == kKeyCols - 1) {  // (uniform) records: kf ct | ut dt as two 16-B pieces, then meta
    const uint64_t* rec = V.kin[1] + row * (kKeyCols - 1);
    const u64x2 q0 = reinterpret_cast<const u64x2*>(rec)[0], q1 = reinterpret_cast<const u64x2*>(rec)[1];
    in.kf[e] = q0.x;
    in.kct[e] = q0.y;
    in.kut[e] = q1.x;
    in.kdt[e] = q1.y;
    in.kmeta[e] = rec[K_META - 1];
  } else {
    in.kf[e] = V.kin[K_KF][row];
    in.kct[e] = V.kin[K_CT][row];
    in.kut[e] = V.kin[K_UT][row];
    in.kdt[e] = V.kin[K_DT][row];
    in.kmeta[e] = V.kin[K_META][row];
  }
}
// Child row `row` (a node row when isn, else a member row) into child slot e.
template <bool REC = false, int KE, int CE>
__device__ __forceinline__ void load_child_row(const RunView& V, bool isn, uint64_t row, int e, WaveIn<KE, CE>& in) {
  const uint64_t* const* col = isn ? V.nin : V.min;
  const uint32_t s = isn ? V.ns : V.ms;
  in.cpkh[e] = col[C_PKH][row];
  if (REC || s == kNodeCols - 1) {  // records: the 40-B record as two 16-B pieces and a word (8-B aligned)
    const uint64_t* rec = col[1] + row * (kNodeCols - 1);
    const u64x2 q0 = reinterpret_cast<const u64x2*>(rec)[0], q1 = reinterpret_cast<const u64x2*>(rec + 2)[0];
    in.cpkf[e] = q0.x;
    in.cid1[e] = q0.y;
    in.cid2[e] = q1.x;
    in.ct[e] = q1.y;
    in.cm[e] = rec[4];
  } else {
    in.cpkf[e] = col[C_PKF][row];
    in.cid1[e] = col[C_ID1][row];
    in.cid2[e] = col[C_ID2][row];
    in.ct[e] = col[C_T][row];
    in.cm[e] = col[C_META][row];
  }
}
template <int KE, int CE>
__device__ __forceinline__ void zero_key_slot(int e, WaveIn<KE, CE>& in) {
  in.kh[e] = in.kf[e] = in.kct[e] = in.kut[e] = in.kdt[e] = in.kaux[e] = in.kmeta[e] = 0;
}
template <int KE, int CE>
__device__ __forceinline__ void zero_child_slot(int e, WaveIn<KE, CE>& in) {
  in.cpkh[e] = in.cpkf[e] = in.cid1[e] = in.cid2[e] = in.ct[e] = in.cm[e] = 0;
}

// The rows of bucket b (KE key rows and CE child rows per lane) from the runs.
template <int KE, int CE = 2 * KE>
__device__ __forceinline__ void load_runs(const WaveArgs& W, const WaveDir& d, const RunMap& qk, const RunMap& qc,
                                          int lane, WaveIn<KE, CE>& in) {
  const RunView& V = W.V;
  in.d = d;
  const uint32_t C = d.N + d.M;
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const uint32_t c = lane + 64 * e;
    zero_key_slot(e, in);
    const uint64_t row = run_row(qk, c);
    if (c < d.K) load_key_row(V, row, e, in);
  }
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const uint32_t c = lane + 64 * e;
    zero_child_slot(e, in);
    if (__ballot(c < C) == 0) continue;  // (uniform) no child in this slot group
    const uint64_t row = run_row(qc, c);
    if (c < C) load_child_row(V, c < d.N, row, e, in);
  }
}

// Workgroups are dispatched round-robin over the 8 XCDs; XCD x takes one contiguous range of
// buckets, so neighbouring buckets (which share the runs' cache lines) meet in one L2.
__device__ __forceinline__ uint32_t xcd_bucket(uint32_t blk, uint32_t G, int wv) {
  const uint32_t q = G / kXcds, r = G % kXcds, x = blk % kXcds, j = blk / kXcds;
  return (x * q + min(x, r) + j) * kWavesPerWG + wv;
}

__global__ void __launch_bounds__(kWavesPerWG * 64, 5) bucket_wave_runs_kernel(WaveArgs W) {
  __shared__ WaveLds<1> lds_all[kWavesPerWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // (wave-uniform: scalar loads of the bucket's directory entry)
  const uint32_t b = __builtin_amdgcn_readfirstlane(W.blo + xcd_bucket(blockIdx.x, gridDim.x, wv));
  if (b >= W.bhi) return;
  // the directory entry (scalar loads) and the bucket's run slices (vector loads) do not depend on
  // each other: both are in flight before either is used
  const WaveDir d = load_dir(W.A, b);
  const RunMap qk = run_map(W.V, b, lane, false), qc = run_map(W.V, b, lane, true);
  if (d.N + d.M <= 64) {  // (wave-uniform) one child slot per lane
    WaveIn<1, 1> in;
    load_runs<1, 1>(W, d, qk, qc, lane, in);
    wave_bucket<1>(W, lds_all[wv], b, lane, in, []() {});
  } else {
    WaveIn<1> in;
    load_runs<1>(W, d, qk, qc, lane, in);
    wave_bucket<1>(W, lds_all[wv], b, lane, in, []() {});
  }
}

// ---------------------------------------------------------------------------------------------
// The persistent, software-pipelined wave tier (runs of at most 8 per family, C4's shape).
//
// bucket_wave_runs_kernel spends most of a bucket waiting: the run-directory pairs, then (after a
// chain of lane shuffles) the rows, then the fold. Here each wave streams through consecutive
// buckets and keeps the next ones' memory in flight while it folds the current one:
//   * bucket b + 2's run-directory pairs are loaded while bucket b folds (rows b + 2 and b + 3 of
//     the bucket-major directory bdir, one 256-B load: lanes 0..7 the key runs, 16..23 the node
//     runs, 24..31 the member runs);
//   * bucket b + 1's run map comes from those pairs by one DPP row scan (keys in DPP row 0, the
//     children in row 1), which also yields its row counts and dense bases -- no directory load;
//   * bucket b + 1's rows are loaded into the input registers as soon as bucket b's inputs are
//     dead (wave_bucket's `next()`, after its children are staged in LDS).
// Work: the bucket range is cut into 8 XCD slabs; waves of XCD x claim chunks of kPipeChunk
// consecutive buckets of slab x from its counter (the next claim is issued when a chunk starts)
// and then help the other slabs. Results are those of bucket_wave_runs_kernel bucket for bucket.
// Units: a wave takes a chunk's buckets in groups -- consecutive buckets packed greedily while their
// rows fit one wave (at most 64 key rows, W.gccap child rows, W.gmax buckets; a bucket beyond one
// wave alone stays a unit of its own, which the wide tier takes). Fixed-width hash buckets vary
// a lot in size (C4: ~40 key rows on average, 5 % over 64), so a unit of one bucket leaves a third
// of the lanes idle; a group of small buckets fills them, and with finer buckets (make_plan's
// pipe target) no bucket is wide.
#ifndef CDB_PIPE_CHUNK
#define CDB_PIPE_CHUNK 32
#endif
constexpr uint32_t kPipeChunk = CDB_PIPE_CHUNK;
#ifndef CDB_PIPE_MINB  // workgroups per CU the register budget is sized for
#define CDB_PIPE_MINB 4
#endif
constexpr uint32_t kPipeDone = 0xFFFFFFFFu;

// The slices of buckets b0 .. b1 - 1 (a group): bucket b0's bdir row (lanes 0..31) and bucket b1's
// (lanes 32..63), two 128-B lines (one 256-B load when b1 = b0 + 1), then lane j < 32 holds slice
// j's (first row, end row).
__device__ __forceinline__ u32x2 pipe_pairs(const RunView& V, uint32_t b0, uint32_t b1, int lane, bool valid) {
  uint32_t v = 0;
  if (valid) v = V.bdir[(uint64_t)(lane < 32 ? b0 : b1 - 1) * kBdirRow + (uint32_t)lane];
  const uint32_t e = (uint32_t)__shfl((int)v, (lane + 32) & 63, 64);
  u32x2 se = {v, e};
  if (lane >= 32) se = {0u, 0u};
  return se;
}

struct PipeMap {
  uint32_t incl, off;  // inclusive prefix of the slice lengths in the lane's DPP row; row of slot c = off + c
};
__device__ __forceinline__ uint32_t dpp_row_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  return x;
}
__device__ __forceinline__ PipeMap pipe_map(const RunView& V, u32x2 se, WaveDir& d) {
  const uint32_t n = se.y - se.x;
  PipeMap q;
  q.incl = dpp_row_scan(n);
  q.off = se.x - (q.incl - n);
  const uint32_t ss = dpp_row_scan(se.x);
  // (bdir slots: key runs 0..7, node runs 16..23, member runs 24..31; unused slots are empty)
  d.K = (uint32_t)__builtin_amdgcn_readlane((int)q.incl, 7);
  const uint32_t cn = (uint32_t)__builtin_amdgcn_readlane((int)q.incl, 23);
  const uint32_t cc = (uint32_t)__builtin_amdgcn_readlane((int)q.incl, 31);
  d.N = cn;
  d.M = cc - cn;
  const uint32_t sk = (uint32_t)__builtin_amdgcn_readlane((int)ss, 7);
  const uint32_t sn = (uint32_t)__builtin_amdgcn_readlane((int)ss, 23);
  const uint32_t sc = (uint32_t)__builtin_amdgcn_readlane((int)ss, 31);
  d.kb = sk - V.rs_sum[0];
  d.nb0 = sn - V.rs_sum[1];
  d.mb0 = sc - sn - V.rs_sum[2];
  return q;
}
// Row of slot c among the L slices held by lanes base .. base + L - 1.
__device__ __forceinline__ uint32_t pipe_row(const PipeMap& q, int base, uint32_t L, uint32_t c) {
  uint32_t r = 0, k = 1;
  while (2 * k <= L) k <<= 1;
  for (; k; k >>= 1) {
    const uint32_t v = (uint32_t)__shfl((int)q.incl, base + (int)min(r + k - 1, L - 1), 64);
    if (r + k <= L && v <= c) r += k;
  }
  r = min(r, L - 1);
  return (uint32_t)__shfl((int)q.off, base + (int)r, 64) + c;
}
// (REC: the records layout, known at compile time; else the layout is read from V)
template <bool REC, int CE>
__device__ __forceinline__ void pipe_load_child(const RunView& V, const WaveDir& d, const PipeMap& q, int lane, int e,
                                                WaveIn<1, CE>& in) {
  const uint32_t c = lane + 64 * e;
  zero_child_slot(e, in);
  const uint32_t row = pipe_row(q, 16, 16, c);
  if (c < d.N + d.M) load_child_row<REC>(V, c < d.N, row, e, in);
}
template <bool REC>
__device__ __forceinline__ void pipe_load(const RunView& V, const WaveDir& d, const PipeMap& q, int lane,
                                          WaveIn<1, 1>& in) {
  in.d = d;
  zero_key_slot(0, in);
  const uint32_t krow = pipe_row(q, 0, 8, (uint32_t)lane);
  if ((uint32_t)lane < d.K) load_key_row<REC>(V, krow, 0, in);
  pipe_load_child<REC>(V, d, q, lane, 0, in);
}

// REC: every family in the records layout (the host checks the strides)
template <bool REC>
__global__ void __launch_bounds__(kWavesPerWG * 64, CDB_PIPE_MINB) bucket_wave_pipe_kernel(WaveArgs W) {
  __shared__ WaveLds<1> lds_all[kWavesPerWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WaveLds<1>& L = lds_all[wv];
  const RunView& V = W.V;
  const uint32_t x0 = blockIdx.x % kXcds;  // (workgroups are dispatched round-robin over the XCDs)
  const uint64_t span = W.bhi - W.blo;
  auto slab_lo = [&](uint32_t x) { return W.blo + (uint32_t)(span * x / kXcds); };
  auto claim = [&](uint32_t x) {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(W.pipe_next + x, 1u);
    return v;  // (lane 0's; read once the chunk is needed)
  };
  // the unit stream (wave-uniform): chunk [sc, se) of slab xs; gm = the unit starts in it not yet
  // taken (bit i: bucket sc + i), ge = the end of its last unit; the next chunk's claim in flight
  const __attribute__((address_space(4))) uint32_t* units =
      (const __attribute__((address_space(4))) uint32_t*)W.units;  // (scalar loads)
  // A unit travels as one word, first bucket << 4 | (buckets - 1) (the host keeps nb < 2^28 here).
  uint32_t xs = x0, sc = 0, ge = 0, pend = claim(x0), gm = 0;
  bool done = false;
  auto produce = [&]() -> uint32_t {
    while (gm == 0) {
      if (done) return kPipeDone;
      uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)pend, 0), se = 0;
      for (;;) {
        const uint32_t lo = slab_lo(xs), hi = slab_lo(xs + 1);
        const uint64_t st = (uint64_t)lo + (uint64_t)c * kPipeChunk;
        if (st < hi) {
          sc = (uint32_t)st;
          se = (uint32_t)min((uint64_t)hi, st + kPipeChunk);
          break;
        }
        xs = (xs + 1) % kXcds;  // slab drained: help the next one
        if (xs == x0) {
          done = true;
          return kPipeDone;
        }
        c = (uint32_t)__builtin_amdgcn_readlane((int)claim(xs), 0);
      }
      pend = claim(xs);
      // bits sc .. sc + 63 of the unit bitmap (a unit starts at every multiple of 32: the chunk's
      // last unit ends within them)
      const uint32_t w = sc >> 5, s = sc & 31;
      const uint64_t lo64 = (uint64_t)units[w] | ((uint64_t)units[w + 1] << 32);
      const uint64_t win = s ? (lo64 >> s) | ((uint64_t)units[w + 2] << (64 - s)) : lo64;
      const uint32_t n = se - sc;  // (<= kPipeChunk <= 32)
      gm = (uint32_t)(win & ((1ull << n) - 1));
      const uint64_t rest = win >> n;
      ge = min(W.bhi, sc + (rest ? n + (uint32_t)__builtin_ctzll(rest) : 64u));
    }
    const uint32_t g0 = sc + (uint32_t)__builtin_ctz(gm);
    gm &= gm - 1;
    const uint32_t g1 = gm ? sc + (uint32_t)__builtin_ctz(gm) : ge;
    return (g0 << 4) | (g1 - g0 - 1);
  };
  auto ufirst = [](uint32_t u) { return u >> 4; };
  auto uend = [](uint32_t u) { return (u >> 4) + (u & 15) + 1; };

  uint32_t b = produce();
  if (b == kPipeDone) return;
  WaveIn<1, 1> in;
  PipeMap qc;
  {
    WaveDir d;
    qc = pipe_map(V, pipe_pairs(V, ufirst(b), uend(b), lane, true), d);
    d.G = (b & 15) + 1;
    pipe_load<REC>(V, d, qc, lane, in);
  }
  uint32_t b1 = produce();
  u32x2 pr = pipe_pairs(V, ufirst(b1), uend(b1), lane, b1 != kPipeDone);  // (no unit: zero pairs, an empty map)
  uint32_t folded = 0, nunits = 0;  // (wave-uniform) buckets / units this wave folded: stats.wave_pipe_*
  while (b != kPipeDone) {
    const uint32_t b2 = b1 != kPipeDone ? produce() : kPipeDone;
    // the iteration's arguments, read from the kernel-argument segment behind a barrier (as the
    // second half's below): nothing of them is held in spilled SGPRs from one unit to the next
    const __attribute__((address_space(4))) WaveArgs* Wa =
        (const __attribute__((address_space(4))) WaveArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(Wa));
    const WaveArgs Wi = *(const WaveArgs*)Wa;
    const RunView& Vi = Wi.V;
    const WaveDir d = in.d;
    const uint32_t C = d.N + d.M;
    // 65..128 children: a second child slot per lane, loaded now (9 % of C4's buckets)
    const bool two = C > 64 && C <= WaveLds<1>::CC && d.K <= WaveLds<1>::KC;
    WaveMid<1> mid;
    int act;
    if (!two) {
      act = wave_phase_a<1, 1>(Wi, L, ufirst(b), lane, in, mid);
    } else {
      WaveIn<1, 2> in2;
      in2.d = d;
      in2.kh[0] = in.kh[0];
      in2.kf[0] = in.kf[0];
      in2.kct[0] = in.kct[0];
      in2.kut[0] = in.kut[0];
      in2.kdt[0] = in.kdt[0];
      in2.kaux[0] = in.kaux[0];
      in2.kmeta[0] = in.kmeta[0];
      in2.cpkh[0] = in.cpkh[0];
      in2.cpkf[0] = in.cpkf[0];
      in2.cid1[0] = in.cid1[0];
      in2.cid2[0] = in.cid2[0];
      in2.ct[0] = in.ct[0];
      in2.cm[0] = in.cm[0];
      pipe_load_child<REC>(Vi, d, qc, lane, 1, in2);
      act = wave_phase_a<1, 2>(Wi, L, ufirst(b), lane, in2, mid);
    }
    // bucket b's input registers are dead: bucket b + 1's rows into them and b + 2's pairs, in
    // flight while b's children fold and its outputs are written. (One program point for every
    // path, and unconditional -- past the last bucket the pairs are zero and the map empty -- so
    // the loads land in the registers the next iteration reads: no copy that waits for them.)
    {
      WaveDir dn;
      qc = pipe_map(Vi, pr, dn);
      dn.G = (b1 & 15) + 1;
      pipe_load<REC>(Vi, dn, qc, lane, in);
      pr = pipe_pairs(Vi, ufirst(b2), uend(b2), lane, b2 != kPipeDone);
    }
    if (act != WAVE_DONE) {
      // The outputs' pointers are read from the kernel-argument segment here, behind a barrier the
      // compiler cannot move loads across, so that they are not held in (spilled) SGPRs through the
      // whole loop: the kernel needs more than the 102 SGPRs a wave has, and every reload of a
      // spilled one is a VALU v_readlane.
      const __attribute__((address_space(4))) WaveArgs* Wk =
          (const __attribute__((address_space(4))) WaveArgs*)__builtin_amdgcn_kernarg_segment_ptr();
      asm volatile("" : "+s"(Wk));
      WaveArgs Wb = W;
      Wb.A.kos = Wk->A.kos;
      Wb.A.nos = Wk->A.nos;
      Wb.A.mos = Wk->A.mos;
      Wb.A.kout = Wk->A.kout;
      Wb.A.nout = Wk->A.nout;
      Wb.A.mout = Wk->A.mout;
      Wb.A.stats = Wk->A.stats;
      Wb.big_list = Wk->big_list;
      Wb.big_count = Wk->big_count;
      if (act == WAVE_PUSH) {
        wave_push(Wb, ufirst(b), lane, d.G);
      } else {
        if (!two)
          wave_phase_b<1, 1>(Wb, L, ufirst(b), lane, mid);
        else
          wave_phase_b<1, 2>(Wb, L, ufirst(b), lane, mid);
        folded += d.G;
        ++nunits;
      }
    }
    wave_sync();  // (the next bucket reuses this one's LDS)
    b = b1;
    b1 = b2;
  }
  if (lane == 0 && folded) {
    atomicAdd(&stat_shard(W.A.stats)[ST_PIPE], (unsigned long long)folded);
    atomicAdd(&stat_shard(W.A.stats)[ST_PIPE_UNITS], (unsigned long long)nunits);
  }
}

// The wide tier (65..128 key rows or 129..256 child rows) on the runs: as bucket_wide_kernel.
__global__ void __launch_bounds__(kWavesPerWG * 64) bucket_wide_runs_kernel(WaveArgs W) {
  __shared__ WaveLds<2> lds_all[kWavesPerWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t groups = (W.bhi - W.blo + 63) / 64;
  unsigned long long found = 0;
  uint32_t nx = 0, en = 0;
  for (uint32_t g = wide_group(W, lane, nx, en); g < groups; g = wide_group(W, lane, nx, en)) {
    const uint32_t b = W.blo + g * 64 + lane;
    uint64_t m = __ballot(b < W.bhi && wide_bucket_candidate(W.A, b));
    found += __popcll(m);
    while (m) {
      const int i = __builtin_ctzll(m);
      m &= m - 1;
      const uint32_t bb = W.blo + g * 64 + i;
      WaveIn<2> in;
      if (W.V.bdir) {  // (wave-uniform) the bucket-major directory: one load, no directory entry
        WaveDir d;
        const PipeMap q = pipe_map(W.V, pipe_pairs(W.V, bb, bb + 1, lane, true), d);
        in.d = d;
        const uint32_t C = d.N + d.M;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint32_t c = lane + 64 * e;
          zero_key_slot(e, in);
          const uint32_t row = pipe_row(q, 0, 8, c);
          if (c < d.K) load_key_row(W.V, row, e, in);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t c = lane + 64 * e;
          zero_child_slot(e, in);
          if (__ballot(c < C) == 0) continue;  // (uniform) no child in this slot group
          const uint32_t row = pipe_row(q, 16, 16, c);
          if (c < C) load_child_row(W.V, c < d.N, row, e, in);
        }
      } else {
        const WaveDir d = load_dir(W.A, bb);
        const RunMap qk = run_map(W.V, bb, lane, false), qc = run_map(W.V, bb, lane, true);
        load_runs<2>(W, d, qk, qc, lane, in);
      }
      wave_bucket<2>(W, lds_all[wv], bb, lane, in, []() {});
      wave_sync();  // (the next bucket reuses this one's LDS)
    }
  }
  if (lane == 0 && found) atomicAdd(&stat_shard(W.A.stats)[ST_WIDE], found);
}

// Buckets handed to the workgroup tiers: their rows are copied out of the runs into AoS rows
// (8-word key rows, 6-word child rows) and the row indices of the bucket are written to the
// permutation, so that bucket.hip.h reads them as it reads partitioned rows. Work is split in
// chunks of kMatChunk rows of one (bucket, family), so one over-capacity bucket (C5's hottest
// keys: millions of children) spreads over the chip instead of one workgroup:
//   mat_count_kernel : rows per (listed bucket, family) and chunks per listed bucket;
//   (exclusive scans: each family's AoS row base per bucket, each bucket's first chunk)
//   mat_copy_kernel  : one workgroup per chunk (grid-stride over the device-side chunk total).
constexpr uint32_t kMatChunk = 4096;

struct MatArgs {
  uint64_t *kr, *nr, *mr;        // AoS scratch rows
  uint32_t *kp, *np, *mp;        // permutations (indexed by the bucket's base + slot)
  uint32_t* cnt;                 // [3][nb]: rows per listed bucket and family
  uint32_t* base;                // [3][nb]: exclusive scan of cnt per family (AoS row base)
  uint32_t* chunks;              // [nb]: chunks per listed bucket
  uint32_t* chunk0;              // [nb]: exclusive scan of chunks
  const uint64_t* n_chunks;      // total chunks (device)
  uint32_t nb;
  uint32_t runs_child_max;       // > 0: buckets of at most this many children (and at most kCapK
                                 // keys) get only their keys copied: the chip-wide path reads
                                 // their children from the runs (hot.hip.h, HotArgs::runs)
};

__global__ void __launch_bounds__(256) mat_count_kernel(WaveArgs W, MatArgs M, const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ count) {
  const RunView& V = W.V;
  const uint32_t total = *count;
  for (uint32_t li = blockIdx.x * blockDim.x + threadIdx.x; li < M.nb; li += gridDim.x * blockDim.x) {
    uint32_t ch = 0, n3[3] = {0, 0, 0};
    for (int f = 0; f < 3; ++f) {
      if (li < total) {
        const uint32_t b = list[li];
        for (uint32_t r = 0; r < V.nr; ++r) {
          const uint32_t* row = V.rdir[f] + (uint64_t)r * V.nbp1;
          n3[f] += row[b + 1] - row[b];
        }
      }
    }
    if (M.runs_child_max && n3[0] <= (uint32_t)kCapK && n3[1] + n3[2] <= M.runs_child_max) n3[1] = n3[2] = 0;
    for (int f = 0; f < 3; ++f) {
      M.cnt[(uint64_t)f * M.nb + li] = n3[f];
      ch += (n3[f] + kMatChunk - 1) / kMatChunk;
    }
    M.chunks[li] = ch;
  }
}

__global__ void __launch_bounds__(256) mat_copy_kernel(WaveArgs W, MatArgs M, const uint32_t* __restrict__ list) {
  const RunView& V = W.V;
  const BucketArgs& A = W.A;
  __shared__ uint32_t rs[kMaxRuns + 1], pre[kMaxRuns + 1];
  __shared__ uint64_t rb[kMaxRuns + 1];
  const uint64_t total = *M.n_chunks;
  for (uint64_t ci = blockIdx.x; ci < total; ci += gridDim.x) {
    // the listed bucket holding chunk ci: last li with chunk0[li] <= ci
    uint32_t lo = 0, hi = M.nb;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (M.chunk0[mid] <= ci) lo = mid;
      else hi = mid;
    }
    const uint32_t li = lo, b = list[li];
    uint32_t local = (uint32_t)(ci - M.chunk0[li]);
    int f = 0;
    uint32_t n = M.cnt[li];
    while (f < 2 && local >= (n + kMatChunk - 1) / kMatChunk) {
      local -= (n + kMatChunk - 1) / kMatChunk;
      ++f;
      n = M.cnt[(uint64_t)f * M.nb + li];
    }
    __syncthreads();
    if (threadIdx.x < V.nr) {
      const uint32_t r = threadIdx.x;
      const uint32_t* row = V.rdir[f] + (uint64_t)r * V.nbp1;
      rs[r] = row[b];
      pre[r + 1] = row[b + 1] - row[b];
      rb[r] = 0;  // (the directory holds absolute rows)
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      pre[0] = 0;
      for (uint32_t r = 0; r < V.nr; ++r) pre[r + 1] += pre[r];
    }
    __syncthreads();
    const uint32_t c0 = local * kMatChunk, c1 = min(n, c0 + kMatChunk);
    const uint32_t abase = M.base[(uint64_t)f * M.nb + li];
    const uint32_t pb = f == 0 ? A.kbase[b] : f == 1 ? A.nbase[b] : A.mbase[b];
    for (uint32_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
      uint32_t r = 0, rhi = V.nr;  // last run with pre[r] <= c
      while (rhi - r > 1) {
        const uint32_t mid = (r + rhi) >> 1;
        if (pre[mid] <= c) r = mid;
        else rhi = mid;
      }
      const uint64_t src = rb[r] + rs[r] + (c - pre[r]);
      const uint64_t dst = (uint64_t)abase + c;
      if (f == 0) {
        uint64_t* o = M.kr + dst * kKeyStride;
#pragma unroll
        for (int k = 0; k < kKeyCols; ++k) o[k] = row_field(V.kin, V.ks, k, src);
        o[kKeyCols] = 0;
        M.kp[pb + c] = (uint32_t)dst;
      } else {
        const uint64_t* const* in = f == 1 ? V.nin : V.min;
        const uint32_t s = f == 1 ? V.ns : V.ms;
        uint64_t* o = (f == 1 ? M.nr : M.mr) + dst * kChildStride;
#pragma unroll
        for (int k = 0; k < kChildStride; ++k) o[k] = row_field(in, s, k, src);
        (f == 1 ? M.np : M.mp)[pb + c] = (uint32_t)dst;
      }
    }
  }
}

}  // namespace cdb
