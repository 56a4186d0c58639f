// HIP driver of the merge pipeline (gfx950): partition -> fused bucket merge ->
// over-capacity buckets -> dense compaction. Also the device-level C-ABI entry points.
#include <hip/hip_runtime.h>
#include <mutex>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <map>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bucket.hip.h"
#include "bucket_wave.hip.h"
#include "engine.h"
#include "partition.hip.h"
#include "hot.hip.h"
#include "radix.hip.h"
#include "runs.hip.h"

namespace cdb {

cdb_status fail(cdb_ctx* ctx, cdb_status st, const std::string& msg) {
  // (the decoder's index threads may fail side by side: the message string is written under a lock)
  static std::mutex mu;
  if (ctx) {
    std::lock_guard<std::mutex> g(mu);
    ctx->last_error = msg;
  }
  return st;
}

// The last failed context creation's message (cdb_last_error(NULL)): no context exists to hold it.
std::mutex g_create_mu;
std::string g_create_error;
cdb_status set_create_error(cdb_status st, const std::string& msg) {
  std::lock_guard<std::mutex> g(g_create_mu);
  g_create_error = msg;
  return st;
}

cdb_status hip_check(cdb_ctx* ctx, hipError_t e, const char* what) {
  if (e == hipSuccess) return CDB_OK;
  return fail(ctx, e == hipErrorOutOfMemory ? CDB_OUT_OF_MEMORY : CDB_DEVICE_ERROR,
              std::string(what) + ": " + hipGetErrorString(e));
}

// Launch check. With CDB_SYNC_CHECK set, also synchronises so that a device fault is
// reported at the kernel that caused it (debugging aid; off in normal runs).
cdb_status launch_check(cdb_ctx* ctx, hipStream_t s, const char* what) {
  static const bool sync = std::getenv("CDB_SYNC_CHECK") != nullptr;
  cdb_status st = hip_check(ctx, hipGetLastError(), what);
  if (st == CDB_OK && sync) st = hip_check(ctx, hipStreamSynchronize(s), what);
  return st;
}

// The persistent wave tier (bucket_wave_pipe_kernel) on runs of at most 8 per family. It pays off
// from kPipeMinBuckets buckets on: below it, its resident grid is mostly claiming and the wide tier's
// buckets wait behind it (C1's 100K buckets: 0.33 -> 0.70 ms of bucket phase with it; C3's few
// thousand large buckets likewise). Test and A/B hook, read per merge: CDB_WAVE_PIPE=0 runs the
// one-bucket-per-wave kernel instead, CDB_WAVE_PIPE=force runs the persistent kernel at any bucket
// count (the parity tests pin it against the oracle at sizes the oracle folds in seconds).
constexpr uint64_t kPipeMinBuckets = 1ull << 19;
bool pipe_wave_wanted(uint64_t nb) {
  const char* e = std::getenv("CDB_WAVE_PIPE");
  if (e && e[0] == '0') return false;
  if (e && std::strcmp(e, "force") == 0) return true;
  return nb >= kPipeMinBuckets;
}
// Its units group consecutive buckets (runs.hip.h, at most kGroupMax); the plan then targets ~kPipeFineTarget key rows
// per bucket instead of ~40. Test and A/B hooks: CDB_GROUPS=0 (one bucket per unit, round-5 buckets),
// CDB_PIPE_TARGET (key rows per bucket), CDB_GROUP_CCAP (child rows per unit, 64 or 128).
constexpr uint64_t kPipeFineTarget = 28;  // (C4 step, one box: 24 / 28 -> 16.57-16.63 / 16.32 ms; before the
                                          // parallel unit kernel 20 / 22 / 24 / 26 / 28 -> 17.96 / 17.19 / 16.98 / 17.08 / 17.90)
constexpr uint64_t kGroupMax = 16;
bool groups_wanted() {
  const char* e = std::getenv("CDB_GROUPS");
  return !(e && e[0] == '0');
}
uint64_t pipe_fine_target() {
  const char* e = std::getenv("CDB_PIPE_TARGET");
  return e ? (uint64_t)std::max(8, std::min(64, std::atoi(e))) : kPipeFineTarget;
}
uint32_t group_ccap() {
  const char* e = std::getenv("CDB_GROUP_CCAP");
  const int v = e ? std::atoi(e) : 128;
  return v >= 128 ? 128u : 64u;
}
// Its grid: every workgroup slot of the device (resident workgroups per CU x CUs).
uint32_t pipe_wave_grid(cdb_ctx* ctx) {
  static uint32_t grid[64] = {0};
  const int dev = ctx->device;
  if (dev >= 0 && dev < 64 && grid[dev]) return grid[dev];
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bucket_wave_pipe_kernel<true>, kWavesPerWG * 64, 0) !=
          hipSuccess ||
      per_cu <= 0)
    per_cu = 4;
  (void)hipGetLastError();
  const uint32_t g = (uint32_t)(cus * per_cu);
  if (dev >= 0 && dev < 64) grid[dev] = g;
  return g;
}

void* ws_get(cdb_ctx* ctx, int slot, size_t bytes, cdb_status* st) {
  cdb_ctx::Buf& b = ctx->ws[slot];
  if (b.bytes >= bytes && b.p) return b.p;
  if (b.p) {
    hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 20);
  want = (want + 4095) & ~size_t(4095);
  hipError_t e = hipMalloc(&b.p, want);
  if (e != hipSuccess) {
    *st = hip_check(ctx, e, "hipMalloc(workspace)");
    b.p = nullptr;
    return nullptr;
  }
  b.bytes = want;
  return b.p;
}

namespace {

#define CDB_TRY(...)                  \
  do {                                \
    cdb_status _s = (__VA_ARGS__);    \
    if (_s != CDB_OK) return _s;      \
  } while (0)
#define CDB_HIP(x, what) CDB_TRY(hip_check(ctx, (x), what))

// Empty one-thread launches that bracket a merge in kernel traces: scripts/pmc_traffic.py counts
// the HBM traffic of the dispatches between them (and so not a bench's setup kernels).
__global__ void merge_begin_marker() {}
__global__ void merge_end_marker() {}

__global__ void set_dir_kernel(uint32_t* base, uint32_t* cnt, uint32_t n) {
  base[0] = 0;
  cnt[0] = n;
}

// pos stamp of the host boundary: batch i's rows carry fold position i (meta bits 48..55)
__global__ void stamp_pos_kernel(uint64_t* __restrict__ meta, uint64_t n, uint32_t pos) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t m = meta[i];
    meta[i] = meta_pack(meta_tag(m), pos, meta_src(m));
  }
}

// A result row as an input row of fold position 0 (cdb_dev_state_rows, cdb_merge_into): the
// reference merges peer snapshots into the live server.db (replica/pull.rs:120-128, db.rs:31-43),
// whose rows are what the previous merge produced. A counter's load-time total (aux) is its sum
// (type_counter.rs:89-91, the result's win); src is the row in the result, which resolves bytes.
__global__ void state_rows_kernel(uint64_t* __restrict__ meta, uint64_t* __restrict__ aux, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t T = meta_tag(meta[i]);
    if (aux) aux[i] = T == TAG_COUNTER ? aux[i] : 0;
    meta[i] = meta_pack(T, 0, i);
  }
}

// Any bucket beyond the wide tier's capacity (or a forced workgroup tier)?
__global__ void beyond_wide_kernel(BucketArgs A, uint32_t nb, uint32_t* flag) {
  bool any = false;
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gridDim.x * blockDim.x)
    any |= A.kcnt[b] > (uint32_t)WaveLds<2>::KC || A.ncnt[b] + A.mcnt[b] > (uint32_t)WaveLds<2>::CC;
  if (__ballot(any) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

__global__ void add_stat_kernel(unsigned long long* stats, int which, unsigned long long v) {
  atomicAdd(&stats[which], v);
}

__global__ void iota_kernel(uint32_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i;
}

__global__ void gc_lastbad_kernel(const uint64_t* __restrict__ ct, const uint64_t* __restrict__ meta, uint32_t stride,
                                  uint64_t n, uint64_t wm, unsigned long long* out) {
  uint64_t best = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t m = meta[i * stride];
    if (meta_tag(m) == TAG_DELETE && ct[i * stride] > wm) best = max(best, meta_order(m) + 1);
  }
  for (int o = 32; o > 0; o >>= 1) best = max(best, (uint64_t)__shfl_xor((unsigned long long)best, o, 64));
  if ((threadIdx.x & 63) == 0 && best) atomicMax(out, (unsigned long long)best);
}

struct CompactArgs {
  const uint64_t *ks, *ns, *ms;  // sparse AoS outputs (BucketArgs::kos / nos / mos)
  uint64_t* kd[kKeyOutCols];
  uint64_t* nd[kNodeCols];
  uint64_t* md[kMemberCols];
  const uint32_t *kbase, *nbase, *mbase, *kout, *nout, *mout, *kdoff, *ndoff, *mdoff;
  const unsigned long long* base_tot;  // dense row base per family (a pipelined range's; else zero)
  uint64_t cap[3];                     // rows of each family's sparse slots and dense output
  uint32_t* err;                       // set when an index falls outside them
  const uint32_t* skip_if;             // pipelined ranges: nothing to do once a bucket went to a
                                       // workgroup tier (everything is compacted again at the end)
  // state = 1 (cdb_dev_state_rows from the bucket layout): the destinations are the next merge's
  // input rows -- keys kh kf ct ut dt aux meta, children unchanged, meta = tag | pos 0 | src = the
  // dense index, aux = a counter's sum -- in columns or records (ds: record stride per family)
  int state;
  uint32_t ds[3];
};

// Writes dense row d of a result family as the next merge's input row (position 0): the reference
// merges peer snapshots into its live server.db (replica/pull.rs:120-128, db.rs:31-43), whose rows
// are what the previous merge produced. A counter's load-time total (aux) is its sum
// (type_counter.rs:89-91, the result's win); src is the dense row, which resolves bytes.
template <int FAM>
__device__ __forceinline__ void put_state_row(uint64_t* const* dst, uint32_t ds, uint64_t d, const uint64_t* v) {
  if constexpr (FAM == 0) {
    const uint32_t T = meta_tag(v[O_META]);
    const uint64_t f[kKeyCols] = {v[O_KH], v[O_KF], v[O_CT], v[O_UT], v[O_DT],
                                  T == TAG_COUNTER ? v[O_WIN] : 0, meta_pack(T, 0, d)};
#pragma unroll
    for (int c = 0; c < kKeyCols; ++c) dst[c][c ? d * ds : d] = f[c];
  } else {
#pragma unroll
    for (int c = 0; c < kChildStride; ++c)
      dst[c][c ? d * ds : d] = c == C_META ? meta_pack(meta_tag(v[C_META]), 0, d) : v[c];
  }
}

// The same from a dense (compacted) result: one thread per row.
template <int FAM>
__global__ void state_dense_kernel(const cdb_dev_rows src, cdb_dev_rows dst, uint32_t ds) {
  constexpr int NW = FAM == 0 ? kKeyOutCols : kChildStride;
  uint64_t* dc[8];
  for (int c = 0; c < 8; ++c) dc[c] = dst.col[c];
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < src.n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t v[NW];
#pragma unroll
    for (int c = 0; c < NW; ++c) v[c] = src.col[c][i];
    put_state_row<FAM>(dc, ds, i, v);
  }
}

// Sparse-by-bucket outputs -> dense arrays; child ranges become absolute row indices.
// A group of 64 consecutive buckets' dense output rows are one contiguous range (doff is an
// exclusive scan), so lane t of a pass copies dense row doff[b0] + t from its bucket's sparse
// slot -- coalesced stores, nearly coalesced loads. The source bucket of a dense row is a
// 6-step binary search over the group's offsets in LDS.
constexpr int kCompactWaves = 4;

struct CompactLds {
  uint32_t doff[64], sbase[64], ndoff[64], mdoff[64];
};

__device__ __forceinline__ int group_bucket(const uint32_t* rel, uint32_t t) {  // last j: rel[j] <= t
  int j = 0;
#pragma unroll
  for (int step = 32; step > 0; step >>= 1) j = (rel[j + step] <= t) ? j + step : j;
  return j;
}

// One wave per (group of 64 buckets, family): three independent tasks per group, so more
// waves are in flight; each lane copies two dense rows per pass (their loads overlap). The
// family is a template parameter, so every column pointer is a kernel-argument register
// (selecting pointers by a run-time family put the argument arrays in scratch).
template <int FAM>
__device__ __forceinline__ void compact_row(const CompactArgs& A, const CompactLds& L, uint32_t t, uint32_t d0) {
  const int j = group_bucket(L.doff, t);
  const uint32_t src = L.sbase[j] + (t - L.doff[j]);
  const uint64_t dst = A.base_tot[FAM] + d0 + t;
  if (src >= A.cap[FAM] || dst >= A.cap[FAM]) {  // a broken directory: report, never touch memory
    atomicOr(A.err, 1u);
    return;
  }
  if (A.state) {
    constexpr int NW = FAM == 0 ? kKeyOutCols : kChildStride;
    uint64_t v[NW];
    const ulonglong2* row = (const ulonglong2*)((FAM == 0 ? A.ks : FAM == 1 ? A.ns : A.ms) + (uint64_t)src * NW);
#pragma unroll
    for (int c = 0; c < NW / 2; ++c) {
      const ulonglong2 q = row[c];
      v[2 * c] = q.x;
      v[2 * c + 1] = q.y;
    }
    put_state_row<FAM>(FAM == 0 ? A.kd : FAM == 1 ? A.nd : A.md, A.ds[FAM], dst, v);
    return;
  }
  if constexpr (FAM == 0) {
    uint64_t v[kKeyOutCols];
    const ulonglong2* row = (const ulonglong2*)(A.ks + (uint64_t)src * kKeyOutCols);
#pragma unroll
    for (int c = 0; c < kKeyOutCols / 2; ++c) {
      const ulonglong2 q = row[c];
      v[2 * c] = q.x;
      v[2 * c + 1] = q.y;
    }
    const uint64_t cnt = v[O_CREF] & 0xFFFFFF;
    const uint32_t T = meta_tag(v[O_META]);
    const uint64_t begin =
        cnt ? (v[O_CREF] >> 24) + (T == TAG_COUNTER ? A.base_tot[1] + L.ndoff[j] : A.base_tot[2] + L.mdoff[j]) : 0;
    v[O_CREF] = cref_pack(begin, cnt);
#pragma unroll
    for (int c = 0; c < kKeyOutCols; ++c) A.kd[c][dst] = v[c];
  } else if constexpr (FAM == 1) {
    uint64_t v[kNodeCols];
    const ulonglong2* row = (const ulonglong2*)(A.ns + (uint64_t)src * kChildStride);
#pragma unroll
    for (int c = 0; c < kNodeCols / 2; ++c) {
      const ulonglong2 q = row[c];
      v[2 * c] = q.x;
      v[2 * c + 1] = q.y;
    }
#pragma unroll
    for (int c = 0; c < kNodeCols; ++c) A.nd[c][dst] = v[c];
  } else {
    uint64_t v[kMemberCols];
    const ulonglong2* row = (const ulonglong2*)(A.ms + (uint64_t)src * kChildStride);
#pragma unroll
    for (int c = 0; c < kMemberCols / 2; ++c) {
      const ulonglong2 q = row[c];
      v[2 * c] = q.x;
      v[2 * c + 1] = q.y;
    }
#pragma unroll
    for (int c = 0; c < kMemberCols; ++c) A.md[c][dst] = v[c];
  }
}

// One wave per (family, chunk of kCompactChunk dense rows): the chunk's first bucket by a
// 64-ary search of the dense offsets, then groups of 64 buckets staged in LDS as above. Work
// per wave is bounded by the chunk, however the rows spread over buckets (an over-capacity
// bucket with millions of rows is split over many waves).
constexpr uint32_t kCompactChunk = 4096;

template <int FAM>
__device__ __forceinline__ void compact_chunk(const CompactArgs& A, CompactLds& L, uint64_t chunk, uint32_t nbuckets) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t* out = FAM == 0 ? A.kout : FAM == 1 ? A.nout : A.mout;
  const uint32_t* base = FAM == 0 ? A.kbase : FAM == 1 ? A.nbase : A.mbase;
  const uint32_t* doff = FAM == 0 ? A.kdoff : FAM == 1 ? A.ndoff : A.mdoff;
  const uint32_t total = doff[nbuckets - 1] + out[nbuckets - 1];
  if (chunk * kCompactChunk >= total) return;
  const uint32_t c0 = (uint32_t)(chunk * kCompactChunk), c1 = min(total, c0 + kCompactChunk);
  // last bucket j with doff[j] <= c0 (doff[0] = 0)
  uint32_t lo = 0, hi = nbuckets;
  while (hi - lo > 1) {
    const uint32_t step = (hi - lo + 63) / 64, idx = lo + lane * step;
    const uint64_t ok = __ballot(idx < hi && doff[idx] <= c0);
    const uint32_t k = 63 - __builtin_clzll(ok);  // lane 0 always holds
    lo += k * step;
    hi = min(hi, lo + step);
  }
  for (uint32_t b0 = lo; b0 < nbuckets; b0 += 64) {
    const uint32_t nb = min(64u, nbuckets - b0);
    const uint32_t b = b0 + min(lane, nb - 1);
    const bool in = lane < nb;
    const uint32_t d0 = doff[b0];
    const uint32_t dl = doff[b0 + nb - 1] + out[b0 + nb - 1];
    __builtin_amdgcn_wave_barrier();
    // padding lanes repeat the group end so the search never selects them
    L.doff[lane] = in ? doff[b] - d0 : dl - d0;
    L.sbase[lane] = base[b];
    if (FAM == 0) {
      L.ndoff[lane] = A.ndoff[b];
      L.mdoff[lane] = A.mdoff[b];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t tend = min(c1, dl) - d0;
    uint32_t t = max(c0, d0) - d0 + lane;
    for (; t + 64 < tend; t += 128) {
      compact_row<FAM>(A, L, t, d0);
      compact_row<FAM>(A, L, t + 64, d0);
    }
    if (t < tend) compact_row<FAM>(A, L, t, d0);
    if (dl >= c1) break;
  }
}

// Grid-stride over the (family, chunk) tasks; the task counts follow from the dense totals on
// the device, so one launch of any size covers a bucket range whose output size the host does
// not know (the pipelined bucket phase compacts each range while the next one merges).
__global__ void __launch_bounds__(kCompactWaves * 64) compact_kernel(CompactArgs A, uint32_t nbuckets) {
  __shared__ CompactLds lds_all[kCompactWaves];
  CompactLds& L = lds_all[threadIdx.x >> 6];
  if (nbuckets == 0 || (A.skip_if && *A.skip_if)) return;
  const uint32_t n1 = nbuckets - 1;
  const uint64_t ck = (A.kdoff[n1] + A.kout[n1] + kCompactChunk - 1) / kCompactChunk;
  const uint64_t cn = (A.ndoff[n1] + A.nout[n1] + kCompactChunk - 1) / kCompactChunk;
  const uint64_t cm = (A.mdoff[n1] + A.mout[n1] + kCompactChunk - 1) / kCompactChunk;
  for (uint64_t task = (uint64_t)blockIdx.x * kCompactWaves + (threadIdx.x >> 6); task < ck + cn + cm;
       task += (uint64_t)gridDim.x * kCompactWaves) {
    if (task < ck) compact_chunk<0>(A, L, task, nbuckets);
    else if (task < ck + cn) compact_chunk<1>(A, L, task - ck, nbuckets);
    else compact_chunk<2>(A, L, task - ck - cn, nbuckets);
  }
}

// Dense base of the next bucket range: base[p + 1] = base[p] + the range's totals (3 families).
__global__ void pipe_base_kernel(uint64_t* base, const uint64_t* tot) {
  if (threadIdx.x < 3) base[3 + threadIdx.x] = base[threadIdx.x] + tot[threadIdx.x];
}

template <typename T, typename OutT>
cdb_status exclusive_scan(cdb_ctx* ctx, const T* in, uint64_t n, OutT* out, OutT* out2, uint64_t* d_total,
                          hipStream_t s, int slot = WS_SCAN) {
  const uint64_t tiles = std::max<uint64_t>(1, (n + kScanTile - 1) / kScanTile);
  cdb_status st = CDB_OK;
  uint64_t* sums = (uint64_t*)ws_get(ctx, slot, tiles * sizeof(uint64_t), &st);
  if (!sums) return st;
  scan_reduce_kernel<T><<<tiles, kScanThreads, 0, s>>>(in, n, sums);
  scan_sums_kernel<<<1, kScanThreads, 0, s>>>(sums, tiles, d_total);
  scan_apply_kernel<T, OutT><<<tiles, kScanThreads, 0, s>>>(in, n, sums, out, out2);
  return launch_check(ctx, s, "scan");
}

struct Dir {  // per-family bucket directory
  uint32_t *hist, *base, *cursor, *out, *doff;
};

// Bucket plan: NB = d[0] * ... * d[levels-1] buckets, bucket(h) = floor((h << shift) * NB / 2^64).
struct Plan {
  int levels = 0;
  uint32_t d[4] = {1, 1, 1, 1};
  uint64_t nb = 1;
  bool seg_final = false;  // the last level runs per row-level segment (part_final_kernel)
};

Plan make_plan(uint64_t K, uint64_t N, uint64_t M, uint64_t fine_target = 0) {
  // Test hooks (the only environment knobs of the merge): CDB_PLAN_TARGET / CDB_PLAN_CTARGET
  // override the key / child rows per bucket, so that tests can push buckets into given tiers.
  // Wave-sized buckets: ~40 key rows and at most ~80 child rows (nodes + members) on average.
  // A wave holds 64 key rows (128 in the wide kernel) and 128 child rows, so only the
  // far tail of the bucket-size distribution reaches the workgroup tier. A key's children never
  // split across buckets, so when keys own many children each (more than 8 on average, as in C3:
  // ~300 member rows per key) wave-sized buckets cannot hold them and the wave kernels mostly
  // pass them on: such inputs get a few thousand large buckets instead, all merged by the
  // chip-wide child path (key table, tag sort, per-run fold). Measured C3 ms/step by child
  // target (key target 40): 40 22.0, 120 18.3, 240 16.1, 520 13.4, 1024 11.2, 4096 8.7; with key
  // target 120 as well, 4096 8.3. C5 (2 children per key) by child target: 40 26.0, 80 24.0,
  // 160-240 24.0 (key-bound); C1 and C4 have fewer children than keys and are key-bound.
  const bool child_heavy = N + M > 8 * K;
  uint64_t target = child_heavy ? 120 : (fine_target ? fine_target : 40);
  if (const char* e = std::getenv("CDB_PLAN_TARGET")) target = (uint64_t)std::max(8, std::min(120, std::atoi(e)));
  uint64_t ctarget = child_heavy ? 4096 : std::max<uint64_t>(target, 80);
  if (const char* e = std::getenv("CDB_PLAN_CTARGET")) ctarget = (uint64_t)std::max(8, std::min(65536, std::atoi(e)));
  const uint64_t want = std::max<uint64_t>({(K + target - 1) / target, (N + M + ctarget - 1) / ctarget, 1});
  Plan p;
  // The last level moves only a row index, so it takes a large fan-out (segments of
  // ~d_last buckets, a few hundred KB, stay cache-resident for the bucket kernels' gathers)
  // and the column-moving levels get small fan-outs (long contiguous write runs).
  const uint32_t dlast = 256;
  // Mode 2 (default): ONE moving level of fan-out d0 <= 2048 that writes rows, then the
  // per-segment final level (fan-out d1 <= 8192). Segments are then ~13 MB (all families): the
  // bucket kernels' row reads come from the Infinity Cache, one line per row, instead of
  // needing a second full column-moving pass to make segments L2-sized (mode 1).
  // (Mode 1, SoA levels before the row level so that segments are L2-sized, is what remains for
  // inputs too small or too large for mode 2.)
  const uint64_t d0pref = 768;  // measured on the C4 shard: 768 < 1024 < 512 < 2048 ms/step
  const uint64_t dcap = 1024;   // local digit slots of the row-level kernel
  if (want > 4096 && want <= dcap * kFinalMaxD) {
    p.levels = 2;
    p.seg_final = true;
    const uint64_t d0min = (want + kFinalMaxD - 1) / kFinalMaxD;
    p.d[0] = (uint32_t)std::min<uint64_t>(dcap, std::max(d0min, std::min(d0pref, (want + 63) / 64)));
    p.d[1] = (uint32_t)((want + p.d[0] - 1) / p.d[0]);
    p.nb = (uint64_t)p.d[0] * p.d[1];
    return p;
  }
  if (want <= 512) {  // one moving level that only turns the columns into rows
    p.levels = 2;
    p.d[0] = 1;
    p.d[1] = (uint32_t)want;
  } else {
    const uint64_t rest = (want + dlast - 1) / dlast;
    if (rest <= 512) {
      p.levels = 2;
      p.d[0] = (uint32_t)rest;
      p.d[1] = dlast;
    } else {
      p.levels = 3;
      uint32_t a = 1;
      while ((uint64_t)a * a < rest) ++a;
      p.d[0] = std::min<uint32_t>(a, 512);
      p.d[1] = (uint32_t)std::min<uint64_t>((rest + p.d[0] - 1) / p.d[0], 512);
      p.d[2] = (uint32_t)std::min<uint64_t>((want + (uint64_t)p.d[0] * p.d[1] - 1) / ((uint64_t)p.d[0] * p.d[1]), 512);
    }
  }
  p.nb = 1;
  for (int l = 0; l < p.levels; ++l) p.nb *= p.d[l];
  return p;
}

// Splits `n` rows of an NC-column family into plan.nb buckets (key-hash order). Levels
// 0..L-3 move the columns (SoA ping-pong through A / B); level L-2 moves them into W-word
// rows (AoS) in one of A / B, viewed as n x W words, and copies column 0 to `khcol`; the
// last level writes only `perm`, so bucket b's rows are rows[perm[base[b] .. base[b] +
// hist[b])]. Returns the row buffer in `rows` and the other ping-pong buffer in `spare`.
template <int NC, int W>
cdb_status partition_family(cdb_ctx* ctx, uint64_t* const* in, uint32_t in_stride, uint64_t n, const Plan& plan, int shift,
                            uint64_t* const* A, uint64_t* const* Bf, const Dir& d, uint64_t** rows,
                            uint64_t** spare, uint64_t* khcol, uint32_t* perm, hipStream_t s,
                            int scan_slot) {
  if (n == 0) {
    CDB_HIP(hipMemsetAsync(d.base, 0, sizeof(uint32_t) * plan.nb, s), "memset");
    CDB_HIP(hipMemsetAsync(d.hist, 0, sizeof(uint32_t) * plan.nb, s), "memset");
    *rows = A[0];
    for (int c = 0; c < NC; ++c) spare[c] = Bf[c];
    return CDB_OK;
  }
  const uint64_t tiles = (n + kPartTile - 1) / kPartTile;
  uint64_t* const* cur = in;
  uint64_t nprev = 1;
  for (int l = 0; l < plan.levels; ++l) {
    const int kind = l + 1 == plan.levels ? 2 : (l + 2 == plan.levels ? 1 : 0);  // 0 SoA, 1 rows, 2 index
    uint64_t* const* dst = (l % 2 == 0) ? A : Bf;
    const uint64_t ncur = nprev * plan.d[l];
    const uint64_t* col0 = kind == 2 ? khcol : cur[0];
    if (kind == 2 && plan.seg_final) {
      // the row level's directory (nprev segments) moves to out/doff, free until the merge;
      // the final level writes the bucket directory over base/hist
      CDB_HIP(hipMemcpyAsync(d.out, d.base, nprev * sizeof(uint32_t), hipMemcpyDeviceToDevice, s), "d2d");
      CDB_HIP(hipMemcpyAsync(d.doff, d.hist, nprev * sizeof(uint32_t), hipMemcpyDeviceToDevice, s), "d2d");
      part_final_kernel<<<(uint32_t)nprev, kFinalThreads, 0, s>>>(reinterpret_cast<const uint16_t*>(khcol), d.out,
                                                                  d.doff, nprev, plan.d[l], d.base, d.hist, perm);
      CDB_TRY(launch_check(ctx, s, "partition (final level)"));
      nprev = ncur;
      continue;
    }
    CDB_HIP(hipMemsetAsync(d.hist, 0, ncur * sizeof(uint32_t), s), "memset hist");
    part_hist_kernel<<<tiles, kPartThreads, 0, s>>>(col0, n, nprev, plan.d[l], shift, d.hist);
    CDB_TRY(launch_check(ctx, s, "part_hist"));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, d.hist, ncur, d.base, d.cursor, nullptr, s, scan_slot));
    if (kind == 2) {
      part_scatter_kernel<1, true><<<tiles, kPartThreads, 0, s>>>(ColSet<1>{{khcol}}, ColSet<1>{{nullptr}}, n,
                                                                  nprev, plan.d[l], shift, d.cursor, perm);
      CDB_TRY(launch_check(ctx, s, "partition (index level)"));
    } else {
      ColSet<NC> ci, co;
      for (int c = 0; c < NC; ++c) {  // the caller's rows (level 0) may be records, the workspace's are columns
        ci.c[c] = cur[c];
        ci.s[c] = (cur == in && c) ? in_stride : 1;
        co.c[c] = dst[c];
        co.s[c] = 1;
      }
      if (kind == 1) {
        // before a per-segment final level, leave each row's u16 digit in place of the key hash
        uint16_t* dig = plan.seg_final ? reinterpret_cast<uint16_t*>(khcol) : nullptr;
        const uint32_t d1 = plan.seg_final ? plan.d[l + 1] : 0;
        part_scatter_aos_kernel<NC, W, 1024, 1024><<<(n + 1023) / 1024, kPartThreads, 0, s>>>(
            ci, dst[0], khcol, n, nprev, plan.d[l], shift, d.cursor, dig, d1);
        CDB_TRY(launch_check(ctx, s, "partition (row level)"));
        *rows = dst[0];
        for (int c = 0; c < NC; ++c) spare[c] = (dst == A ? Bf : A)[c];
      } else {
        part_scatter_kernel<NC><<<tiles, kPartThreads, 0, s>>>(ci, co, n, nprev, plan.d[l], shift, d.cursor);
        CDB_TRY(launch_check(ctx, s, "partition"));
      }
      cur = dst;
    }
    nprev = ncur;
  }
  return CDB_OK;
}

}  // namespace

cdb_status stamp_pos(cdb_ctx* ctx, uint64_t* meta, uint64_t n, uint32_t pos, hipStream_t s) {
  if (n == 0) return CDB_OK;
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 4096);
  stamp_pos_kernel<<<(uint32_t)blocks, 256, 0, s>>>(meta, n, pos);
  return launch_check(ctx, s, "stamp_pos");
}

cdb_status state_rows(cdb_ctx* ctx, uint64_t* meta, uint64_t* aux, uint64_t n, hipStream_t s) {
  if (n == 0) return CDB_OK;
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 4096);
  state_rows_kernel<<<(uint32_t)blocks, 256, 0, s>>>(meta, aux, n);
  return launch_check(ctx, s, "state_rows");
}

namespace {
// The input families' layouts (cdb_dev_rows.stride): plain columns, or the hash column + records
// of ncols - 1 words.
struct InLayout {
  uint32_t ks = 1, ns = 1, ms = 1;
};
cdb_status input_layout(cdb_ctx* ctx, const cdb_dev_input* in, InLayout* lay) {
  const cdb_dev_rows* fam[3] = {&in->keys, &in->nodes, &in->members};
  const int ncols[3] = {kKeyCols, kNodeCols, kMemberCols};
  uint32_t* out[3] = {&lay->ks, &lay->ns, &lay->ms};
  for (int f = 0; f < 3; ++f) {
    const cdb_dev_rows& r = *fam[f];
    if (r.stride0 > 1) return fail(ctx, CDB_BAD_ARGUMENT, "input rows: col[0] must be a plain column (stride0 0 or 1)");
    if (r.stride <= 1) {
      *out[f] = 1;
      continue;
    }
    if (r.stride != (uint32_t)(ncols[f] - 1))
      return fail(ctx, CDB_BAD_ARGUMENT, "input rows: records layout needs stride = ncols - 1 (6 keys, 5 children)");
    for (int c = 2; c < ncols[f]; ++c)
      if (r.n && r.col[c] != r.col[1] + (c - 1))
        return fail(ctx, CDB_BAD_ARGUMENT, "input rows: records layout needs col[c] = col[1] + c - 1");
    *out[f] = r.stride;
  }
  return CDB_OK;
}

// Sorted-run input: checks the caller's run bounds, builds the run directories (run_mark_kernel)
// and, when every run really is ordered, the bucket directories of the three families. *ok =
// false sends the merge to the partition path (a run that decreases somewhere).
cdb_status runs_directory(cdb_ctx* ctx, const cdb_dev_input* in, const InLayout& lay, uint64_t nb, int shift,
                          const Dir* dirs, RunView* V, bool* ok, hipStream_t s) {
  *ok = false;
  const uint32_t nr = in->n_runs;
  if (nr > (uint32_t)kMaxRuns) return fail(ctx, CDB_BAD_ARGUMENT, "n_runs > 64");
  if (nr > (uint32_t)kMaxRuns / 2) return CDB_OK;  // a wave maps 2 nr child slices: partition path
  const cdb_dev_rows* fam[3] = {&in->keys, &in->nodes, &in->members};
  for (int f = 0; f < 3; ++f) {
    if (in->run_start[f][0] != 0 || in->run_start[f][nr] != fam[f]->n)
      return fail(ctx, CDB_BAD_ARGUMENT, "run_start must run from 0 to the family's row count");
    for (uint32_t r = 0; r < nr; ++r)
      if (in->run_start[f][r + 1] < in->run_start[f][r]) return fail(ctx, CDB_BAD_ARGUMENT, "run_start decreases");
  }
  cdb_status st = CDB_OK;
  const uint64_t row = nb + 1, per_fam = (uint64_t)nr * row;
  uint32_t* rdir = (uint32_t*)ws_get(ctx, WS_RUNDIR, 3 * per_fam * sizeof(uint32_t), &st);
  if (!rdir) return st;
  const uint32_t gap_cap = (uint32_t)std::min<uint64_t>(nr * (nb / kGapInline + 2), 1u << 30);
  uint8_t* rm = (uint8_t*)ws_get(ctx, WS_RUNMISC, 64 + 3 * (kMaxRuns + 1) * 8 + 3 * (uint64_t)gap_cap * 16, &st);
  if (!rm) return st;
  uint32_t* d_err = (uint32_t*)rm;            // err | gap_count[3]
  uint64_t* d_rbase = (uint64_t*)(rm + 64);   // 3 x 65 run starts
  uint32_t* d_gaps = (uint32_t*)(rm + 64 + 3 * (kMaxRuns + 1) * 8);
  for (int f = 0; f < 3; ++f)
    for (uint32_t r = 0; r <= (uint32_t)kMaxRuns; ++r)
      ctx->runs_host[f * (kMaxRuns + 1) + r] = r <= nr ? in->run_start[f][r] : in->run_start[f][nr];
  CDB_HIP(hipMemcpyAsync(d_rbase, ctx->runs_host, sizeof ctx->runs_host, hipMemcpyHostToDevice, s), "h2d runs");
  CDB_HIP(hipMemsetAsync(d_err, 0, 16, s), "memset");
  // the three families' directories are independent: nodes and members on the side streams
  CDB_HIP(hipEventRecord(ctx->ev_pfork, s), "event");
  CDB_HIP(hipStreamWaitEvent(ctx->side, ctx->ev_pfork, 0), "wait");
  CDB_HIP(hipStreamWaitEvent(ctx->side2, ctx->ev_pfork, 0), "wait");
  for (int f = 0; f < 3; ++f) {
    hipStream_t fs = f == 0 ? s : f == 1 ? ctx->side : ctx->side2;
    uint32_t* rd = rdir + f * per_fam;
    for (uint32_t r = 0; r < nr; ++r)  // empty runs: every bucket starts at the run's (absolute) first row
      if (in->run_start[f][r + 1] == in->run_start[f][r])
        CDB_HIP(hipMemsetD32Async((hipDeviceptr_t)(rd + r * row), (int)(uint32_t)in->run_start[f][r], row, fs),
                "memset run");
    const uint64_t n = fam[f]->n;
    if (n) {
      RunMarkArgs a;
      a.kh = fam[f]->col[0];
      a.rs = d_rbase + f * (kMaxRuns + 1);
      a.nr = nr;
      a.nb = nb;
      a.shift = shift;
      a.rdir = rd;
      a.gaps = d_gaps + (uint64_t)f * gap_cap * 4;
      a.gap_count = d_err + 1 + f;
      a.gap_cap = gap_cap;
      a.err = d_err;
      if (((uintptr_t)a.kh & 15) == 0) {
        const uint64_t blocks = std::min<uint64_t>((n / 4 + 256) / 256, 16384);
        run_mark4_kernel<<<(uint32_t)blocks, 256, 0, fs>>>(a, n);
      } else {
        const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 16384);
        run_mark_kernel<<<(uint32_t)blocks, 256, 0, fs>>>(a, n);
      }
      CDB_TRY(launch_check(ctx, fs, "run_mark_kernel"));
      run_gap_kernel<<<1024, 256, 0, fs>>>(a.gaps, a.gap_count, gap_cap, rd, nb);
      CDB_TRY(launch_check(ctx, fs, "run_gap_kernel"));
    }
    V->rdir[f] = rd;
  }
  CDB_HIP(hipEventRecord(ctx->ev_pn, ctx->side), "event");
  CDB_HIP(hipEventRecord(ctx->ev_pm, ctx->side2), "event");
  CDB_HIP(hipStreamWaitEvent(s, ctx->ev_pn, 0), "wait");
  CDB_HIP(hipStreamWaitEvent(s, ctx->ev_pm, 0), "wait");
  CDB_HIP(hipMemcpyAsync(&ctx->runs_err, d_err, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "d2h");
  CDB_HIP(hipStreamSynchronize(s), "sync");
  if (ctx->runs_err) return CDB_OK;  // a run is not ordered (or the gap list overflowed)
  for (int f = 0; f < 3; ++f) {
    uint64_t rs_sum = 0;
    for (uint32_t r = 0; r < nr; ++r) rs_sum += ctx->runs_host[f * (kMaxRuns + 1) + r];
    V->rs_sum[f] = (uint32_t)rs_sum;
  }
  V->bdir = nullptr;
  if (nr <= 8 && pipe_wave_wanted(nb)) {
    // the persistent wave tier's bucket-major directory, built with the three bucket directories
    uint32_t* bdir = (uint32_t*)ws_get(ctx, WS_RUNBDIR, row * kBdirRow * sizeof(uint32_t), &st);
    if (!bdir) return st;
    Reduce3Args a;
    a.rdir = rdir;
    a.nr = nr;
    a.nb = nb;
    for (int f = 0; f < 3; ++f) {
      a.rs_sum[f] = V->rs_sum[f];
      a.base[f] = dirs[f].base;
      a.cnt[f] = dirs[f].hist;
    }
    a.bdir = bdir;
    run_reduce3_kernel<<<(uint32_t)std::min<uint64_t>((row + 255) / 256, 8192), 256, 0, s>>>(a);
    CDB_TRY(launch_check(ctx, s, "run_reduce3_kernel"));
    V->bdir = bdir;
  } else {
    for (int f = 0; f < 3; ++f) {
      const uint64_t blocks = std::min<uint64_t>((nb + 255) / 256, 8192);
      run_reduce_kernel<<<(uint32_t)blocks, 256, 0, s>>>(V->rdir[f], nr, nb, V->rs_sum[f], dirs[f].base, dirs[f].hist);
      CDB_TRY(launch_check(ctx, s, "run_reduce_kernel"));
    }
  }
  V->rbase = d_rbase;
  V->nr = nr;
  V->nbp1 = (uint32_t)row;
  V->ks = lay.ks;
  V->ns = lay.ns;
  V->ms = lay.ms;
  for (int c = 0; c < kKeyCols; ++c) V->kin[c] = in->keys.col[c];
  for (int c = 0; c < kNodeCols; ++c) {
    V->nin[c] = in->nodes.col[c];
    V->min[c] = in->members.col[c];
  }
  *ok = true;
  return CDB_OK;
}
}  // namespace

// Stable LSD radix sort of n (u64 key, u32 value) pairs on bits [lo, bits) in 8-bit passes from
// lo; returns the buffers holding the result (the inputs or the spare pair).
cdb_status radix_sort_pairs(cdb_ctx* ctx, uint64_t** k, uint32_t** v, uint64_t* k2, uint32_t* v2, uint64_t n,
                            int lo, int bits, hipStream_t s) {
  if (n == 0) return CDB_OK;
  const uint32_t tiles = (uint32_t)((n + kRadixTile - 1) / kRadixTile);
  cdb_status st = CDB_OK;
  uint32_t* hist = (uint32_t*)ws_get(ctx, WS_RADIX, 2ull * 256 * tiles * sizeof(uint32_t), &st);
  if (!hist) return st;
  uint32_t* base = hist + 256ull * tiles;
  uint64_t *ka = *k, *kb = k2;
  uint32_t *va = *v, *vb = v2;
  for (int sh = lo; sh < bits; sh += 8) {
    radix_hist_kernel<<<tiles, kRadixThreads, 0, s>>>(ka, n, sh, hist, tiles);
    CDB_TRY(launch_check(ctx, s, "radix_hist_kernel"));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, hist, 256ull * tiles, base, (uint32_t*)nullptr, nullptr, s));
    radix_scatter_kernel<<<tiles, kRadixThreads, 0, s>>>(ka, va, n, sh, base, tiles, kb, vb);
    CDB_TRY(launch_check(ctx, s, "radix_scatter_kernel"));
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  *k = ka;
  *v = va;
  return CDB_OK;
}

cdb_status exclusive_scan_u32(cdb_ctx* ctx, const uint32_t* in, uint64_t n, uint64_t* out, uint64_t* d_total,
                              hipStream_t s) {
  return exclusive_scan<uint32_t, uint64_t>(ctx, in, n, out, (uint64_t*)nullptr, d_total, s);
}

namespace {

// The chip-wide child path (hot.hip.h) over one batch of buckets: ids in ascending order, their
// key rows (prefix hk_off) and child rows (prefix c_off); tk < 2^23 key rows and tc < 2^32 child
// rows in the batch (the key table's index width in the sort tag and the child row indices).
cdb_status chip_wide(cdb_ctx* ctx, BucketArgs& A, const std::vector<uint32_t>& wide_ids,
                     const std::vector<uint32_t>& hk_off, const std::vector<uint32_t>& c_off, uint64_t tk,
                     uint64_t tc, uint64_t cmax, uint64_t kmax, const RunView* rv, const RunView* orv,
                     uint64_t child_rows, hipStream_t s) {
  cdb_status st = CDB_OK;
  const bool run_order = orv != nullptr;  // sorted-run input (rv: and this batch reads its children from the runs)
  const uint32_t H = (uint32_t)wide_ids.size();
  // device: ids[H] | hk_off[H + 1] | c_off[H + 1] | hk_kout[H] | run count
  uint32_t* meta = (uint32_t*)ws_get(ctx, WS_HOTMETA, (6ull * H + 8) * sizeof(uint32_t), &st);
  if (!meta) return st;
  HotArgs HA;
  std::memset(&HA, 0, sizeof HA);
  if (rv) {  // children read from the runs (their rows were not copied)
    HA.runs = 1;
    HA.V = *rv;
  }
  uint32_t* d_ids = meta;
  uint32_t* d_hk_off = meta + H;
  uint32_t* d_c_off = d_hk_off + H + 1;
  HA.ids = d_ids;
  HA.hk_off = d_hk_off;
  HA.c_off = d_c_off;
  HA.hk_kout = d_c_off + H + 1;
  HA.first_run = HA.hk_kout + H;
  uint64_t* d_runs = (uint64_t*)(((uintptr_t)(HA.first_run + H) + 7) & ~(uintptr_t)7);
  HA.H = H;
  HA.n_children = tc;
  // Tag layout W = G << g_shift | id hash bits << 6 | pos, sorted on bits [lo, g_shift + gbits) in
  // 8-bit passes. On the sorted-run path (run_order) lo = 6: the pos bits are not sorted, the
  // stable sort keeps a W-run's rows in flat order, which is run order there -- fold order when
  // the runs are the fold positions (the fold checks, and takes the selection path where they
  // are not); a partition leaves a bucket's rows in arbitrary order, so lo = 0. The id bits only
  // separate a key's children: ids sharing them take the successor-selection fold (exact, but
  // slow for long runs), so a bucket of c children gets at least log2(c) + 9 of them (about
  // c / 1024 rows sharing), and where fewer than 34 bits reach the next pass boundary they save
  // whole passes: C3 (buckets of a few thousand children, a 400K-key table) sorts in 5 passes
  // instead of 8; C5's hottest keys keep all 34.
  int gbits = 0, cbits = 0;
  while (gbits < 32 && (tk >> gbits)) ++gbits;
  while (cbits < 40 && (cmax >> cbits)) ++cbits;
  const int min_id = std::max(kHotMinIdBits, cbits + 9);
  const int lo = run_order ? 6 : 0;
  const int passes = (gbits + 6 - lo + std::min(min_id, kHotIdBits - 6) + 7) / 8;
  int id_bits = std::min(kHotIdBits - 6, 8 * passes - 6 + lo - gbits);
  // Run order and buckets of at most kSortCap children: the per-bucket LDS path
  // (hot_sortfold_kernel), whose 32-bit tags take kSortIdBits id bits (test hook CDB_HOT_LDS=0:
  // the global sort for every batch).
  const char* lds_env = std::getenv("CDB_HOT_LDS");
  const bool lds = run_order && cmax <= kSortCap && !(lds_env && lds_env[0] == '0');
  if (lds) id_bits = kSortIdBits;
  // test hook: fewer id bits force the collision (successor-selection) fold
  if (const char* e = std::getenv("CDB_HOT_ID_BITS")) {
    const int bits = std::atoi(e);
    if (bits >= 1 && bits <= (lds ? kSortIdBits : kHotIdBits - 6)) id_bits = bits;
  }
  HA.g_shift = 6 + id_bits;
  HA.id_shift = 64 - id_bits;
  if (std::getenv("CDB_HOT_PROF"))  // test hook
    std::fprintf(stderr, "chip_wide: H %u tk %llu tc %llu cmax %llu kmax %llu gbits %d id_bits %d lds %d\n", H,
                 (unsigned long long)tk, (unsigned long long)tc, (unsigned long long)cmax, (unsigned long long)kmax,
                 gbits, id_bits, (int)lds);
  CDB_HIP(hipMemcpyAsync(d_ids, wide_ids.data(), H * 4, hipMemcpyHostToDevice, s), "h2d");
  CDB_HIP(hipMemcpyAsync(d_hk_off, hk_off.data(), (H + 1) * 4, hipMemcpyHostToDevice, s), "h2d");
  CDB_HIP(hipMemcpyAsync(d_c_off, c_off.data(), (H + 1) * 4, hipMemcpyHostToDevice, s), "h2d");
  const uint64_t nk = std::max<uint64_t>(tk, 1), nc = std::max<uint64_t>(tc, 1);
  uint8_t* kt = (uint8_t*)ws_get(ctx, WS_HOTK, nk * (4 * 8 + 4 * 4) + 64, &st);
  if (!kt) return st;
  HA.hk_h = (uint64_t*)kt;
  HA.hk_f = HA.hk_h + nk;
  HA.hk_vm = HA.hk_f + nk;
  HA.hk_sum = (unsigned long long*)(HA.hk_vm + nk);
  HA.hk_tp = (uint32_t*)(HA.hk_sum + nk);
  HA.hk_cnt = HA.hk_tp + nk;
  HA.hk_cb = HA.hk_cnt + nk;
  HA.hk_bkt = HA.hk_cb + nk;
  // (+ 40 B per child: the global fold's per-run stash, fold_rec / fold_hg)
  uint8_t* ct = (uint8_t*)ws_get(ctx, WS_HOTCH, nc * (32 + 2 * 8 + 2 * 4 + 6 * 4 + 40) + 64, &st);
  if (!ct) return st;
  HA.rec = (ulonglong2*)ct;  // (the workspace is 256-B aligned)
  ct += nc * 32;
  uint64_t* w = (uint64_t*)ct;
  uint64_t* w2 = w + nc;
  uint32_t* v = (uint32_t*)(w2 + nc);
  uint32_t* v2 = v + nc;
  HA.c_h = v2 + nc;
  HA.emit_n = HA.c_h + nc;
  HA.emit_m = HA.emit_n + nc;
  uint32_t* rank_n = HA.emit_m + nc;
  uint32_t* rank_m = rank_n + nc;
  uint32_t* run_list = rank_m + nc;
  HA.fold_rec = (ulonglong2*)(((uintptr_t)(run_list + nc) + 15) & ~(uintptr_t)15);
  HA.fold_hg = (uint2*)(HA.fold_rec + 2 * nc);
  HA.rank_n = rank_n;
  HA.rank_m = rank_m;
  HA.w = w;
  HA.v = v;
  if (kmax <= 256)
    hot_keys_kernel<256><<<H, kBktThreads, 0, s>>>(A, HA);
  else
    hot_keys_kernel<kCapK><<<H, kBktThreads, 0, s>>>(A, HA);
  CDB_TRY(launch_check(ctx, s, "hot_keys_kernel"));
  if (lds) {  // fold results per run go to the (unused) tag arrays
    HA.fold_v = w;
    HA.fold_q = v;
    // The fold reads each child's 32-B record, which the tag pass writes. CDB_HOT_DIRECT=1 (A/B and
    // test hook): it reads the child's row in the runs instead -- no record writes (C3: 0.95 GB less
    // written per step), but the rows' unaligned 32-B field reads cost more than the records: C3
    // 3.37-3.42 vs 3.22-3.29 ms per step.
    const char* direct_env = std::getenv("CDB_HOT_DIRECT");
    HA.direct = child_rows < (1ull << 30) && direct_env && direct_env[0] == '1';
    const bool prof = std::getenv("CDB_HOT_PROF") != nullptr;  // test hook: phase clocks to stderr
    if (prof) {
      HA.prof = nc >= 8 ? (unsigned long long*)w2 : nullptr;  // (the global sort's spare keys)
      if (HA.prof) CDB_HIP(hipMemsetAsync(HA.prof, 0, 64, s), "memset");
    }
    if (cmax <= SortSmall::Cap && kmax <= SortSmall::KCap)
      hot_sortfold_kernel<SortSmall><<<H, SortSmall::Threads, 0, s>>>(A, HA, id_bits);
    else
      hot_sortfold_kernel<SortBig><<<H, SortBig::Threads, 0, s>>>(A, HA, id_bits);
    CDB_TRY(launch_check(ctx, s, "hot_sortfold_kernel"));
    CDB_HIP(hipStreamSynchronize(s), "sync");  // the host vectors are copy sources
    if (prof && HA.prof) {
      uint64_t t[8];
      CDB_HIP(hipMemcpy(t, HA.prof, 64, hipMemcpyDeviceToHost), "d2h");
      const char* names[6] = {"tag", "sort", "runs", "fold0+scan", "fold1", "finish"};
      double tot = 0;
      for (int i = 0; i < 6; ++i) tot += (double)t[i];
      std::fprintf(stderr, "hot_sortfold H=%u tc=%llu:", H, (unsigned long long)tc);
      for (int i = 0; i < 6; ++i) std::fprintf(stderr, " %s %.1f%%", names[i], 100.0 * t[i] / std::max(tot, 1.0));
      std::fprintf(stderr, " (%.3f ms summed over workgroups / 256)\n", tot / 100e3 / 256);
    }
    return CDB_OK;
  }
  const uint32_t grid = (uint32_t)std::min<uint64_t>((tc + 255) / 256, 16384);
  if (tc) {
    HA.small_keys = kmax <= kTagKeys ? 1 : 0;
    // the global path's fold reads each child's row itself (v = the row): the tag writes no 32-B
    // records (test hook CDB_HOT_DIRECT=0: the records)
    const char* direct_env = std::getenv("CDB_HOT_DIRECT");
    HA.direct = child_rows < (1ull << 30) && !(direct_env && direct_env[0] == '0');
    // Children read from the runs: their lists are merged when they arrive sorted (a merge
    // result's child order, hot.hip.h), else radix-sorted (test hook CDB_HOT_MERGE=0: always sorted)
    const char* merge_env = std::getenv("CDB_HOT_MERGE");
    bool merged = false;
    if (run_order && orv->nr >= 2 && tc < (1ull << 31) && !(merge_env && merge_env[0] == '0')) {
      // (a batch of copied rows keeps each bucket's run slices in run order: the same lists)
      if (!HA.runs) HA.V = *orv;
      uint32_t L = 2;
      while (L < 2 * HA.V.nr) L <<= 1;
      const uint64_t jobs0 = (uint64_t)H * (L / 2);
      const uint64_t tiles_cap = tc / kMergeTile + jobs0 + 1;  // (a round's tiles: at most this many)
      uint8_t* mw = (uint8_t*)ws_get(ctx, WS_HOTMERGE, ((uint64_t)H * (L + 1) + 2 * jobs0) * 4 + tiles_cap * 8 + 128,
                                     &st);
      if (!mw) return st;
      uint64_t* d_ntiles = (uint64_t*)mw;
      uint32_t* d_unsorted = (uint32_t*)(mw + 8);
      uint32_t* bounds = (uint32_t*)(mw + 64);
      uint32_t* tcnt = bounds + (uint64_t)H * (L + 1);
      uint32_t* toff = tcnt + jobs0;
      uint2* splits = (uint2*)(((uintptr_t)(toff + jobs0) + 15) & ~(uintptr_t)15);
      CDB_HIP(hipMemsetAsync(d_unsorted, 0, 4, s), "memset");
      HA.inline_markers = 1;
      hot_lists_kernel<<<(H + 255) / 256, 256, 0, s>>>(HA, L, bounds, d_unsorted);
      CDB_TRY(launch_check(ctx, s, "hot_lists_kernel"));
      // sampled pairs first: an input out of child order skips the tag for the merge at once
      hot_sample_kernel<<<1, 256, 0, s>>>(A, HA, L, bounds, d_unsorted);
      CDB_TRY(launch_check(ctx, s, "hot_sample_kernel"));
      uint32_t unsorted = 0;
      CDB_HIP(hipMemcpyAsync(&unsorted, d_unsorted, 4, hipMemcpyDeviceToHost, s), "d2h");
      CDB_HIP(hipStreamSynchronize(s), "sync");
      if (!unsorted) {
        hot_tag_kernel<<<(uint32_t)((tc + kTagChunk - 1) / kTagChunk), 256, 0, s>>>(A, HA);
        CDB_TRY(launch_check(ctx, s, "hot_tag_kernel"));
        HA.orphans_counted = 1;  // (a fallback re-tag below must not count them twice)
        uint64_t *wa = w, *wb = w2;
        uint32_t *va = v, *vb = v2;
        for (uint32_t span = 1; span < L; span <<= 1) {
          MergeArgs M;
          M.bounds = bounds;
          M.L = L;
          M.span = span;
          M.n_jobs = (uint32_t)((uint64_t)H * (L / (2 * span)));
          M.tiles = toff;
          M.n_tiles = d_ntiles;
          M.wi = wa;
          M.vi = va;
          M.wo = wb;
          M.vo = vb;
          M.unsorted = d_unsorted;
          M.check = span == 1;
          MergeArgs Mc = M;
          Mc.tiles = tcnt;
          hot_merge_count_kernel<<<(M.n_jobs + 255) / 256, 256, 0, s>>>(Mc);
          CDB_TRY(launch_check(ctx, s, "hot_merge_count_kernel"));
          CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, tcnt, M.n_jobs, toff, (uint32_t*)nullptr, d_ntiles, s));
          const uint64_t tiles_max = tc / kMergeTile + M.n_jobs;
          hot_merge_split_kernel<<<(uint32_t)((tiles_max + 255) / 256), 256, 0, s>>>(M, splits);
          CDB_TRY(launch_check(ctx, s, "hot_merge_split_kernel"));
          hot_merge_kernel<<<(uint32_t)tiles_max, 256, 0, s>>>(M, splits);
          CDB_TRY(launch_check(ctx, s, "hot_merge_kernel"));
          std::swap(wa, wb);
          std::swap(va, vb);
        }
        CDB_HIP(hipMemcpyAsync(&unsorted, d_unsorted, 4, hipMemcpyDeviceToHost, s), "d2h");
        CDB_HIP(hipStreamSynchronize(s), "sync");
        if (!unsorted) {
          HA.w = wa;
          HA.v = va;
          HA.flagged = 1;
          merged = true;
          add_stat_kernel<<<1, 1, 0, s>>>(A.stats, ST_HOT_MERGED, tc);
          CDB_TRY(launch_check(ctx, s, "add_stat_kernel"));
        }
      }
      HA.inline_markers = 0;
      if (std::getenv("CDB_HOT_PROF"))  // test hook
        std::fprintf(stderr, "chip_wide: list merge of %u buckets x %u lists: %s\n", H, L,
                     merged ? "merged" : "a list is not sorted (radix sort)");
    }
    if (!merged) {
      hot_tag_kernel<<<(uint32_t)((tc + kTagChunk - 1) / kTagChunk), 256, 0, s>>>(A, HA);
      CDB_TRY(launch_check(ctx, s, "hot_tag_kernel"));
      // (per-bucket bitonic sorts in LDS measured slower than this global radix sort: C3 9.98 vs
      // 8.90 ms, C5 25.9 vs 24.3 ms; profiles/r03/experiments_r3.txt)
      CDB_TRY(radix_sort_pairs(ctx, &HA.w, &HA.v, w2, v2, tc, lo, HA.g_shift + gbits, s));
    }
    // the sort's other buffers are free now: fold results per run start
    HA.fold_v = HA.w == w ? w2 : w;
    HA.fold_q = HA.v == v ? v2 : v;
    HA.run_count = d_runs;
    HA.run_list = run_list;
    // run starts -> run list (ascending): per-tile counts in emit_n, their scan in rank_n
    const uint32_t ntile = (uint32_t)((tc + kRunTile - 1) / kRunTile);
    hot_runcount_kernel<<<ntile, 256, 0, s>>>(HA, HA.emit_n);
    CDB_TRY(launch_check(ctx, s, "hot_runcount_kernel"));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, HA.emit_n, ntile, rank_n, (uint32_t*)nullptr, d_runs, s));
    hot_runlist_kernel<<<ntile, 256, 0, s>>>(HA, rank_n);
    CDB_TRY(launch_check(ctx, s, "hot_runlist_kernel"));
    hot_first_run_kernel<<<(H + 255) / 256, 256, 0, s>>>(HA);
    CDB_TRY(launch_check(ctx, s, "hot_first_run_kernel"));
    // the fold's counts, folds and ranks are per run: the scans run over the runs, not the rows
    uint64_t nruns = 0;
    CDB_HIP(hipMemcpyAsync(&nruns, d_runs, sizeof nruns, hipMemcpyDeviceToHost, s), "d2h");
    CDB_HIP(hipStreamSynchronize(s), "sync");
    const uint32_t fgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nruns + 255) / 256, 16384));
    hot_fold_kernel<<<fgrid, 256, 0, s>>>(A, HA, 0);
    CDB_TRY(launch_check(ctx, s, "hot_fold_kernel"));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, HA.emit_n, nruns, rank_n, (uint32_t*)nullptr, nullptr, s));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, HA.emit_m, nruns, rank_m, (uint32_t*)nullptr, nullptr, s));
    hot_fold_kernel<<<fgrid, 256, 0, s>>>(A, HA, 1);
    CDB_TRY(launch_check(ctx, s, "hot_fold_kernel"));
  }
  hot_finish_kernel<<<H, 256, 0, s>>>(A, HA);
  CDB_TRY(launch_check(ctx, s, "hot_finish_kernel"));
  CDB_HIP(hipStreamSynchronize(s), "sync");  // the host vectors are copy sources
  return CDB_OK;
}

// Buckets beyond the workgroup tier's LDS pool (the mid kernel lists them), and the mid tier's
// buckets when there are many. Buckets whose keys fit the pool take the chip-wide child path, in
// batches of fewer than kHotKeyCap key rows (the key table's index width): a child-heavy input of
// any size stays on it. A bucket of more than kCapK key rows (or force_tier 4) runs the whole
// bucket algorithm on one workgroup over a global scratch slab (bucket_hot_kernel).
constexpr uint64_t kHotKeyCap = 1ull << 23;

// rv / runs_child_max: sorted-run input whose buckets of at most runs_child_max children (and at
// most kCapK keys) had only their keys copied (MatArgs): those take the chip-wide path in runs
// mode, in batches of their own.
cdb_status over_capacity(cdb_ctx* ctx, BucketArgs& A, const uint32_t* d_hot_list, uint32_t hot, hipStream_t s,
                         const RunView* rv = nullptr, uint32_t runs_child_max = 0, uint64_t child_rows = ~0ull) {
  cdb_status st = CDB_OK;
  uint32_t* d_cnt3 = (uint32_t*)ws_get(ctx, WS_HOTC3, 4ull * hot * sizeof(uint32_t), &st);
  if (!d_cnt3) return st;
  hot_counts_kernel<<<(hot + 255) / 256, 256, 0, s>>>(A, d_hot_list, hot, d_cnt3);
  CDB_TRY(launch_check(ctx, s, "hot_counts_kernel"));
  std::vector<uint32_t> ids(hot), cnt3(3ull * hot);
  CDB_HIP(hipMemcpyAsync(ids.data(), d_hot_list, hot * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "d2h");
  CDB_HIP(hipMemcpyAsync(cnt3.data(), d_cnt3, 3ull * hot * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "d2h");
  CDB_HIP(hipStreamSynchronize(s), "sync");
  const bool hprof = std::getenv("CDB_HOT_PROF") != nullptr;  // test hook: host clock to stderr
  const auto h0 = std::chrono::steady_clock::now();
  // (bucket id, list slot) sorted by bucket id: two 16-bit counting passes (std::sort took 0.48 ms
  // of host time on C5's 14.7K listed buckets)
  std::vector<uint64_t> packed(hot), spare(hot);
  for (uint32_t i = 0; i < hot; ++i) packed[i] = (uint64_t)ids[i] << 32 | i;
  for (int sh = 32; sh < 64; sh += 16) {
    std::vector<uint32_t> at(65537, 0);
    for (uint64_t x : packed) ++at[((x >> sh) & 0xFFFF) + 1];
    for (int d = 0; d < 65536; ++d) at[d + 1] += at[d];
    for (uint64_t x : packed) spare[at[(x >> sh) & 0xFFFF]++] = x;
    packed.swap(spare);
  }
  std::vector<uint32_t> order(hot);
  for (uint32_t i = 0; i < hot; ++i) order[i] = (uint32_t)packed[i];
  const double sort_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
  // test hook: a smaller batch cap runs the chip-wide path in many batches on small inputs
  uint64_t key_cap = kHotKeyCap;
  if (const char* e = std::getenv("CDB_HOT_KEY_CAP"))
    key_cap = std::max<uint64_t>(kCapK + 1, std::min<uint64_t>(kHotKeyCap, std::strtoull(e, nullptr, 10)));
  const bool legacy_all = A.force_tier == 4;
  std::vector<uint32_t> wide_ids, legacy;  // wide: the chip-wide child path
  std::vector<uint32_t> hk_off(1, 0), c_off(1, 0);
  std::vector<uint32_t> lk, ln, lm;
  uint64_t tk = 0, tc = 0, cmax = 0, kmax = 0, orphans = 0;
  bool runs_batch = false;  // the batch being built reads its children from the runs
  auto flush = [&]() -> cdb_status {
    if (wide_ids.empty()) return CDB_OK;
    if (hprof)
      std::fprintf(stderr, "over_capacity: hot %u, batch of %zu buckets after %.3f ms of host work (sort %.3f)\n",
                   hot, wide_ids.size(),
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count(), sort_ms);
    const cdb_status r =
        chip_wide(ctx, A, wide_ids, hk_off, c_off, tk, tc, cmax, kmax, runs_batch ? rv : nullptr, rv, child_rows, s);
    wide_ids.clear();
    hk_off.assign(1, 0);
    c_off.assign(1, 0);
    tk = tc = cmax = kmax = 0;
    return r;
  };
  // the same rule as mat_count_kernel's: runs-mode buckets first, then the copied ones
  auto runs_mode = [&](uint32_t i) {
    return rv && runs_child_max && !legacy_all && cnt3[3 * i] <= (uint32_t)kCapK &&
           cnt3[3 * i + 1] + cnt3[3 * i + 2] <= runs_child_max;
  };
  // Each kind in size classes: the sort's id bits follow the batch's largest bucket and its key
  // bits the batch's key count, so many small buckets and a few huge ones sorted together can take
  // a pass more than either alone (C5: 20.1 -> 19.6 ms split). On run order the LDS path's two
  // shapes are classes of their own (at most 2048 children and 256 keys; at most kSortCap
  // children), the rest takes the global sort.
  auto size_class = [&](uint32_t i) -> int {
    const uint32_t K = cnt3[3 * i], C = cnt3[3 * i + 1] + cnt3[3 * i + 2];
    if (!rv) return C > 16384 ? 2 : 1;
    if (C <= SortSmall::Cap && K <= SortSmall::KCap) return 0;
    return C <= kSortCap ? 1 : 2;
  };
  std::vector<uint32_t> lists[6];  // (runs mode ? 0 : 3) + size class, each in bucket order
  for (uint32_t i : order) lists[(runs_mode(i) ? 0 : 3) + size_class(i)].push_back(i);
  for (int pass = 0; pass < 6; ++pass) {
    runs_batch = pass < 3;
    for (uint32_t i : lists[pass]) {
      const uint32_t K = cnt3[3 * i], N = cnt3[3 * i + 1], M = cnt3[3 * i + 2];
      if (K == 0) {  // no key rows: every child is an orphan and nothing is output (the bucket's
        orphans += N + M;  // counts were zeroed when it was listed); kept off the chip-wide path,
        continue;          // whose per-bucket marker needs a key row
      }
      if (legacy_all || K > (uint32_t)kCapK) {
        legacy.push_back(ids[i]);
        lk.push_back(K);
        ln.push_back(N);
        lm.push_back(M);
        continue;
      }
      if (tk + K >= key_cap || tc + N + M >= (1ull << 32)) CDB_TRY(flush());
      wide_ids.push_back(ids[i]);
      tk += K;
      tc += N + M;
      cmax = std::max<uint64_t>(cmax, N + M);
      kmax = std::max<uint64_t>(kmax, K);
      hk_off.push_back((uint32_t)tk);
      c_off.push_back((uint32_t)tc);
    }
    CDB_TRY(flush());
  }
  if (orphans) {
    add_stat_kernel<<<1, 1, 0, s>>>(A.stats, ST_ORPHANS, orphans);
    CDB_TRY(launch_check(ctx, s, "add_stat_kernel"));
  }
  if (!legacy.empty()) {
    const uint32_t nl = (uint32_t)legacy.size();
    std::vector<uint64_t> off(nl);
    uint64_t total = 0;
    for (uint32_t i = 0; i < nl; ++i) {
      off[i] = total;
      total += hot_scratch_words(lk[i], std::max(ln[i], lm[i]));
      total = (total + 15) & ~uint64_t(15);
    }
    uint8_t* slab = (uint8_t*)ws_get(ctx, WS_HOT, total * 8 + nl * 12 + 64, &st);
    if (!slab) return st;
    uint64_t* d_off = (uint64_t*)(slab + total * 8);
    uint32_t* d_ids = (uint32_t*)(d_off + nl);
    CDB_HIP(hipMemcpyAsync(d_off, off.data(), nl * 8, hipMemcpyHostToDevice, s), "h2d");
    CDB_HIP(hipMemcpyAsync(d_ids, legacy.data(), nl * 4, hipMemcpyHostToDevice, s), "h2d");
    A.hot_in = d_ids;
    A.hot_scratch = (uint64_t*)slab;
    A.hot_scratch_off = d_off;
    bucket_hot_kernel<<<nl, kBktThreads, 0, s>>>(A);
    CDB_TRY(launch_check(ctx, s, "bucket_hot_kernel"));
    CDB_HIP(hipStreamSynchronize(s), "sync");  // the host vectors above are copy sources
  }
  return CDB_OK;
}
}  // namespace

cdb_status merge_device_impl(cdb_ctx* ctx, const cdb_dev_input* in, const cdb_merge_opts* opts,
                             cdb_dev_output* out, cdb_merge_stats* stats, hipStream_t s) {
  const uint64_t K = in->keys.n, N = in->nodes.n, M = in->members.n;
  if (in->n_pos > (uint32_t)kMaxPos) return fail(ctx, CDB_BAD_ARGUMENT, "at most 63 fold positions per merge");
  if (K >= (1ull << 32) || N >= (1ull << 32) || M >= (1ull << 32))
    return fail(ctx, CDB_BAD_ARGUMENT, "row counts must be < 2^32 per family per device");
  const uint32_t flags = opts ? opts->flags : 0;
  const uint64_t wm = opts ? opts->gc_watermark : 0;
  InLayout lay;
  CDB_TRY(input_layout(ctx, in, &lay));
  Plan plan = make_plan(K, N, M);
  // Sorted runs that the persistent wave tier will merge (at most 8 per family, enough buckets):
  // finer buckets, which its units group back to one wave's worth of rows each (runs.hip.h), so
  // that no bucket is beyond a wave and the waves' lanes are full. (A run found out of order sends
  // the merge to the partition path with these buckets: the same result.)
  if (in->n_runs && in->n_runs <= 8 && pipe_wave_wanted(plan.nb) && !std::getenv("CDB_PLAN_TARGET") && groups_wanted()) {
    const Plan fine = make_plan(K, N, M, pipe_fine_target());
    if (fine.nb > plan.nb) plan = fine;
  }
  const int shift = opts ? (int)opts->key_shift : 0;
  if (shift < 0 || shift > 16) return fail(ctx, CDB_BAD_ARGUMENT, "key_shift");
  const uint64_t nb = plan.nb;
  cdb_status st = CDB_OK;

  // ---- workspace
  auto cols = [&](int slot, int ncol, uint64_t rows, uint64_t** p) -> cdb_status {
    const uint64_t r = std::max<uint64_t>(rows, 1);
    uint64_t* base = (uint64_t*)ws_get(ctx, slot, ncol * r * sizeof(uint64_t), &st);
    if (!base) return st;
    for (int c = 0; c < ncol; ++c) p[c] = base + c * r;
    return CDB_OK;
  };
  uint64_t *KA[8], *KB[8], *NA[6], *NB[6], *MA[6], *MBf[6];
  CDB_TRY(cols(WS_KA, 8, K, KA));
  CDB_TRY(cols(WS_KB, 8, K, KB));
  CDB_TRY(cols(WS_NA, 6, N, NA));
  CDB_TRY(cols(WS_NB, 6, N, NB));
  CDB_TRY(cols(WS_MA, 6, M, MA));
  CDB_TRY(cols(WS_MB, 6, M, MBf));
  const uint64_t dn = nb + 1;
  uint32_t* dir = (uint32_t*)ws_get(ctx, WS_DIR, 15 * dn * sizeof(uint32_t), &st);
  if (!dir) return st;
  Dir dk{dir, dir + dn, dir + 2 * dn, dir + 3 * dn, dir + 4 * dn};
  Dir dnd{dir + 5 * dn, dir + 6 * dn, dir + 7 * dn, dir + 8 * dn, dir + 9 * dn};
  Dir dm{dir + 10 * dn, dir + 11 * dn, dir + 12 * dn, dir + 13 * dn, dir + 14 * dn};
  // misc: (64) | last_bad u64 at 64 | totals[3] u64 | hot_count u32 | big_count u32 | compaction error u32 |
  //       pipelined compaction error u32 | beyond-wide flag u32 at 112 | zero[3] u64 at 128 |
  //       stats[ST_COUNT] u64 at 160 | hot_list[nb] u32 at 256 | big_list[nb] u32
  uint8_t* misc = (uint8_t*)ws_get(ctx, WS_MISC, 256 + 2 * nb * sizeof(uint32_t), &st);
  if (!misc) return st;
  static_assert(ST_COUNT * 8 <= 96, "statistics fit the misc header");
  unsigned long long* d_stats = (unsigned long long*)(misc + 160);
  unsigned long long* d_last_bad = (unsigned long long*)(misc + 64);
  uint64_t* d_totals = (uint64_t*)(misc + 72);
  uint32_t* d_hot_count = (uint32_t*)(misc + 96);
  uint32_t* d_big_count = (uint32_t*)(misc + 100);
  uint32_t* d_hot_list = (uint32_t*)(misc + 256);
  uint32_t* d_big_list = d_hot_list + nb;
  CDB_HIP(hipMemsetAsync(misc, 0, 256, s), "memset misc");
  unsigned long long* d_shards =
      (unsigned long long*)ws_get(ctx, WS_STATS, kStatShards * kStatStride * sizeof(unsigned long long), &st);
  if (!d_shards) return st;
  CDB_HIP(hipMemsetAsync(d_shards, 0, kStatShards * kStatStride * sizeof(unsigned long long), s), "memset stats");

  merge_begin_marker<<<1, 1, 0, s>>>();
  CDB_HIP(hipEventRecord(ctx->ev0, s), "event");
  // ---- 1. bucket partition of each family by (parent) key hash, or, for sorted runs, the
  //         run directories (runs.hip.h)
  uint64_t *krows = nullptr, *nrows = nullptr, *mrows = nullptr;
  uint64_t *ksp[8], *nsp[6], *msp[6];
  uint64_t* kin[8];
  uint64_t* nin[6];
  uint64_t* min_[6];
  for (int c = 0; c < 8; ++c) kin[c] = in->keys.col[c];
  for (int c = 0; c < 6; ++c) {
    nin[c] = in->nodes.col[c];
    min_[c] = in->members.col[c];
  }
  uint32_t* perm = (uint32_t*)ws_get(ctx, WS_PERM, (K + N + M + 3) * sizeof(uint32_t), &st);
  if (!perm) return st;
  uint32_t *kperm = perm, *nperm = perm + K, *mperm = perm + K + N;
  RunView RV;
  std::memset(&RV, 0, sizeof RV);
  bool use_runs = false;
  if (in->n_runs) {
    const Dir dirs[3] = {dk, dnd, dm};
    CDB_TRY(runs_directory(ctx, in, lay, nb, shift, dirs, &RV, &use_runs, s));
  }
  if (use_runs) {  // rows stay in the runs; KA/NA/MA take the rows of the workgroup tiers
    krows = KA[0];
    nrows = NA[0];
    mrows = MA[0];
    for (int c = 0; c < 8; ++c) ksp[c] = KB[c];
    for (int c = 0; c < 6; ++c) {
      nsp[c] = NB[c];
      msp[c] = MBf[c];
    }
  } else {
  uint64_t* khcol = (uint64_t*)ws_get(ctx, WS_KHCOL, (K + N + M + 3) * sizeof(uint64_t), &st);
  if (!khcol) return st;
  // the three families partition independently (own buffers, directories, scan scratch):
  // nodes and members run on side streams beside the keys
  hipStream_t sn = ctx->side, sm = ctx->side2;
  CDB_HIP(hipEventRecord(ctx->ev_pfork, s), "event");
  CDB_HIP(hipStreamWaitEvent(sn, ctx->ev_pfork, 0), "wait");
  CDB_HIP(hipStreamWaitEvent(sm, ctx->ev_pfork, 0), "wait");
  CDB_TRY(partition_family<kKeyCols, kKeyStride>(ctx, kin, lay.ks, K, plan, shift, KA, KB, dk, &krows, ksp, khcol,
                                                 kperm, s, WS_SCAN));
  CDB_TRY(partition_family<kNodeCols, kChildStride>(ctx, nin, lay.ns, N, plan, shift, NA, NB, dnd, &nrows, nsp,
                                                    khcol + K, nperm, sn, WS_SCAN2));
  CDB_TRY(partition_family<kMemberCols, kChildStride>(ctx, min_, lay.ms, M, plan, shift, MA, MBf, dm, &mrows, msp,
                                                      khcol + K + N, mperm, sm, WS_SCAN3));
  CDB_HIP(hipEventRecord(ctx->ev_pn, sn), "event");
  CDB_HIP(hipEventRecord(ctx->ev_pm, sm), "event");
  CDB_HIP(hipStreamWaitEvent(s, ctx->ev_pn, 0), "wait");
  CDB_HIP(hipStreamWaitEvent(s, ctx->ev_pm, 0), "wait");
  {  // sparse key outputs (8 columns) go to the ping-pong buffer that does not hold the rows
    uint64_t* const* free_k = (krows == KA[0]) ? KB : KA;
    for (int c = 0; c < 8; ++c) ksp[c] = free_k[c];
  }
  }  // partition path

  CDB_HIP(hipEventRecord(ctx->ev_part, s), "event");
  // ---- 2. GC watermark scan (DB::gc's LIFO stop point)
  if ((flags & CDB_MERGE_GC_DELETES) && K) {
    gc_lastbad_kernel<<<1024, 256, 0, s>>>(in->keys.col[K_CT], in->keys.col[K_META], lay.ks, K, wm, d_last_bad);
    CDB_TRY(launch_check(ctx, s, "gc_lastbad"));
  }

  // ---- 3. fused bucket merge
  BucketArgs A;
  std::memset(&A, 0, sizeof A);
  A.kr = krows;
  A.nr = nrows;
  A.mr = mrows;
  // sparse outputs, AoS, in the ping-pong buffers that do not hold the rows (8 / 6 columns of
  // K / N / M rows each: exactly K / N / M output rows)
  A.kos = ksp[0];
  A.nos = nsp[0];
  A.mos = msp[0];
  A.kp = kperm; A.np = nperm; A.mp = mperm;
  A.kbase = dk.base; A.kcnt = dk.hist;
  A.nbase = dnd.base; A.ncnt = dnd.hist;
  A.mbase = dm.base; A.mcnt = dm.hist;
  A.nbuckets = nb;
  A.kout = dk.out; A.nout = dnd.out; A.mout = dm.out;
  A.flags = (flags & CDB_MERGE_STRICT_DICT_PANIC ? F_DICT_STRICT : 0) |
            (flags & CDB_MERGE_GC_DELETES ? F_GC_DELETES : 0) | (flags & CDB_MERGE_GC_MEMBERS ? F_GC_MEMBERS : 0);
  A.gc_wm = wm;
  A.force_tier = opts ? opts->force_tier : 0;
  A.key_shift = shift;
  A.bw = ~0ull / nb;
  {
    const uint64_t span = A.bw + 2 * nb + 2;  // > the hash span of any bucket measured from b * bw
    int bits = 0;
    while (bits < 64 && (span >> bits)) ++bits;
    if (span < A.bw) bits = 64;  // (wrapped: a handful of buckets)
    A.rel_shift = bits > 44 ? bits - 44 : 0;
  }
  A.last_bad = (const uint64_t*)d_last_bad;
  A.stats = d_shards;
  A.hot_list = d_hot_list;
  A.hot_count = d_hot_count;
  // zero dense bases of the compaction (a pipelined range adds its range base instead)
  const unsigned long long* d_zero3 = (const unsigned long long*)(misc + 128);
  WaveArgs WA;
  WA.A = A;
  WA.nbuckets = (uint32_t)nb;
  WA.blo = 0;
  WA.bhi = (uint32_t)nb;
  WA.big_list = d_big_list;
  WA.big_count = d_big_count;
  WA.V = RV;
  WA.units = nullptr;
  // counters: the wide tier's per range [0, 64), the persistent wave tier's per (range, XCD slab)
  uint32_t* d_wide = (uint32_t*)ws_get(ctx, WS_WIDE, (64 + 64 * kXcds) * sizeof(uint32_t), &st);
  if (!d_wide) return st;
  CDB_HIP(hipMemsetAsync(d_wide, 0, (64 + 64 * kXcds) * sizeof(uint32_t), s), "memset wide");
  // the persistent wave tier (runs of at most 8 per family): one resident grid
  const bool wave_pipe = use_runs && RV.bdir != nullptr && nb < (1ull << 28);  // (a unit: one word)
  const uint32_t pipe_grid = wave_pipe ? pipe_wave_grid(ctx) : 0;
  CDB_HIP(hipEventRecord(ctx->ev_fork, s), "event");  // inputs of both bucket tiers are ready
  // The wave and wide tiers run over P consecutive bucket ranges. Range p is scanned and compacted
  // into the dense outputs on stream cs while range p + 1 merges: the tiers are VALU-bound and
  // the compaction HBM-bound, so the two overlap. Only valid when no bucket goes to a workgroup
  // tier (those add outputs after every range): then everything is compacted again at the end.
  // (small merges: the ranges' extra launches cost more than the overlap wins; C1 0.8 -> 1.6 ms)
  // A bucket beyond the wide tier's capacity goes to a workgroup tier, which adds outputs after
  // every range, so the range compactions would stand down and only their scans would run (C5:
  // 24 idle scans per step): such merges run as one range (one flag read before the bucket phase).
  // The bucket layout (out->compact == 0) has no compaction to overlap: one range.
  constexpr uint32_t kPipeRanges = 8;
  const bool dense_out = out->compact != 0;
  const uint32_t pipe_opt = (opts && dense_out) ? opts->pipe_ranges : 0;
  bool pipe_auto = dense_out && !(K + N + M < (64ull << 20) || nb < 64ull * kPipeRanges);
  if (!pipe_opt && pipe_auto) {
    uint32_t* d_over = (uint32_t*)(misc + 112);  // zeroed with the misc header
    beyond_wide_kernel<<<(uint32_t)std::min<uint64_t>((nb + 255) / 256, 4096), 256, 0, s>>>(A, (uint32_t)nb, d_over);
    CDB_TRY(launch_check(ctx, s, "beyond_wide_kernel"));
    uint32_t over = 0;
    CDB_HIP(hipMemcpyAsync(&over, d_over, sizeof over, hipMemcpyDeviceToHost, s), "d2h");
    CDB_HIP(hipStreamSynchronize(s), "sync");
    pipe_auto = over == 0;
  }
  const uint32_t P = pipe_opt ? (uint32_t)std::min<uint64_t>({pipe_opt, std::max<uint64_t>(nb, 1), 64})
                     : pipe_auto ? kPipeRanges : 1;
  const bool pipelined = P > 1;
  if (wave_pipe) {  // the persistent tier's units (runs.hip.h): a group's hash span must fit the
                    // sort word as one bucket's does. Where fewer than 4 buckets fit (below ~2^22
                    // buckets; below ~2^21 one bucket's span already needs a shifted word, and the
                    // child lookup compares shifted words) the shift grows to fit kGroupMax buckets,
                    // so that groups form at every size (an equal shifted word of two hashes goes to
                    // the exact tier, as ever)
    if (groups_wanted() && !A.force_tier &&
        (unsigned __int128)4 * A.bw + 2 * nb + 2 >= (unsigned __int128)1 << (44 + A.rel_shift)) {
      const unsigned __int128 span = (unsigned __int128)kGroupMax * A.bw + 2 * nb + 2;
      int bits = 0;
      while (bits < 80 && (span >> bits)) ++bits;
      A.rel_shift = std::max(A.rel_shift, std::min(bits, 64) - 44);
      WA.A.rel_shift = A.rel_shift;
    }
    const unsigned __int128 lim = (unsigned __int128)1 << (44 + A.rel_shift);
    uint64_t g = 1;
    while (g < kGroupMax && (unsigned __int128)(g + 1) * A.bw + 2 * nb + 2 < lim) ++g;
    UnitArgs ua;
    ua.kcnt = A.kcnt;
    ua.ncnt = A.ncnt;
    ua.mcnt = A.mcnt;
    ua.nb = nb;
    ua.P = P;
    ua.gmax = (A.force_tier || !groups_wanted()) ? 1u : (uint32_t)g;
    ua.ccap = group_ccap();
    const uint64_t words = (nb + 31) / 32 + 3;
    ua.units = (uint32_t*)ws_get(ctx, WS_UNITS, words * sizeof(uint32_t), &st);
    if (!ua.units) return st;
    pipe_units_kernel<<<(uint32_t)std::min<uint64_t>((words + 7) / 8, 4096), 256, 0, s>>>(ua);
    CDB_TRY(launch_check(ctx, s, "pipe_units_kernel"));
    WA.units = ua.units;
    // the wide tier's side-stream launch waits for the units too, so that it is not dispatched
    // while the persistent kernel waits behind them (it then holds CUs the persistent grid needs:
    // +1.3 ms measured with one-bucket units)
    CDB_HIP(hipEventRecord(ctx->ev_fork, s), "event");
  }
  CompactArgs C;
  C.ks = ksp[0];
  C.ns = nsp[0];
  C.ms = msp[0];
  for (int c = 0; c < kKeyOutCols; ++c) C.kd[c] = out->keys.col[c];
  for (int c = 0; c < kNodeCols; ++c) {
    C.nd[c] = out->nodes.col[c];
    C.md[c] = out->members.col[c];
  }
  C.kbase = dk.base; C.nbase = dnd.base; C.mbase = dm.base;
  C.kout = dk.out; C.nout = dnd.out; C.mout = dm.out;
  C.kdoff = dk.doff; C.ndoff = dnd.doff; C.mdoff = dm.doff;
  C.base_tot = d_zero3;
  C.cap[0] = K;
  C.cap[1] = N;
  C.cap[2] = M;
  uint32_t* d_cerr = (uint32_t*)(misc + 104);   // zeroed with the misc header
  uint32_t* d_cerr_p = (uint32_t*)(misc + 108);  // the pipelined compaction's
  C.err = d_cerr;
  C.skip_if = nullptr;
  C.state = 0;
  C.ds[0] = C.ds[1] = C.ds[2] = 1;
  uint64_t* d_pipe = nullptr;  // [P + 1][3] dense bases | [P][3] range totals
  hipStream_t ws = ctx->side;
  hipStream_t cs = ctx->side2;
  CDB_HIP(hipStreamWaitEvent(ws, ctx->ev_fork, 0), "wait");
  if (pipelined) {
    d_pipe = (uint64_t*)ws_get(ctx, WS_PIPE, (6 * P + 3) * sizeof(uint64_t), &st);
    if (!d_pipe) return st;
    CDB_HIP(hipStreamWaitEvent(cs, ctx->ev_fork, 0), "wait");
    CDB_HIP(hipMemsetAsync(d_pipe, 0, 3 * sizeof(uint64_t), cs), "memset pipe");
  }
  for (uint32_t p = 0; p < P; ++p) {
    const uint32_t lo = (uint32_t)(nb * p / P), hi = (uint32_t)(nb * (p + 1) / P), nr_b = hi - lo;
    WA.blo = lo;
    WA.bhi = hi;
    if (nr_b == 0) continue;
    // the wide tier strides over its buckets beside the wave tier: 256 workgroups (one per CU)
    // measured ~1 ms faster per C4 step than 1024, which crowd the wave tier's workgroups out
    const uint32_t gw = (uint32_t)std::min<uint64_t>((nr_b + 64 * kWavesPerWG - 1) / (64 * kWavesPerWG), 256);
    // behind the wave tier, a wider launch of the same kernel takes the wide groups still left
    // (they share the range's counter; with none left its workgroups exit at once)
    const uint32_t gt = (uint32_t)std::min<uint64_t>((nr_b + 64 * kWavesPerWG - 1) / (64 * kWavesPerWG), 1024);
    WA.wide_next = d_wide + p;  // (P <= 64: the counters were zeroed before the fork)
    WA.pipe_next = d_wide + 64 + kXcds * p;
    static const bool wide_first = std::getenv("CDB_WIDE_FIRST") != nullptr;  // A/B hook
    if (wave_pipe && wide_first) {
      bucket_wide_runs_kernel<<<gt, kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wide_runs_kernel"));
      const uint32_t g = (uint32_t)std::min<uint64_t>(pipe_grid, (nr_b + kPipeChunk - 1) / kPipeChunk * kXcds);
      const bool rec = RV.ks == kKeyCols - 1 && RV.ns == kNodeCols - 1 && RV.ms == kMemberCols - 1;
      if (rec)
        bucket_wave_pipe_kernel<true><<<std::max<uint32_t>(g, 1), kWavesPerWG * 64, 0, s>>>(WA);
      else
        bucket_wave_pipe_kernel<false><<<std::max<uint32_t>(g, 1), kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wave_pipe_kernel"));
    } else if (wave_pipe) {
      const uint32_t g = (uint32_t)std::min<uint64_t>(pipe_grid, (nr_b + kPipeChunk - 1) / kPipeChunk * kXcds);
      const bool rec = RV.ks == kKeyCols - 1 && RV.ns == kNodeCols - 1 && RV.ms == kMemberCols - 1;
      if (rec)
        bucket_wave_pipe_kernel<true><<<std::max<uint32_t>(g, 1), kWavesPerWG * 64, 0, s>>>(WA);
      else
        bucket_wave_pipe_kernel<false><<<std::max<uint32_t>(g, 1), kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wave_pipe_kernel"));
      bucket_wide_runs_kernel<<<gw, kWavesPerWG * 64, 0, ws>>>(WA);
      CDB_TRY(launch_check(ctx, ws, "bucket_wide_runs_kernel"));
      bucket_wide_runs_kernel<<<gt, kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wide_runs_kernel"));
    } else if (use_runs) {
      bucket_wave_runs_kernel<<<(nr_b + kWavesPerWG - 1) / kWavesPerWG, kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wave_runs_kernel"));
      // the wide tier's buckets are disjoint from the wave tier's: beside it on a side stream
      bucket_wide_runs_kernel<<<gw, kWavesPerWG * 64, 0, ws>>>(WA);
      CDB_TRY(launch_check(ctx, ws, "bucket_wide_runs_kernel"));
      bucket_wide_runs_kernel<<<gt, kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wide_runs_kernel"));
    } else {
      bucket_wave_kernel<<<(nr_b + kWavesPerWG - 1) / kWavesPerWG, kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wave_kernel"));
      bucket_wide_kernel<<<gw, kWavesPerWG * 64, 0, ws>>>(WA);
      CDB_TRY(launch_check(ctx, ws, "bucket_wide_kernel"));
      bucket_wide_kernel<<<gt, kWavesPerWG * 64, 0, s>>>(WA);
      CDB_TRY(launch_check(ctx, s, "bucket_wide_kernel"));
    }
    if (pipelined) {  // range p: scans and compaction on cs once both tiers are through it
      CDB_HIP(hipEventRecord(ctx->ev_cs, s), "event");
      CDB_HIP(hipStreamWaitEvent(cs, ctx->ev_cs, 0), "wait");
      CDB_HIP(hipEventRecord(ctx->ev_cw, ws), "event");
      CDB_HIP(hipStreamWaitEvent(cs, ctx->ev_cw, 0), "wait");
      uint64_t* base = d_pipe + 3 * p;
      uint64_t* tot = d_pipe + 3 * (P + 1) + 3 * p;
      CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, dk.out + lo, nr_b, dk.doff + lo, (uint32_t*)nullptr, tot + 0, cs,
                                                 WS_SCAN2));
      CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, dnd.out + lo, nr_b, dnd.doff + lo, (uint32_t*)nullptr, tot + 1,
                                                 cs, WS_SCAN2));
      CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, dm.out + lo, nr_b, dm.doff + lo, (uint32_t*)nullptr, tot + 2, cs,
                                                 WS_SCAN2));
      pipe_base_kernel<<<1, 64, 0, cs>>>(base, tot);
      CDB_TRY(launch_check(ctx, cs, "pipe_base_kernel"));
      CompactArgs Cp = C;
      Cp.kbase += lo; Cp.nbase += lo; Cp.mbase += lo;
      Cp.kout += lo; Cp.nout += lo; Cp.mout += lo;
      Cp.kdoff += lo; Cp.ndoff += lo; Cp.mdoff += lo;
      Cp.base_tot = (const unsigned long long*)base;
      Cp.err = d_cerr_p;
      Cp.skip_if = d_big_count;  // (pushed during this or an earlier range's merge)
      compact_kernel<<<1024, 64 * kCompactWaves, 0, cs>>>(Cp, nr_b);
      CDB_TRY(launch_check(ctx, cs, "compact_kernel"));
    }
  }
  CDB_HIP(hipEventRecord(ctx->ev_join, ws), "event");
  CDB_HIP(hipStreamWaitEvent(s, ctx->ev_join, 0), "wait");
  WA.blo = 0;
  WA.bhi = (uint32_t)nb;
  // ---- 4. buckets beyond the wave tiers: the mid tier (one workgroup per bucket, LDS), or,
  //         when there are many of them, the chip-wide child path of the over-capacity
  //         buckets (hot.hip.h): buckets of a few keys with hundreds of children each (C3's
  //         sets) sort their children serially inside one workgroup, but spread over the chip
  //         they fold in parallel; then the over-capacity buckets
  uint32_t counts[2] = {0, 0};  // hot, big (mid tier)
  CDB_HIP(hipMemcpyAsync(counts, d_hot_count, sizeof counts, hipMemcpyDeviceToHost, s), "d2h");
  CDB_HIP(hipStreamSynchronize(s), "sync");
  constexpr uint32_t kMidChipWide = 4096;  // mid-tier buckets from which they go chip-wide
  const bool mid_wide = A.force_tier == 0 && counts[1] >= kMidChipWide;
  // Going chip-wide from sorted runs, buckets keep their children in the runs (only their keys
  // are copied): the tag pass reads each bucket's run slices in order and writes the fold's
  // records, so a copy of the children first only costs (C3: 1.35 ms of copies; C5 with copies
  // of the buckets over 16K children 21.5 ms, without 20.2). With fewer than kMidChipWide mid
  // buckets the over-capacity ones still take the copy batch (children copied by mat_copy).
  constexpr uint32_t kRunsChildMax = 0xFFFFFFFFu;
  const uint32_t runs_child_max = (use_runs && mid_wide) ? kRunsChildMax : 0;
  // (no bucket went to the workgroup tiers -- C1 and C4 -- : neither their copies nor the mid tier
  // run; their scans and empty launches were ~0.35 ms of every C4 step)
  if (use_runs && counts[1] > 0) {
    // the workgroup tiers' buckets: copied out of the runs into AoS rows + row indices
    MatArgs MA_;
    MA_.runs_child_max = runs_child_max;
    MA_.kr = krows;
    MA_.nr = nrows;
    MA_.mr = mrows;
    MA_.kp = kperm;
    MA_.np = nperm;
    MA_.mp = mperm;
    uint32_t* mw = (uint32_t*)ws_get(ctx, WS_MAT, (8 * nb + 4) * sizeof(uint32_t) + 64, &st);
    if (!mw) return st;
    MA_.cnt = mw;
    MA_.base = mw + 3 * nb;
    MA_.chunks = mw + 6 * nb;
    MA_.chunk0 = mw + 7 * nb;
    uint64_t* d_nchunks = (uint64_t*)(((uintptr_t)(mw + 8 * nb) + 15) & ~(uintptr_t)15);
    MA_.n_chunks = d_nchunks;
    MA_.nb = (uint32_t)nb;
    mat_count_kernel<<<(uint32_t)std::min<uint64_t>((nb + 255) / 256, 4096), 256, 0, s>>>(WA, MA_, d_big_list,
                                                                                          d_big_count);
    CDB_TRY(launch_check(ctx, s, "mat_count_kernel"));
    for (int f = 0; f < 3; ++f)
      CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, MA_.cnt + f * nb, nb, MA_.base + f * nb, (uint32_t*)nullptr,
                                                 nullptr, s));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, MA_.chunks, nb, MA_.chunk0, (uint32_t*)nullptr, d_nchunks, s));
    mat_copy_kernel<<<4096, 256, 0, s>>>(WA, MA_, d_big_list);
    CDB_TRY(launch_check(ctx, s, "mat_copy_kernel"));
  }
  if (mid_wide) {
    CDB_TRY(over_capacity(ctx, A, d_big_list, counts[1], s, use_runs ? &RV : nullptr, runs_child_max, std::max(N, M)));
  } else if (counts[1] > 0) {
    bucket_mid_kernel<<<std::min<uint64_t>(nb, 2048), kBktThreads, 0, s>>>(A, d_big_list, d_big_count);
    CDB_TRY(launch_check(ctx, s, "bucket_mid_kernel"));
  }
  CDB_HIP(hipEventRecord(ctx->ev_bucket, s), "event");
  if (!mid_wide && counts[1] > 0) {  // the mid tier forwards buckets over its capacity
    CDB_HIP(hipMemcpyAsync(counts, d_hot_count, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "d2h");
    CDB_HIP(hipStreamSynchronize(s), "sync");
  }
  const uint32_t hot = mid_wide ? 0 : counts[0];
  // (sorted-run input: the forwarded buckets' rows were copied in run order -- their child lists
  // can be merged, and the small ones take the per-bucket LDS path)
  if (hot) CDB_TRY(over_capacity(ctx, A, d_hot_list, hot, s, use_runs ? &RV : nullptr, 0, std::max(N, M)));

  // ---- 5. dense compaction into the caller's output columns (already done range by range when
  //         the bucket phase was pipelined and no workgroup tier added outputs)
  const bool recompact = !pipelined || counts[1] > 0;
  if (pipelined) {
    CDB_HIP(hipEventRecord(ctx->ev_cdone, cs), "event");
    CDB_HIP(hipStreamWaitEvent(s, ctx->ev_cdone, 0), "wait");
  }
  if (recompact) {  // the three families' dense bases side by side (each scan is a few small launches)
    hipStream_t sn = ctx->side, sm = ctx->side2;
    CDB_HIP(hipEventRecord(ctx->ev_pfork, s), "event");
    CDB_HIP(hipStreamWaitEvent(sn, ctx->ev_pfork, 0), "wait");
    CDB_HIP(hipStreamWaitEvent(sm, ctx->ev_pfork, 0), "wait");
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, dk.out, nb, dk.doff, (uint32_t*)nullptr, d_totals + 0, s, WS_SCAN));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, dnd.out, nb, dnd.doff, (uint32_t*)nullptr, d_totals + 1, sn,
                                               WS_SCAN2));
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, dm.out, nb, dm.doff, (uint32_t*)nullptr, d_totals + 2, sm,
                                               WS_SCAN3));
    CDB_HIP(hipEventRecord(ctx->ev_pn, sn), "event");
    CDB_HIP(hipEventRecord(ctx->ev_pm, sm), "event");
    CDB_HIP(hipStreamWaitEvent(s, ctx->ev_pn, 0), "wait");
    CDB_HIP(hipStreamWaitEvent(s, ctx->ev_pm, 0), "wait");
  }
  if (recompact && dense_out) {
    // one wave per 4096 output rows of a family (the kernel strides over any excess)
    const uint64_t tasks = (K + N + M) / kCompactChunk + 3;
    compact_kernel<<<(uint32_t)std::min<uint64_t>((tasks + kCompactWaves - 1) / kCompactWaves, 65536),
                     64 * kCompactWaves, 0, s>>>(C, (uint32_t)nb);
    CDB_TRY(launch_check(ctx, s, "compact_kernel"));
  } else if (!recompact) {  // the pipelined ranges compacted everything: their totals
    CDB_HIP(hipMemcpyAsync(d_totals, d_pipe + 3 * P, 3 * sizeof(uint64_t), hipMemcpyDeviceToDevice, s), "d2d");
    CDB_HIP(hipMemcpyAsync(d_cerr, d_cerr_p, sizeof(uint32_t), hipMemcpyDeviceToDevice, s), "d2d");
  }
  stats_reduce_kernel<<<1, 64, 0, s>>>(d_shards, d_stats);
  CDB_TRY(launch_check(ctx, s, "stats_reduce_kernel"));
  CDB_HIP(hipEventRecord(ctx->ev1, s), "event");
  merge_end_marker<<<1, 1, 0, s>>>();

  uint64_t totals[3];
  unsigned long long hs[ST_COUNT];
  CDB_HIP(hipMemcpyAsync(totals, d_totals, sizeof totals, hipMemcpyDeviceToHost, s), "d2h");
  CDB_HIP(hipMemcpyAsync(hs, d_stats, sizeof hs, hipMemcpyDeviceToHost, s), "d2h");
  uint32_t cerr = 0;
  CDB_HIP(hipMemcpyAsync(&cerr, d_cerr, sizeof cerr, hipMemcpyDeviceToHost, s), "d2h");
  CDB_HIP(hipStreamSynchronize(s), "sync");
  if (cerr) return fail(ctx, CDB_DEVICE_ERROR, "compaction: a source or destination row fell outside the family's rows");
  if (!dense_out) {  // the bucket layout: the rows stay in their slots, the directory says where
    const Dir* dd[3] = {&dk, &dnd, &dm};
    cdb_dev_rows* fam[3] = {&out->keys, &out->nodes, &out->members};
    uint64_t* base[3] = {ksp[0], nsp[0], msp[0]};
    for (int f = 0; f < 3; ++f) {
      std::memset(fam[f], 0, sizeof *fam[f]);
      const int w = f == 0 ? kKeyOutCols : kChildStride;
      for (int c = 0; c < w; ++c) fam[f]->col[c] = base[f] + c;
      fam[f]->stride = fam[f]->stride0 = (uint32_t)w;
      out->buckets.first[f] = dd[f]->base;
      out->buckets.count[f] = dd[f]->out;
      out->buckets.dense[f] = dd[f]->doff;
    }
    out->buckets.nb = nb;
  }
  out->keys.n = totals[0];
  out->nodes.n = totals[1];
  out->members.n = totals[2];
  if (stats) {
    std::memset(stats, 0, sizeof *stats);
    stats->key_rows_in = K;
    stats->node_rows_in = N;
    stats->member_rows_in = M;
    stats->key_rows_out = totals[0];
    stats->node_rows_out = totals[1];
    stats->member_rows_out = totals[2];
    stats->type_conflicts = hs[ST_TYPE_CONFLICTS];
    stats->dict_merges = hs[ST_DICT_MERGES];
    stats->deletes_gced = hs[ST_DELETES_GCED];
    stats->members_gced = hs[ST_MEMBERS_GCED];
    stats->duplicate_rows = hs[ST_DUP_ROWS];
    stats->orphan_children = hs[ST_ORPHANS];
    stats->hot_buckets = hot;
    stats->wide_buckets = hs[ST_WIDE];
    stats->mid_buckets = counts[1];
    float ms = 0;
    hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    stats->device_ms = ms;
    hipEventElapsedTime(&ms, ctx->ev0, ctx->ev_part);
    stats->partition_ms = ms;
    hipEventElapsedTime(&ms, ctx->ev_part, ctx->ev_bucket);
    stats->bucket_ms = ms;
    hipEventElapsedTime(&ms, ctx->ev_bucket, ctx->ev1);
    stats->finish_ms = ms;
    stats->sorted_runs = use_runs ? 1 : 0;
    stats->hot_slow_runs = hs[ST_HOT_SLOW];
    stats->hot_merged_children = hs[ST_HOT_MERGED];
    stats->wave_pipe_buckets = hs[ST_PIPE];
    stats->wave_pipe_units = hs[ST_PIPE_UNITS];
  }
  if ((flags & CDB_MERGE_STRICT_DICT_PANIC) && hs[ST_DICT_MERGES])
    return fail(ctx, CDB_DICT_MERGE_UNIMPLEMENTED, "Dict::merge reached (lwwhash.rs:180 unimplemented!())");
  return CDB_OK;
}

}  // namespace cdb

using namespace cdb;

extern "C" {

cdb_status cdb_ctx_create(cdb_ctx** out, int device) {
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return CDB_NO_DEVICE;
  cdb_ctx* ctx = new cdb_ctx();
  ctx->device = device;
  cdb_status st = hip_check(ctx, hipSetDevice(device), "hipSetDevice");
  if (st == CDB_OK) st = hip_check(ctx, hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking), "stream");
  if (st == CDB_OK) st = hip_check(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking), "stream");
  if (st == CDB_OK) st = hip_check(ctx, hipStreamCreateWithFlags(&ctx->side2, hipStreamNonBlocking), "stream");
  for (hipEvent_t* e : {&ctx->ev_pfork, &ctx->ev_pn, &ctx->ev_pm, &ctx->ev_cs, &ctx->ev_cw, &ctx->ev_cdone})
    if (st == CDB_OK) st = hip_check(ctx, hipEventCreateWithFlags(e, hipEventDisableTiming), "event");
  if (st == CDB_OK) st = hip_check(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming), "event");
  if (st == CDB_OK) st = hip_check(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming), "event");
  if (st == CDB_OK) st = hip_check(ctx, hipEventCreate(&ctx->ev0), "event");
  if (st == CDB_OK) st = hip_check(ctx, hipEventCreate(&ctx->ev1), "event");
  if (st == CDB_OK) st = hip_check(ctx, hipEventCreate(&ctx->ev_part), "event");
  if (st == CDB_OK) st = hip_check(ctx, hipEventCreate(&ctx->ev_bucket), "event");
  if (st != CDB_OK) {
    cdb_ctx_destroy(ctx);
    return st;
  }
  *out = ctx;
  return CDB_OK;
}

void cdb_ctx_destroy(cdb_ctx* ctx) {
  if (!ctx) return;
  if (ctx->node) node_destroy(ctx->node);
  for (cdb_ctx* sh : ctx->shards) cdb_ctx_destroy(sh);
  hipSetDevice(ctx->device);
  for (auto& b : ctx->ws)
    if (b.p) hipFree(b.p);
  if (ctx->ev0) hipEventDestroy(ctx->ev0);
  if (ctx->ev1) hipEventDestroy(ctx->ev1);
  if (ctx->ev_part) hipEventDestroy(ctx->ev_part);
  if (ctx->ev_bucket) hipEventDestroy(ctx->ev_bucket);
  if (ctx->ev_fork) hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) hipEventDestroy(ctx->ev_join);
  for (hipEvent_t e : {ctx->ev_pfork, ctx->ev_pn, ctx->ev_pm, ctx->ev_cs, ctx->ev_cw, ctx->ev_cdone})
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : ctx->pin_ev)
    if (e) hipEventDestroy(e);
  if (ctx->pin) hipHostFree(ctx->pin);
  for (hipStream_t k : ctx->idx_streams)
    if (k) hipStreamDestroy(k);
  if (ctx->dec_pin) hipHostFree(ctx->dec_pin);
  if (ctx->side) hipStreamDestroy(ctx->side);
  if (ctx->side2) hipStreamDestroy(ctx->side2);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* cdb_last_error(const cdb_ctx* ctx) {
  if (ctx) return ctx->last_error.c_str();
  std::lock_guard<std::mutex> g(g_create_mu);
  return g_create_error.c_str();
}

cdb_status cdb_dev_rows_alloc(cdb_ctx* ctx, cdb_dev_rows* r, uint64_t rows, int ncols) {
  std::memset(r, 0, sizeof *r);
  if (ncols < 1 || ncols > 8) return fail(ctx, CDB_BAD_ARGUMENT, "ncols");
  hipSetDevice(ctx->device);
  const uint64_t n = std::max<uint64_t>(rows, 1);
  uint64_t* p = nullptr;
  // (+16 B: readable up to the 16-B boundary after the last row, cdb_merge.h)
  cdb_status st = hip_check(ctx, hipMalloc(&p, ncols * n * sizeof(uint64_t) + 16), "hipMalloc(rows)");
  if (st != CDB_OK) return st;
  for (int c = 0; c < ncols; ++c) r->col[c] = p + c * n;
  r->n = rows;
  return CDB_OK;
}

cdb_status cdb_dev_rows_alloc_records(cdb_ctx* ctx, cdb_dev_rows* r, uint64_t rows, int ncols) {
  std::memset(r, 0, sizeof *r);
  if (ncols != kKeyCols && ncols != kNodeCols) return fail(ctx, CDB_BAD_ARGUMENT, "records layout: ncols 6 or 7");
  hipSetDevice(ctx->device);
  const uint64_t n = std::max<uint64_t>(rows, 1);
  const uint64_t hash_words = (n + 1) & ~1ull;  // records start 16-B aligned
  uint64_t* p = nullptr;
  cdb_status st =
      hip_check(ctx, hipMalloc(&p, (hash_words + (uint64_t)(ncols - 1) * n) * sizeof(uint64_t) + 16), "hipMalloc(rows)");
  if (st != CDB_OK) return st;
  r->col[0] = p;
  for (int c = 1; c < ncols; ++c) r->col[c] = p + hash_words + (c - 1);
  r->n = rows;
  r->stride = (uint32_t)(ncols - 1);
  return CDB_OK;
}

void cdb_dev_rows_release(cdb_ctx* ctx, cdb_dev_rows* r) {
  if (ctx) hipSetDevice(ctx->device);
  if (r && r->col[0]) hipFree(r->col[0]);
  if (r) std::memset(r, 0, sizeof *r);
}

cdb_status cdb_partition_owner(cdb_ctx* ctx, const cdb_dev_rows* in, int ncols, int owner_bits, cdb_dev_rows* out,
                               uint64_t* counts, void* stream) {
  if (!ctx || !in || !out || !counts || owner_bits < 0 || owner_bits > 9 || (ncols != 6 && ncols != 7 && ncols != 8))
    return CDB_BAD_ARGUMENT;
  if (in->n >= (1ull << 32)) return fail(ctx, CDB_BAD_ARGUMENT, "row count must be < 2^32");
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const uint64_t n = in->n, nb = 1ull << owner_bits;
  cdb_status st = CDB_OK;
  uint32_t* dir = (uint32_t*)ws_get(ctx, WS_OWNER, 3 * (nb + 1) * sizeof(uint32_t) + 64, &st);
  if (!dir) return st;
  uint32_t *hist = dir, *base = dir + nb + 1, *cursor = dir + 2 * (nb + 1);
  CDB_HIP(hipMemsetAsync(hist, 0, nb * sizeof(uint32_t), s), "memset");
  const uint64_t tiles = std::max<uint64_t>(1, (n + kPartTile - 1) / kPartTile);
  if (n) {
    part_hist_kernel<<<tiles, kPartThreads, 0, s>>>(in->col[0], n, 1, (uint32_t)nb, 0, hist);
    CDB_TRY(exclusive_scan<uint32_t, uint32_t>(ctx, hist, nb, base, cursor, nullptr, s));
    if (ncols == 6) {
      ColSet<6> ci, co;
      for (int c = 0; c < 6; ++c) {
        ci.c[c] = in->col[c];
        ci.s[c] = c ? std::max<uint32_t>(in->stride, 1) : 1;
        co.c[c] = out->col[c];
        co.s[c] = c ? std::max<uint32_t>(out->stride, 1) : 1;
      }
      part_scatter_kernel<6><<<tiles, kPartThreads, 0, s>>>(ci, co, n, 1, (uint32_t)nb, 0, cursor);
    } else if (ncols == 7) {
      ColSet<7> ci, co;
      for (int c = 0; c < 7; ++c) {
        ci.c[c] = in->col[c];
        ci.s[c] = c ? std::max<uint32_t>(in->stride, 1) : 1;
        co.c[c] = out->col[c];
        co.s[c] = c ? std::max<uint32_t>(out->stride, 1) : 1;
      }
      part_scatter_kernel<7><<<tiles, kPartThreads, 0, s>>>(ci, co, n, 1, (uint32_t)nb, 0, cursor);
    } else {
      ColSet<8> ci, co;
      for (int c = 0; c < 8; ++c) {
        ci.c[c] = in->col[c];
        ci.s[c] = c ? std::max<uint32_t>(in->stride, 1) : 1;
        co.c[c] = out->col[c];
        co.s[c] = c ? std::max<uint32_t>(out->stride, 1) : 1;
      }
      part_scatter_kernel<8><<<tiles, kPartThreads, 0, s>>>(ci, co, n, 1, (uint32_t)nb, 0, cursor);
    }
    CDB_TRY(launch_check(ctx, s, "partition_owner"));
  }
  std::vector<uint32_t> h(nb, 0);
  CDB_HIP(hipMemcpyAsync(h.data(), hist, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "d2h");
  CDB_HIP(hipStreamSynchronize(s), "sync");
  for (uint64_t i = 0; i < nb; ++i) counts[i] = n ? h[i] : 0;
  out->n = n;
  return CDB_OK;
}

cdb_status cdb_dev_state_rows(cdb_ctx* ctx, const cdb_dev_output* state, cdb_dev_rows* keys, cdb_dev_rows* nodes,
                              cdb_dev_rows* members, void* stream) {
  if (!ctx || !state || !keys || !nodes || !members) return CDB_BAD_ARGUMENT;
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const cdb_dev_rows* src[3] = {&state->keys, &state->nodes, &state->members};
  cdb_dev_rows* dst[3] = {keys, nodes, members};
  const int ncols[3] = {kKeyCols, kNodeCols, kMemberCols};
  uint32_t ds[3];
  for (int f = 0; f < 3; ++f) {
    ds[f] = std::max<uint32_t>(dst[f]->stride, 1);
    if (dst[f]->stride0 > 1 || (ds[f] > 1 && ds[f] != (uint32_t)(ncols[f] - 1)))
      return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_state_rows: destination rows must be columns or records");
    for (int c = 0; c < ncols[f]; ++c)
      if (src[f]->n && !dst[f]->col[c]) return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_state_rows: missing column");
  }
  if (state->compact) {
    for (int f = 0; f < 3; ++f) {
      const uint64_t n = src[f]->n;
      if (n == 0) continue;
      const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
      if (f == 0) state_dense_kernel<0><<<blocks, 256, 0, s>>>(*src[f], *dst[f], ds[f]);
      else state_dense_kernel<1><<<blocks, 256, 0, s>>>(*src[f], *dst[f], ds[f]);
      CDB_TRY(launch_check(ctx, s, "state_dense_kernel"));
    }
  } else {
    const cdb_dev_buckets& B = state->buckets;
    if (B.nb == 0 || B.nb >= (1ull << 32)) return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_state_rows: no bucket directory");
    cdb_status st = CDB_OK;
    uint8_t* w = (uint8_t*)ws_get(ctx, WS_STATE, 64, &st);
    if (!w) return st;
    CDB_HIP(hipMemsetAsync(w, 0, 64, s), "memset");
    CompactArgs C;
    std::memset(&C, 0, sizeof C);
    C.ks = src[0]->col[0];
    C.ns = src[1]->col[0];
    C.ms = src[2]->col[0];
    for (int c = 0; c < kKeyCols; ++c) C.kd[c] = keys->col[c];
    for (int c = 0; c < kNodeCols; ++c) {
      C.nd[c] = nodes->col[c];
      C.md[c] = members->col[c];
    }
    C.kbase = B.first[0]; C.nbase = B.first[1]; C.mbase = B.first[2];
    C.kout = B.count[0]; C.nout = B.count[1]; C.mout = B.count[2];
    C.kdoff = B.dense[0]; C.ndoff = B.dense[1]; C.mdoff = B.dense[2];
    C.base_tot = (const unsigned long long*)w;  // zero bases
    for (int f = 0; f < 3; ++f) C.cap[f] = std::max<uint64_t>(src[f]->n, 1) + (uint64_t)UINT32_MAX;  // slots: ours
    C.err = (uint32_t*)(w + 32);
    C.state = 1;
    for (int f = 0; f < 3; ++f) C.ds[f] = ds[f];
    const uint64_t tasks = (src[0]->n + src[1]->n + src[2]->n) / kCompactChunk + 3;
    compact_kernel<<<(uint32_t)std::min<uint64_t>((tasks + kCompactWaves - 1) / kCompactWaves, 65536),
                     64 * kCompactWaves, 0, s>>>(C, (uint32_t)B.nb);
    CDB_TRY(launch_check(ctx, s, "compact_kernel(state)"));
  }
  for (int f = 0; f < 3; ++f) dst[f]->n = src[f]->n;
  return hip_check(ctx, hipStreamSynchronize(s), "cdb_dev_state_rows");
}

namespace {
// Appends rows of one family (any input layout) behind `at` rows of dst (any input layout), the
// meta word's fold position raised by dpos.
struct AppendArgs {
  const uint64_t* src[8];
  uint64_t* dst[8];
  uint32_t ss, ds;  // record strides (1: columns)
  int ncols;
  uint64_t n, at;
  uint32_t dpos;
};
__global__ void append_rows_kernel(AppendArgs a) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t d = a.at + i;
    for (int c = 0; c < a.ncols; ++c) {
      uint64_t v = row_field(a.src, a.ss, c, i);
      if (c == a.ncols - 1) v = meta_pack(meta_tag(v), meta_pos(v) + a.dpos, meta_src(v));
      a.dst[c][c ? d * a.ds : d] = v;
    }
  }
}
}  // namespace

cdb_status cdb_dev_input_append(cdb_ctx* ctx, cdb_dev_input* dst, const cdb_dev_input* src, uint32_t pos_offset,
                                void* stream) {
  if (!ctx || !dst || !src) return CDB_BAD_ARGUMENT;
  if (src->n_pos + pos_offset > (uint32_t)kMaxPos) return fail(ctx, CDB_BAD_ARGUMENT, "at most 63 fold positions");
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  cdb_dev_rows* D[3] = {&dst->keys, &dst->nodes, &dst->members};
  const cdb_dev_rows* S[3] = {&src->keys, &src->nodes, &src->members};
  const int ncols[3] = {kKeyCols, kNodeCols, kMemberCols};
  const bool runs = dst->n_runs > 0 && src->n_runs > 0 && dst->n_runs + src->n_runs <= CDB_MAX_RUNS;
  uint64_t at[3];
  for (int f = 0; f < 3; ++f) {
    const uint32_t ds = std::max<uint32_t>(D[f]->stride, 1), ss = std::max<uint32_t>(S[f]->stride, 1);
    if (D[f]->stride0 > 1 || S[f]->stride0 > 1 || (ds > 1 && ds != (uint32_t)(ncols[f] - 1)) ||
        (ss > 1 && ss != (uint32_t)(ncols[f] - 1)))
      return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_input_append: rows must be columns or records");
    at[f] = D[f]->n;
    if (!S[f]->n) continue;
    AppendArgs a;
    std::memset(&a, 0, sizeof a);
    for (int c = 0; c < ncols[f]; ++c) {
      a.src[c] = S[f]->col[c];
      a.dst[c] = D[f]->col[c];
      if (!a.src[c] || !a.dst[c]) return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_input_append: missing column");
    }
    a.ss = ss;
    a.ds = ds;
    a.ncols = ncols[f];
    a.n = S[f]->n;
    a.at = at[f];
    a.dpos = pos_offset;
    append_rows_kernel<<<(uint32_t)std::min<uint64_t>((a.n + 255) / 256, 8192), 256, 0, s>>>(a);
    CDB_TRY(launch_check(ctx, s, "append_rows_kernel"));
    D[f]->n += S[f]->n;
  }
  if (runs) {
    for (int f = 0; f < 3; ++f)
      for (uint32_t r = 0; r <= src->n_runs; ++r) dst->run_start[f][dst->n_runs + r] = at[f] + src->run_start[f][r];
    dst->n_runs += src->n_runs;
  } else {
    dst->n_runs = 0;
  }
  dst->n_pos = std::max(dst->n_pos, src->n_pos + pos_offset);
  return hip_check(ctx, hipStreamSynchronize(s), "cdb_dev_input_append");
}

cdb_status cdb_dev_output_compact(cdb_ctx* ctx, const cdb_dev_output* src, cdb_dev_output* dst, void* stream) {
  if (!ctx || !src || !dst) return CDB_BAD_ARGUMENT;
  if (src->compact) return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_output_compact: the source is already dense");
  const cdb_dev_buckets& B = src->buckets;
  if (B.nb == 0 || B.nb >= (1ull << 32)) return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_output_compact: no bucket directory");
  const cdb_dev_rows* from[3] = {&src->keys, &src->nodes, &src->members};
  cdb_dev_rows* to[3] = {&dst->keys, &dst->nodes, &dst->members};
  for (int f = 0; f < 3; ++f)
    for (int c = 0; c < (f == 0 ? kKeyOutCols : kChildStride); ++c)
      if (from[f]->n && !to[f]->col[c]) return fail(ctx, CDB_BAD_ARGUMENT, "cdb_dev_output_compact: missing column");
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  cdb_status st = CDB_OK;
  uint8_t* w = (uint8_t*)ws_get(ctx, WS_STATE, 64, &st);
  if (!w) return st;
  CDB_HIP(hipMemsetAsync(w, 0, 64, s), "memset");
  CompactArgs C;
  std::memset(&C, 0, sizeof C);
  C.ks = from[0]->col[0];
  C.ns = from[1]->col[0];
  C.ms = from[2]->col[0];
  for (int c = 0; c < kKeyOutCols; ++c) C.kd[c] = dst->keys.col[c];
  for (int c = 0; c < kNodeCols; ++c) {
    C.nd[c] = dst->nodes.col[c];
    C.md[c] = dst->members.col[c];
  }
  C.kbase = B.first[0]; C.nbase = B.first[1]; C.mbase = B.first[2];
  C.kout = B.count[0]; C.nout = B.count[1]; C.mout = B.count[2];
  C.kdoff = B.dense[0]; C.ndoff = B.dense[1]; C.mdoff = B.dense[2];
  C.base_tot = (const unsigned long long*)w;
  for (int f = 0; f < 3; ++f) C.cap[f] = std::max<uint64_t>(from[f]->n, 1) + (uint64_t)UINT32_MAX;
  C.err = (uint32_t*)(w + 32);
  C.ds[0] = C.ds[1] = C.ds[2] = 1;
  const uint64_t tasks = (from[0]->n + from[1]->n + from[2]->n) / kCompactChunk + 3;
  compact_kernel<<<(uint32_t)std::min<uint64_t>((tasks + kCompactWaves - 1) / kCompactWaves, 65536),
                   64 * kCompactWaves, 0, s>>>(C, (uint32_t)B.nb);
  CDB_TRY(launch_check(ctx, s, "compact_kernel"));
  for (int f = 0; f < 3; ++f) {
    to[f]->n = from[f]->n;
    to[f]->stride = to[f]->stride0 = 0;
  }
  dst->compact = 1;
  return hip_check(ctx, hipStreamSynchronize(s), "cdb_dev_output_compact");
}

cdb_status cdb_merge_device(cdb_ctx* ctx, const cdb_dev_input* in, const cdb_merge_opts* opts, cdb_dev_output* out,
                            cdb_merge_stats* stats, void* stream) {
  if (!ctx || !in || !out) return CDB_BAD_ARGUMENT;
  hipSetDevice(ctx->device);
  return merge_device_impl(ctx, in, opts, out, stats, stream ? (hipStream_t)stream : ctx->stream);
}

}  // extern "C"
