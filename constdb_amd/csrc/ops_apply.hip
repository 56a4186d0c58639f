// Op-stream apply on the device: the write commands of a replicate stream
// (replica/pull.rs:184-235; handlers in cmd.rs, type_counter.rs, type_set.rs, type_hash.rs),
// decoded into op rows by ops.cpp, applied to a merged DB state in one batched call.
//
// The reference runs the commands one at a time on its main task. Every effect is per key
// (the DB object, its expires/deletes entries) or per (key, child) (a counter node, a set or
// dict member), so the batch regroups the work:
//   1. key events = the state's key rows followed by the op rows, stably sorted by key
//      (LSD radix sort, 8-bit digits, wave-match ranks): each key's events end up contiguous,
//      state first, then its ops in stream order;
//   2. one thread per key replays the handlers' key-level logic in stream order (DB::query's
//      expire side effect, Object::new on first touch, the type check, updated_at and the
//      time maxima) and records per op: applied?, the delete time an SADD/HSET saw, and the
//      latest later DELSET/DELDICT;
//   3. counter nodes and set/dict members (state children + op arguments) are stably sorted by
//      (key, node | member); one thread per (key, child) folds Counter::change in order, or
//      takes the LWW argmax over (time, stream order) of the member's tag operations
//      (lwwhash.rs:87-128: every set/rem is accepted iff its time >= the current tag time);
//   4. dense compaction of keys, nodes and members into the merge-result layout.
// Integer and ordering work only; HBM-bound sort passes dominate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "common.h"
#include "engine.h"
#include "ops.h"

namespace cdb {
namespace {

constexpr int kThreads = 256;
constexpr int kSortItems = 8;
constexpr int kSortTile = kThreads * kSortItems;  // 2048 keys per sort tile
constexpr uint32_t kNone = 0xFFFFFFFFu;

#define OPS_TRY(...)               \
  do {                             \
    cdb_status _s = (__VA_ARGS__); \
    if (_s != CDB_OK) return _s;   \
  } while (0)

inline uint32_t grid_for(uint64_t n, uint32_t per = kThreads) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, 65535ull * 4));
}

// ------------------------------------------------------------------------ radix sort
// Global digit histograms of all 8 byte positions (one read): passes whose digit is the same
// for every key are skipped by the host.
__global__ void __launch_bounds__(kThreads) rs_hist8_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                            uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[8][256];
  for (int i = threadIdx.x; i < 8 * 256; i += kThreads) (&h[0][0])[i] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads) {
    const uint64_t k = keys[i];
#pragma unroll
    for (int p = 0; p < 8; ++p) atomicAdd(&h[p][(k >> (8 * p)) & 255], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 8 * 256; i += kThreads) {
    const uint32_t v = (&h[0][0])[i];
    if (v) atomicAdd(&hist[i], v);
  }
}

// Per-tile histogram of one digit, digit-major: th[d * tiles + tile].
__global__ void __launch_bounds__(kThreads) rs_tile_hist_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                                int shift, uint32_t tiles, uint32_t* __restrict__ th) {
  __shared__ uint32_t h[256];
  const uint32_t tile = blockIdx.x;
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)tile * kSortTile;
#pragma unroll
  for (int r = 0; r < kSortItems; ++r) {
    const uint64_t i = base + r * kThreads + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255], 1u);
  }
  __syncthreads();
  th[(uint64_t)threadIdx.x * tiles + tile] = h[threadIdx.x];
}

// Stable scatter of one digit. Items are taken in index order, 256 per round: a lane's rank
// is the count of earlier equal digits in its wave (8 ballots give the match mask), plus the
// earlier waves' counts of that digit this round, plus the tile's running count.
__global__ void __launch_bounds__(kThreads) rs_scatter_kernel(const uint64_t* __restrict__ kin,
                                                              const uint32_t* __restrict__ vin, uint64_t n, int shift,
                                                              uint32_t tiles, const uint32_t* __restrict__ off,
                                                              uint64_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  __shared__ uint32_t run[256];
  __shared__ uint32_t wcnt[kThreads / 64][256];
  const uint32_t tile = blockIdx.x;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  run[t] = off[(uint64_t)t * tiles + tile];
  for (int k = 0; k < kThreads / 64; ++k) wcnt[k][t] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)tile * kSortTile;
  const unsigned long long lt = (1ull << lane) - 1;
  for (int r = 0; r < kSortItems; ++r) {
    const uint64_t i = base + r * kThreads + t;
    const bool valid = i < n;
    const uint64_t k = valid ? kin[i] : 0;
    const uint32_t v = valid ? vin[i] : 0;
    const uint32_t d = (uint32_t)(k >> shift) & 255;
    unsigned long long m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1;
      const unsigned long long bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    if (valid && (63 - __clzll(m)) == lane) wcnt[w][d] = __popcll(m);
    __syncthreads();
    if (valid) {
      uint32_t pos = run[d] + __popcll(m & lt);
      for (int k2 = 0; k2 < w; ++k2) pos += wcnt[k2][d];
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    uint32_t s = 0;
    for (int k2 = 0; k2 < kThreads / 64; ++k2) {
      s += wcnt[k2][t];
      wcnt[k2][t] = 0;
    }
    run[t] += s;
    __syncthreads();
  }
}

// ------------------------------------------------------------------------ scan (u32)
constexpr int kScanTile = kThreads * 8;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* total) {
  __shared__ uint32_t ws[kThreads / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
  for (int k = 0; k < kThreads / 64; ++k) {
    if (k < w) pre += ws[k];
    tot += ws[k];
  }
  __syncthreads();
  *total = tot;
  return pre + inc - x;
}

__global__ void __launch_bounds__(kThreads) scan_reduce_kernel(const uint32_t* __restrict__ in, uint64_t n,
                                                               uint32_t* __restrict__ sums) {
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint32_t s = 0;
  for (int r = 0; r < 8; ++r) {
    const uint64_t i = base + r * kThreads + threadIdx.x;
    if (i < n) s += in[i];
  }
  uint32_t tot;
  block_excl_scan(s, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kThreads) scan_sums_kernel(uint32_t* __restrict__ sums, uint32_t nb,
                                                             uint32_t* __restrict__ total) {
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += kThreads) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t x = i < nb ? sums[i] : 0;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(x, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ void __launch_bounds__(kThreads) scan_apply_kernel(const uint32_t* __restrict__ in, uint64_t n,
                                                              const uint32_t* __restrict__ sums,
                                                              uint32_t* __restrict__ out) {
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  // each thread owns 8 consecutive items
  uint32_t x[8], s = 0;
  for (int r = 0; r < 8; ++r) {
    const uint64_t i = base + threadIdx.x * 8 + r;
    x[r] = i < n ? in[i] : 0;
    s += x[r];
  }
  uint32_t tot;
  uint32_t pre = block_excl_scan(s, &tot) + sums[blockIdx.x];
  for (int r = 0; r < 8; ++r) {
    const uint64_t i = base + threadIdx.x * 8 + r;
    if (i < n) out[i] = pre;
    pre += x[r];
  }
}

// ------------------------------------------------------------------------ device state
struct Dev {
  std::vector<void*> bufs;
  cdb_ctx* ctx;
  ~Dev() {
    for (void* p : bufs) hipFree(p);
  }
  template <typename T>
  cdb_status alloc(T** p, uint64_t n) {
    void* q = nullptr;
    OPS_TRY(hip_check(ctx, hipMalloc(&q, std::max<uint64_t>(n, 1) * sizeof(T)), "hipMalloc(ops)"));
    bufs.push_back(q);
    *p = (T*)q;
    return CDB_OK;
  }
};

struct Scratch {  // sort + scan scratch, sized for the largest family
  uint64_t *ka, *kb;
  uint32_t *va, *vb, *th, *hist8, *sums, *total;
  uint64_t cap;
};

cdb_status excl_scan(cdb_ctx* ctx, Scratch& S, const uint32_t* in, uint64_t n, uint32_t* out, uint32_t* host_total,
                     hipStream_t s) {
  const uint32_t tiles = (uint32_t)std::max<uint64_t>(1, (n + kScanTile - 1) / kScanTile);
  scan_reduce_kernel<<<tiles, kThreads, 0, s>>>(in, n, S.sums);
  scan_sums_kernel<<<1, kThreads, 0, s>>>(S.sums, tiles, S.total);
  scan_apply_kernel<<<tiles, kThreads, 0, s>>>(in, n, S.sums, out);
  OPS_TRY(launch_check(ctx, s, "ops scan"));
  if (host_total) {
    OPS_TRY(hip_check(ctx, hipMemcpyAsync(host_total, S.total, 4, hipMemcpyDeviceToHost, s), "scan total"));
    OPS_TRY(hip_check(ctx, hipStreamSynchronize(s), "scan total"));
  }
  return CDB_OK;
}

// Stable sort of (S.ka[0..n), S.va[0..n)) by the low `bits` bits of the key. Result in
// (S.ka, S.va) (the buffers swap internally).
cdb_status sort_pairs(cdb_ctx* ctx, Scratch& S, uint64_t n, int bits, hipStream_t s) {
  if (n <= 1) return CDB_OK;
  const uint32_t tiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
  OPS_TRY(hip_check(ctx, hipMemsetAsync(S.hist8, 0, 8 * 256 * 4, s), "memset"));
  rs_hist8_kernel<<<grid_for(n, kThreads * 16), kThreads, 0, s>>>(S.ka, n, S.hist8);
  uint32_t h[8 * 256];
  OPS_TRY(hip_check(ctx, hipMemcpyAsync(h, S.hist8, sizeof h, hipMemcpyDeviceToHost, s), "hist8"));
  OPS_TRY(hip_check(ctx, hipStreamSynchronize(s), "hist8"));
  for (int p = 0; p * 8 < bits; ++p) {
    bool trivial = false;
    for (int d = 0; d < 256; ++d)
      if (h[p * 256 + d] == n) trivial = true;
    if (trivial) continue;
    rs_tile_hist_kernel<<<tiles, kThreads, 0, s>>>(S.ka, n, 8 * p, tiles, S.th);
    OPS_TRY(excl_scan(ctx, S, S.th, (uint64_t)tiles * 256, S.th, nullptr, s));
    rs_scatter_kernel<<<tiles, kThreads, 0, s>>>(S.ka, S.va, n, 8 * p, tiles, S.th, S.kb, S.vb);
    OPS_TRY(launch_check(ctx, s, "rs_scatter"));
    std::swap(S.ka, S.kb);
    std::swap(S.va, S.vb);
  }
  return CDB_OK;
}

// ------------------------------------------------------------------------ small kernels
__global__ void iota_gather_kernel(const uint64_t* __restrict__ a, uint64_t na, const uint64_t* __restrict__ b,
                                   uint64_t n, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    keys[i] = i < na ? a[i] : b[i - na];
    vals[i] = (uint32_t)i;
  }
}

// keys[i] = (col_a | col_b)[vals[i]] — the next (more significant) LSD key of a stable multi-key sort
__global__ void regather_kernel(const uint64_t* __restrict__ a, uint64_t na, const uint64_t* __restrict__ b,
                                const uint32_t* __restrict__ vals, uint64_t n, uint64_t* __restrict__ keys) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t e = vals[i];
    keys[i] = e < na ? a[e] : b[e - na];
  }
}
__global__ void regather32_kernel(const uint32_t* __restrict__ a, const uint32_t* __restrict__ vals, uint64_t n,
                                  uint64_t* __restrict__ keys) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    keys[i] = a[vals[i]];
}

// Segment heads over sorted items: (k1, k2, k3)[perm[i]] differs from its predecessor's.
// `bad` counts neighbours equal in k1 (and k3) but not k2 (64-bit hash collisions).
__global__ void heads_kernel(const uint32_t* __restrict__ perm, uint64_t n, const uint64_t* k1a, uint64_t na,
                             const uint64_t* k1b, const uint64_t* k2a, const uint64_t* k2b,
                             const uint32_t* __restrict__ k3, uint32_t* __restrict__ head,
                             unsigned long long* __restrict__ bad) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t e = perm[i];
    uint32_t h = 1;
    if (i > 0) {
      const uint32_t p = perm[i - 1];
      const uint64_t a1 = e < na ? k1a[e] : k1b[e - na], b1 = p < na ? k1a[p] : k1b[p - na];
      const uint64_t a2 = e < na ? k2a[e] : k2b[e - na], b2 = p < na ? k2a[p] : k2b[p - na];
      const bool s3 = !k3 || k3[e] == k3[p];
      h = !(a1 == b1 && a2 == b2 && s3);
      if (a1 == b1 && a2 != b2 && s3) atomicAdd(bad, 1ull);
    }
    head[i] = h;
  }
}

// seg_start[seg(i)] = i for heads (seg = exclusive scan of heads); seg_start[nseg] = n
__global__ void seg_start_kernel(const uint32_t* __restrict__ head, const uint32_t* __restrict__ segx, uint64_t n,
                                 uint32_t* __restrict__ seg_start) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (head[i]) seg_start[segx[i]] = (uint32_t)i;
  if (blockIdx.x == 0 && threadIdx.x == 0) seg_start[segx[n - 1] + head[n - 1]] = (uint32_t)n;
}

// ------------------------------------------------------------------------ key fold
struct KeyIn {
  // state key rows (merge-result layout): kh kf ct ut dt meta win cref
  const uint64_t *s_ct, *s_ut, *s_dt, *s_meta, *s_win;
  uint64_t Ks;
  // op rows: uuid, meta (code | pos | row)
  const uint64_t *o_uuid, *o_meta;
  uint32_t pos_ops;
};
struct KeyOut {
  uint32_t* ev_seg;     // per event: its key segment
  uint32_t* op_valid;   // per op: the handler got past its type check
  uint64_t* op_dt;      // per op: the object's delete time when an SADD/HSET ran
  uint64_t *sfx_u;      // per op: latest (time, op) DELSET/DELDICT after it, (0, kNone) if none
  uint32_t* sfx_seq;
  uint64_t* seg_sfx_u;  // per segment: the same over all of the key's ops
  uint32_t* seg_sfx_seq;
  // per segment final key state
  uint32_t* flags;      // exists | has_exp << 1 | has_del << 2 | tag << 8
  uint64_t *ct, *ut, *dt, *kmeta, *win, *exp_t, *exp_meta, *del_t, *del_meta;
  unsigned long long* stats;  // [0] type errors, [1] expired on query
};

__device__ __forceinline__ void updated_at(uint64_t& ct, uint64_t& ut, uint64_t dt, uint64_t u) {  // object.rs:35-49
  if (ut < u) ut = u;
  if (ct < dt && u >= dt) ct = u;  // created again
}

__device__ __forceinline__ uint32_t op_type(uint32_t code) {
  switch (code) {
    case OP_SET: case OP_DELBYTES: return TAG_BYTES;
    case OP_INCR: case OP_DECR: case OP_DELCNT: return TAG_COUNTER;
    case OP_SADD: case OP_SREM: case OP_DELSET: return TAG_SET;
    default: return TAG_DICT;
  }
}

__global__ void __launch_bounds__(kThreads) key_fold_kernel(KeyIn I, KeyOut O, const uint32_t* __restrict__ perm,
                                                            const uint32_t* __restrict__ seg_start, uint32_t nseg) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
    const uint32_t b = seg_start[s], e_end = seg_start[s + 1];
    bool exists = false, has_exp = false, has_del = false;
    uint32_t tag = 0;
    uint64_t ct = 0, ut = 0, dt = 0, kmeta = 0, win = 0, exp_t = 0, exp_meta = 0, del_t = 0, del_meta = 0;
    unsigned long long type_err = 0, expired = 0;
    for (uint32_t i = b; i < e_end; ++i) {
      const uint32_t e = perm[i];
      O.ev_seg[e] = s;
      if (e < I.Ks) {  // the DB state: one data row, at most one expires and one deletes row
        const uint64_t m = I.s_meta[e];
        const uint32_t T = meta_tag(m);
        if (T == TAG_EXPIRE) {
          has_exp = true, exp_t = I.s_ct[e], exp_meta = m;
        } else if (T == TAG_DELETE) {
          has_del = true, del_t = I.s_ct[e], del_meta = m;
        } else {
          exists = true, tag = T, ct = I.s_ct[e], ut = I.s_ut[e], dt = I.s_dt[e], kmeta = m, win = I.s_win[e];
        }
        continue;
      }
      const uint32_t o = e - (uint32_t)I.Ks;
      const uint32_t code = meta_tag(I.o_meta[o]);
      const uint64_t u = I.o_uuid[o];
      // DB::query (db.rs:52-66): an expired, alive object is deleted at its expire time
      if (exists && has_exp && ct >= dt && ct < exp_t && exp_t <= u) {
        dt = exp_t;
        updated_at(ct, ut, dt, exp_t);
        has_del = true, del_t = exp_t;
        del_meta = meta_pack(TAG_DELETE, meta_pos(kmeta), meta_src(kmeta));
        ++expired;
      }
      const uint32_t want = op_type(code);
      if (!exists) {  // Object::new(enc, uuid, 0) (object.rs:25-32)
        exists = true, tag = want, ct = u, ut = 0, dt = 0;
        kmeta = meta_pack(want, I.pos_ops, o);
        win = (code == OP_SET || code == OP_DELBYTES) ? meta_pack(0, I.pos_ops, o) : 0;
      }
      bool ok = tag == want;
      if (code == OP_SET) {  // cmd.rs:188-210: the update-time check comes before the type check
        if (ut > u) {
          ok = false;
        } else if (ok) {
          win = meta_pack(0, I.pos_ops, o);
          updated_at(ct, ut, dt, u);
        } else {
          ++type_err;
        }
      } else if (!ok) {
        ++type_err;
      } else {
        switch (code) {
          case OP_DELBYTES: case OP_DELCNT: case OP_DELSET: case OP_DELDICT:
            dt = max(dt, u), ut = max(ut, u);
            break;
          case OP_SADD: case OP_HSET:
            O.op_dt[o] = dt;
            updated_at(ct, ut, dt, u);
            break;
          default:  // INCR DECR SREM HDEL
            updated_at(ct, ut, dt, u);
        }
      }
      O.op_valid[o] = ok;
    }
    // DELSET/DELDICT reach every member present when they run: for each op, the latest
    // (time, op) of the key's valid delete-all ops after it.
    uint64_t bu = 0;
    uint32_t bs = kNone;
    for (uint32_t i = e_end; i-- > b;) {
      const uint32_t e = perm[i];
      if (e < I.Ks) continue;
      const uint32_t o = e - (uint32_t)I.Ks;
      O.sfx_u[o] = bu, O.sfx_seq[o] = bs;
      const uint32_t code = meta_tag(I.o_meta[o]);
      if ((code == OP_DELSET || code == OP_DELDICT) && O.op_valid[o]) {
        const uint64_t u = I.o_uuid[o];
        if (bs == kNone || u > bu) bu = u, bs = o;
      }
    }
    O.seg_sfx_u[s] = bu, O.seg_sfx_seq[s] = bs;
    O.flags[s] = (exists ? 1u : 0u) | (has_exp ? 2u : 0u) | (has_del ? 4u : 0u) | (tag << 8);
    O.ct[s] = ct, O.ut[s] = ut, O.dt[s] = dt, O.kmeta[s] = kmeta, O.win[s] = win;
    O.exp_t[s] = exp_t, O.exp_meta[s] = exp_meta, O.del_t[s] = del_t, O.del_meta[s] = del_meta;
    if (type_err) atomicAdd(&O.stats[0], type_err);
    if (expired) atomicAdd(&O.stats[1], expired);
  }
}

// State children inherit their key's segment: one thread per state key row walks its range.
__global__ void state_child_seg_kernel(const uint64_t* __restrict__ s_meta, const uint64_t* __restrict__ s_cref,
                                       uint64_t Ks, const uint32_t* __restrict__ ev_seg,
                                       uint32_t* __restrict__ nseg_of, uint32_t* __restrict__ mseg_of) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < Ks; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t T = meta_tag(s_meta[r]);
    if (T > TAG_SET) continue;
    const uint64_t cr = s_cref[r], cb = cr >> 24, cc = cr & 0xFFFFFF;
    uint32_t* dst = T == TAG_COUNTER ? nseg_of : mseg_of;
    if (T == TAG_BYTES) continue;
    const uint32_t sg = ev_seg[r];
    for (uint64_t j = cb; j < cb + cc; ++j) dst[j] = sg;
  }
}

__global__ void op_child_seg_kernel(const uint64_t* __restrict__ c_op, uint64_t n, uint64_t off,
                                    const uint32_t* __restrict__ op_seg_ev, uint64_t Ks,
                                    uint32_t* __restrict__ seg_of) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x)
    seg_of[off + j] = op_seg_ev[Ks + c_op[j]];
}

// ------------------------------------------------------------------------ child folds
struct ChildIn {
  // state children (merge-result layout): pkh pkf id1 id2 t meta
  const uint64_t *s_pkh, *s_pkf, *s_id1, *s_id2, *s_t, *s_meta;
  uint64_t Ns;
  // op children: id1 (node | member hash) id2 (delta | member fp) op
  const uint64_t *c_id1, *c_id2, *c_op;
  // op rows
  const uint64_t *o_kh, *o_kf, *o_uuid, *o_meta;
  const uint32_t *op_valid;
  const uint64_t *op_dt, *sfx_u, *seg_sfx_u;
  const uint32_t *sfx_seq, *seg_sfx_seq;
  const uint32_t* seg_of;  // per child event: key segment
  uint32_t pos_ops;
};
struct ChildOut {
  uint64_t *pkh, *pkf, *id1, *id2, *t, *meta;  // sparse: one slot per child segment
  uint32_t* produce;
  uint32_t* seg;        // key segment of the slot
};

// Counter::change (type_counter.rs:37-51) per (key, node) in stream order: the first op on an
// absent node inserts (delta, uuid); later ops add delta only if the node's time < uuid; the
// time never changes.
__global__ void __launch_bounds__(kThreads) node_fold_kernel(ChildIn I, ChildOut O, const uint32_t* __restrict__ perm,
                                                             const uint32_t* __restrict__ cs, uint32_t ncs) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ncs; g += gridDim.x * blockDim.x) {
    bool have = false;
    uint64_t v = 0, t = 0, meta = 0, pkh = 0, pkf = 0, node = 0;
    uint32_t sg = 0;
    for (uint32_t i = cs[g]; i < cs[g + 1]; ++i) {
      const uint32_t c = perm[i];
      sg = I.seg_of[c];
      if (c < I.Ns) {
        have = true, v = I.s_id2[c], t = I.s_t[c], meta = I.s_meta[c];
        pkh = I.s_pkh[c], pkf = I.s_pkf[c], node = I.s_id1[c];
        continue;
      }
      const uint32_t j = c - (uint32_t)I.Ns;
      const uint32_t o = (uint32_t)I.c_op[j];
      if (!I.op_valid[o]) continue;
      const uint64_t u = I.o_uuid[o], d = I.c_id2[j];
      if (!have) {
        have = true, v = d, t = u, meta = meta_pack(0, I.pos_ops, j);
        pkh = I.o_kh[o], pkf = I.o_kf[o], node = I.c_id1[j];
      } else if (t < u) {
        v += d;  // wrapping i64
      }
    }
    O.produce[g] = have;
    O.seg[g] = sg;
    if (have) O.pkh[g] = pkh, O.pkf[g] = pkf, O.id1[g] = node, O.id2[g] = v, O.t[g] = t, O.meta[g] = meta;
  }
}

// Set/Dict member tags per (key, member): LWWHash::set / rem (lwwhash.rs:87-128) accept an op
// iff its time >= the current tag time, so the final tag is the argmax over (time, stream
// order) of: the state tag; each applied SADD/HSET (add at uuid, then a del at the delete
// time it saw if uuid < that time, type_set.rs:34-37 / type_hash.rs:37-42); each SREM/HDEL
// (del at uuid); and the latest DELSET/DELDICT after the member first existed
// (type_set.rs:128-130 / type_hash.rs:113-115 remove every member present then).
__global__ void __launch_bounds__(kThreads) member_fold_kernel(ChildIn I, ChildOut O, const uint32_t* __restrict__ perm,
                                                               const uint32_t* __restrict__ cs, uint32_t ncs) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ncs; g += gridDim.x * blockDim.x) {
    bool present = false, any = false;
    uint64_t bt = 0, bord = 0;  // best (time, order); order = (op + 1) << 1 | sub, state = 0
    uint32_t bkind = 0;
    uint64_t bmeta = 0, src_meta = 0, pkh = 0, pkf = 0, mh = 0, mf = 0;
    uint32_t first = kNone, sg = 0;
    auto take = [&](uint64_t t, uint64_t ord, uint32_t kind, uint64_t m) {
      if (!any || t > bt || (t == bt && ord >= bord)) bt = t, bord = ord, bkind = kind, bmeta = m, any = true;
    };
    for (uint32_t i = cs[g]; i < cs[g + 1]; ++i) {
      const uint32_t c = perm[i];
      sg = I.seg_of[c];
      if (c < I.Ns) {
        present = true;
        const uint64_t m = I.s_meta[c];
        take(I.s_t[c], 0, meta_tag(m), m);
        src_meta = m, pkh = I.s_pkh[c], pkf = I.s_pkf[c], mh = I.s_id1[c], mf = I.s_id2[c];
        continue;
      }
      const uint32_t j = c - (uint32_t)I.Ns;
      const uint32_t o = (uint32_t)I.c_op[j];
      if (!I.op_valid[o]) continue;
      const uint32_t code = meta_tag(I.o_meta[o]);
      const uint64_t u = I.o_uuid[o];
      const uint64_t mj = meta_pack(0, I.pos_ops, j);
      if (first == kNone && !present) {
        first = o;
        src_meta = mj, pkh = I.o_kh[o], pkf = I.o_kf[o], mh = I.c_id1[j], mf = I.c_id2[j];
      }
      const uint64_t ord = ((uint64_t)o + 1) << 1;
      if (code == OP_SADD || code == OP_HSET) {
        take(u, ord, KIND_ADD, mj);
        const uint64_t d = I.op_dt[o];
        if (u < d) take(d, ord | 1, KIND_DEL, mj);
      } else {  // SREM / HDEL
        take(u, ord, KIND_DEL, mj);
      }
    }
    const bool produce = present || first != kNone;
    if (produce) {
      const uint64_t du = present ? I.seg_sfx_u[sg] : I.sfx_u[first];
      const uint32_t ds = present ? I.seg_sfx_seq[sg] : I.sfx_seq[first];
      if (ds != kNone) take(du, ((uint64_t)ds + 1) << 1, KIND_DEL, src_meta);
    }
    O.produce[g] = produce;
    O.seg[g] = sg;
    if (produce) {
      O.pkh[g] = pkh, O.pkf[g] = pkf, O.id1[g] = mh, O.id2[g] = mf, O.t[g] = bt;
      O.meta[g] = meta_pack(bkind, meta_pos(bmeta), meta_src(bmeta));
    }
  }
}

// Dense child rows; per key segment: first dense row, count and (counters) the wrapping sum.
__global__ void child_compact_kernel(ChildOut O, const uint32_t* __restrict__ dense, uint32_t ncs, cdb_dev_rows out,
                                     uint32_t* __restrict__ cbeg, uint32_t* __restrict__ ccnt,
                                     unsigned long long* __restrict__ csum) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ncs; g += gridDim.x * blockDim.x) {
    if (!O.produce[g]) continue;
    const uint32_t d = dense[g], sg = O.seg[g];
    out.col[0][d] = O.pkh[g], out.col[1][d] = O.pkf[g], out.col[2][d] = O.id1[g];
    out.col[3][d] = O.id2[g], out.col[4][d] = O.t[g], out.col[5][d] = O.meta[g];
    atomicMin(&cbeg[sg], d);
    atomicAdd(&ccnt[sg], 1u);
    if (csum) atomicAdd(&csum[sg], (unsigned long long)O.id2[g]);
  }
}

__global__ void key_count_kernel(const uint32_t* __restrict__ flags, uint32_t nseg, uint32_t* __restrict__ cnt) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
    const uint32_t f = flags[s];
    cnt[s] = (f & 1) + ((f >> 1) & 1) + ((f >> 2) & 1);
  }
}

struct KeyEmit {
  const uint32_t* flags;
  const uint64_t *ct, *ut, *dt, *kmeta, *win, *exp_t, *exp_meta, *del_t, *del_meta;
  const uint32_t *ncbeg, *nccnt, *mcbeg, *mccnt;
  const unsigned long long* nsum;
  const uint32_t* dense;
  const uint32_t* perm;         // sorted events -> event; seg_start gives a segment's first event
  const uint32_t* seg_start;
  const uint64_t *s_kh, *s_kf, *o_kh, *o_kf;
  uint64_t Ks;
};
__global__ void key_emit_kernel(KeyEmit E, uint32_t nseg, cdb_dev_rows out) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
    const uint32_t f = E.flags[s];
    uint32_t d = E.dense[s];
    const uint32_t e = E.perm[E.seg_start[s]];
    const uint64_t kh = e < E.Ks ? E.s_kh[e] : E.o_kh[e - E.Ks], kf = e < E.Ks ? E.s_kf[e] : E.o_kf[e - E.Ks];
    auto row = [&](uint64_t ct, uint64_t ut, uint64_t dt, uint64_t meta, uint64_t win, uint64_t cref) {
      out.col[O_KH][d] = kh, out.col[O_KF][d] = kf, out.col[O_CT][d] = ct, out.col[O_UT][d] = ut;
      out.col[O_DT][d] = dt, out.col[O_META][d] = meta, out.col[O_WIN][d] = win, out.col[O_CREF][d] = cref;
      ++d;
    };
    if (f & 1) {
      const uint32_t tag = f >> 8;
      uint64_t win = E.win[s], cref = 0;
      if (tag == TAG_COUNTER) {
        win = E.nsum[s];
        if (E.nccnt[s]) cref = cref_pack(E.ncbeg[s], E.nccnt[s]);
      } else if (tag == TAG_SET || tag == TAG_DICT) {
        win = 0;
        if (E.mccnt[s]) cref = cref_pack(E.mcbeg[s], E.mccnt[s]);
      }
      row(E.ct[s], E.ut[s], E.dt[s], E.kmeta[s], win, cref);
    }
    if (f & 2) row(E.exp_t[s], 0, 0, E.exp_meta[s], 0, 0);
    if (f & 4) row(E.del_t[s], 0, 0, E.del_meta[s], 0, 0);
  }
}

}  // namespace

// Applies `ops` (pos = pos_ops in their meta words) to the state rows. Host vectors in, host
// vectors out (the cdb_merged layout); device time of the pipeline in stats.
cdb_status apply_ops_impl(cdb_ctx* ctx, const ColVec* sk, const ColVec* sn, const ColVec* sm, const Batch& B, uint32_t pos_ops,
                          ColVec* ok, ColVec* on, ColVec* om,
                          cdb_apply_stats* stats) {
  hipStream_t s = ctx->stream;
  const uint64_t Ks = sk[O_KH].size(), Ns = sn[0].size(), Ms = sm[0].size();
  const uint64_t Ko = B.kh.size(), Nn = B.n_pkh.size(), Mm = B.m_pkh.size();
  const uint64_t E = Ks + Ko, Cn = Ns + Nn, Cm = Ms + Mm;
  if (E >= (1ull << 31) || Cn >= (1ull << 31) || Cm >= (1ull << 31))
    return fail(ctx, CDB_BAD_ARGUMENT, "op apply: row counts must be < 2^31 per family");
  Dev D{{}, ctx};
  auto up = [&](const auto& v, uint64_t** p) -> cdb_status {
    OPS_TRY(D.alloc(p, v.size()));
    if (!v.empty())
      OPS_TRY(staged_h2d(ctx, *p, v.data(), v.size() * 8, s));
    return CDB_OK;
  };
  uint64_t *sk_d[kKeyOutCols], *sn_d[kNodeCols], *sm_d[kMemberCols];
  for (int c = 0; c < kKeyOutCols; ++c) OPS_TRY(up(sk[c], &sk_d[c]));
  for (int c = 0; c < kNodeCols; ++c) OPS_TRY(up(sn[c], &sn_d[c]));
  for (int c = 0; c < kMemberCols; ++c) OPS_TRY(up(sm[c], &sm_d[c]));
  ColVec ometa(B.meta);
  for (auto& m : ometa) m = meta_pack(meta_tag(m), pos_ops, meta_src(m));
  uint64_t *o_kh, *o_kf, *o_uuid, *o_meta, *n_node, *n_v, *n_op, *m_h, *m_f, *m_op;
  OPS_TRY(up(B.kh, &o_kh));
  OPS_TRY(up(B.kf, &o_kf));
  OPS_TRY(up(B.ct, &o_uuid));
  OPS_TRY(up(ometa, &o_meta));
  OPS_TRY(up(B.n_node, &n_node));
  OPS_TRY(up(B.n_v, &n_v));
  OPS_TRY(up(B.n_t, &n_op));
  OPS_TRY(up(B.m_h, &m_h));
  OPS_TRY(up(B.m_f, &m_f));
  OPS_TRY(up(B.m_t, &m_op));

  const uint64_t cap = std::max<uint64_t>({E, Cn, Cm, 1});
  Scratch S;
  S.cap = cap;
  const uint64_t tiles_max = (cap + kSortTile - 1) / kSortTile;
  OPS_TRY(D.alloc(&S.ka, cap));
  OPS_TRY(D.alloc(&S.kb, cap));
  OPS_TRY(D.alloc(&S.va, cap));
  OPS_TRY(D.alloc(&S.vb, cap));
  OPS_TRY(D.alloc(&S.th, tiles_max * 256));
  OPS_TRY(D.alloc(&S.hist8, 8 * 256));
  OPS_TRY(D.alloc(&S.sums, (tiles_max * 256 + kScanTile - 1) / kScanTile + (cap + kScanTile - 1) / kScanTile + 1));
  OPS_TRY(D.alloc(&S.total, 1));
  unsigned long long* dstats;
  OPS_TRY(D.alloc(&dstats, 8));
  OPS_TRY(hip_check(ctx, hipMemsetAsync(dstats, 0, 64, s), "memset"));
  // per event / segment / op
  uint32_t *perm, *head, *segx, *seg_start, *ev_seg;
  OPS_TRY(D.alloc(&perm, E));
  OPS_TRY(D.alloc(&head, cap));
  OPS_TRY(D.alloc(&segx, cap));
  OPS_TRY(D.alloc(&seg_start, E + 1));
  OPS_TRY(D.alloc(&ev_seg, E));
  KeyOut KO;
  KO.ev_seg = ev_seg;
  KO.stats = dstats;
  OPS_TRY(D.alloc(&KO.op_valid, Ko));
  OPS_TRY(D.alloc(&KO.op_dt, Ko));
  OPS_TRY(D.alloc(&KO.sfx_u, Ko));
  OPS_TRY(D.alloc(&KO.sfx_seq, Ko));
  OPS_TRY(hip_check(ctx, hipMemsetAsync(KO.op_dt, 0, std::max<uint64_t>(Ko, 1) * 8, s), "memset"));

  hipEvent_t e0 = ctx->ev0, e1 = ctx->ev1;
  OPS_TRY(hip_check(ctx, hipEventRecord(e0, s), "event"));
  uint32_t nseg = 0;
  unsigned long long* dbad = dstats + 4;
  if (E) {
    // ---- 1. key events sorted by key hash (state rows first within a key: stable)
    iota_gather_kernel<<<grid_for(E), kThreads, 0, s>>>(sk_d[O_KH], Ks, o_kh, E, S.ka, S.va);
    OPS_TRY(sort_pairs(ctx, S, E, 64, s));
    heads_kernel<<<grid_for(E), kThreads, 0, s>>>(S.va, E, sk_d[O_KH], Ks, o_kh, sk_d[O_KF], o_kf, nullptr, head,
                                                   dbad);
    unsigned long long bad = 0;
    OPS_TRY(hip_check(ctx, hipMemcpyAsync(&bad, dbad, 8, hipMemcpyDeviceToHost, s), "d2h"));
    OPS_TRY(hip_check(ctx, hipStreamSynchronize(s), "sync"));
    if (bad) {  // a 64-bit key-hash collision: order by (kh, kf) exactly (kf first, then kh)
      iota_gather_kernel<<<grid_for(E), kThreads, 0, s>>>(sk_d[O_KF], Ks, o_kf, E, S.ka, S.va);
      OPS_TRY(sort_pairs(ctx, S, E, 64, s));
      regather_kernel<<<grid_for(E), kThreads, 0, s>>>(sk_d[O_KH], Ks, o_kh, S.va, E, S.ka);
      OPS_TRY(sort_pairs(ctx, S, E, 64, s));
      heads_kernel<<<grid_for(E), kThreads, 0, s>>>(S.va, E, sk_d[O_KH], Ks, o_kh, sk_d[O_KF], o_kf, nullptr, head,
                                                     dbad);
    }
    OPS_TRY(hip_check(ctx, hipMemcpyAsync(perm, S.va, E * 4, hipMemcpyDeviceToDevice, s), "d2d"));
    OPS_TRY(excl_scan(ctx, S, head, E, segx, &nseg, s));
    seg_start_kernel<<<grid_for(E), kThreads, 0, s>>>(head, segx, E, seg_start);
    OPS_TRY(launch_check(ctx, s, "ops key sort"));
  }
  // ---- 2. key fold
  const uint64_t NS = std::max<uint32_t>(nseg, 1);
  OPS_TRY(D.alloc(&KO.seg_sfx_u, NS));
  OPS_TRY(D.alloc(&KO.seg_sfx_seq, NS));
  OPS_TRY(D.alloc(&KO.flags, NS));
  OPS_TRY(D.alloc(&KO.ct, NS));
  OPS_TRY(D.alloc(&KO.ut, NS));
  OPS_TRY(D.alloc(&KO.dt, NS));
  OPS_TRY(D.alloc(&KO.kmeta, NS));
  OPS_TRY(D.alloc(&KO.win, NS));
  OPS_TRY(D.alloc(&KO.exp_t, NS));
  OPS_TRY(D.alloc(&KO.exp_meta, NS));
  OPS_TRY(D.alloc(&KO.del_t, NS));
  OPS_TRY(D.alloc(&KO.del_meta, NS));
  KeyIn KI{sk_d[O_CT], sk_d[O_UT], sk_d[O_DT], sk_d[O_META], sk_d[O_WIN], Ks, o_uuid, o_meta, pos_ops};
  if (nseg) key_fold_kernel<<<grid_for(nseg), kThreads, 0, s>>>(KI, KO, perm, seg_start, nseg);
  OPS_TRY(launch_check(ctx, s, "key_fold_kernel"));

  // ---- 3. children: counter nodes, then set/dict members
  uint32_t *ncbeg, *nccnt, *mcbeg, *mccnt;
  unsigned long long* nsum;
  OPS_TRY(D.alloc(&ncbeg, NS));
  OPS_TRY(D.alloc(&nccnt, NS));
  OPS_TRY(D.alloc(&mcbeg, NS));
  OPS_TRY(D.alloc(&mccnt, NS));
  OPS_TRY(D.alloc(&nsum, NS));
  OPS_TRY(hip_check(ctx, hipMemsetAsync(ncbeg, 0xFF, NS * 4, s), "memset"));
  OPS_TRY(hip_check(ctx, hipMemsetAsync(mcbeg, 0xFF, NS * 4, s), "memset"));
  OPS_TRY(hip_check(ctx, hipMemsetAsync(nccnt, 0, NS * 4, s), "memset"));
  OPS_TRY(hip_check(ctx, hipMemsetAsync(mccnt, 0, NS * 4, s), "memset"));
  OPS_TRY(hip_check(ctx, hipMemsetAsync(nsum, 0, NS * 8, s), "memset"));
  uint32_t *nseg_of, *mseg_of;
  OPS_TRY(D.alloc(&nseg_of, Cn));
  OPS_TRY(D.alloc(&mseg_of, Cm));
  if (Ks) state_child_seg_kernel<<<grid_for(Ks), kThreads, 0, s>>>(sk_d[O_META], sk_d[O_CREF], Ks, ev_seg, nseg_of,
                                                                    mseg_of);
  if (Nn) op_child_seg_kernel<<<grid_for(Nn), kThreads, 0, s>>>(n_op, Nn, Ns, ev_seg, Ks, nseg_of);
  if (Mm) op_child_seg_kernel<<<grid_for(Mm), kThreads, 0, s>>>(m_op, Mm, Ms, ev_seg, Ks, mseg_of);
  OPS_TRY(launch_check(ctx, s, "child segments"));
  int seg_bits = 1;
  while (seg_bits < 32 && (1ull << seg_bits) < NS) ++seg_bits;

  uint64_t out_n[2] = {0, 0};
  uint64_t* node_out[6];
  uint64_t* mem_out[6];
  for (int fam = 0; fam < 2; ++fam) {
    const bool nodes = fam == 0;
    const uint64_t C = nodes ? Cn : Cm, Cs = nodes ? Ns : Ms;
    uint64_t** outc = nodes ? node_out : mem_out;
    for (int c = 0; c < 6; ++c) OPS_TRY(D.alloc(&outc[c], C));
    if (!C) continue;
    const uint64_t* const* st = nodes ? sn_d : sm_d;
    const uint64_t* id1b = nodes ? n_node : m_h;
    const uint64_t* id2b = nodes ? n_v : m_f;
    const uint64_t* opb = nodes ? n_op : m_op;
    uint32_t* seg_of = nodes ? nseg_of : mseg_of;
    // (key segment, id1) stably: id1 first, then the segment (LSD)
    iota_gather_kernel<<<grid_for(C), kThreads, 0, s>>>(st[C_ID1], Cs, id1b, C, S.ka, S.va);
    OPS_TRY(sort_pairs(ctx, S, C, 64, s));
    regather32_kernel<<<grid_for(C), kThreads, 0, s>>>(seg_of, S.va, C, S.ka);
    OPS_TRY(sort_pairs(ctx, S, C, seg_bits, s));
    OPS_TRY(hip_check(ctx, hipMemsetAsync(dbad, 0, 8, s), "memset"));
    heads_kernel<<<grid_for(C), kThreads, 0, s>>>(S.va, C, st[C_ID1], Cs, id1b, nodes ? st[C_ID1] : st[C_ID2],
                                                   nodes ? id1b : id2b, seg_of, head, dbad);
    if (!nodes) {
      unsigned long long bad = 0;
      OPS_TRY(hip_check(ctx, hipMemcpyAsync(&bad, dbad, 8, hipMemcpyDeviceToHost, s), "d2h"));
      OPS_TRY(hip_check(ctx, hipStreamSynchronize(s), "sync"));
      if (bad) {  // member-hash collision inside a key: order by (segment, mh, mf)
        iota_gather_kernel<<<grid_for(C), kThreads, 0, s>>>(st[C_ID2], Cs, id2b, C, S.ka, S.va);
        OPS_TRY(sort_pairs(ctx, S, C, 64, s));
        regather_kernel<<<grid_for(C), kThreads, 0, s>>>(st[C_ID1], Cs, id1b, S.va, C, S.ka);
        OPS_TRY(sort_pairs(ctx, S, C, 64, s));
        regather32_kernel<<<grid_for(C), kThreads, 0, s>>>(seg_of, S.va, C, S.ka);
        OPS_TRY(sort_pairs(ctx, S, C, seg_bits, s));
        heads_kernel<<<grid_for(C), kThreads, 0, s>>>(S.va, C, st[C_ID1], Cs, id1b, st[C_ID2], id2b, seg_of, head,
                                                       dbad);
      }
    }
    uint32_t *cp, *cs_start;
    OPS_TRY(D.alloc(&cp, C));
    OPS_TRY(D.alloc(&cs_start, C + 1));
    OPS_TRY(hip_check(ctx, hipMemcpyAsync(cp, S.va, C * 4, hipMemcpyDeviceToDevice, s), "d2d"));
    uint32_t ncs = 0;
    OPS_TRY(excl_scan(ctx, S, head, C, segx, &ncs, s));
    seg_start_kernel<<<grid_for(C), kThreads, 0, s>>>(head, segx, C, cs_start);
    ChildIn CI;
    CI.s_pkh = st[C_PKH], CI.s_pkf = st[C_PKF], CI.s_id1 = st[C_ID1], CI.s_id2 = st[C_ID2], CI.s_t = st[C_T];
    CI.s_meta = st[C_META], CI.Ns = Cs;
    CI.c_id1 = id1b, CI.c_id2 = id2b, CI.c_op = opb;
    CI.o_kh = o_kh, CI.o_kf = o_kf, CI.o_uuid = o_uuid, CI.o_meta = o_meta;
    CI.op_valid = KO.op_valid, CI.op_dt = KO.op_dt, CI.sfx_u = KO.sfx_u, CI.seg_sfx_u = KO.seg_sfx_u;
    CI.sfx_seq = KO.sfx_seq, CI.seg_sfx_seq = KO.seg_sfx_seq, CI.seg_of = seg_of, CI.pos_ops = pos_ops;
    ChildOut CO;
    OPS_TRY(D.alloc(&CO.pkh, ncs));
    OPS_TRY(D.alloc(&CO.pkf, ncs));
    OPS_TRY(D.alloc(&CO.id1, ncs));
    OPS_TRY(D.alloc(&CO.id2, ncs));
    OPS_TRY(D.alloc(&CO.t, ncs));
    OPS_TRY(D.alloc(&CO.meta, ncs));
    OPS_TRY(D.alloc(&CO.produce, ncs));
    OPS_TRY(D.alloc(&CO.seg, ncs));
    if (nodes)
      node_fold_kernel<<<grid_for(ncs), kThreads, 0, s>>>(CI, CO, cp, cs_start, ncs);
    else
      member_fold_kernel<<<grid_for(ncs), kThreads, 0, s>>>(CI, CO, cp, cs_start, ncs);
    OPS_TRY(launch_check(ctx, s, "child fold"));
    uint32_t* dense;
    OPS_TRY(D.alloc(&dense, ncs));
    uint32_t nout = 0;
    OPS_TRY(excl_scan(ctx, S, CO.produce, ncs, dense, &nout, s));
    cdb_dev_rows R;
    std::memset(&R, 0, sizeof R);
    for (int c = 0; c < 6; ++c) R.col[c] = outc[c];
    child_compact_kernel<<<grid_for(ncs), kThreads, 0, s>>>(CO, dense, ncs, R, nodes ? ncbeg : mcbeg,
                                                             nodes ? nccnt : mccnt, nodes ? nsum : nullptr);
    OPS_TRY(launch_check(ctx, s, "child compact"));
    out_n[fam] = nout;
  }

  // ---- 4. keys
  uint64_t* key_out[kKeyOutCols];
  for (int c = 0; c < kKeyOutCols; ++c) OPS_TRY(D.alloc(&key_out[c], E));
  uint32_t nkeys = 0;
  if (nseg) {
    uint32_t *cnt, *dense;
    OPS_TRY(D.alloc(&cnt, nseg));
    OPS_TRY(D.alloc(&dense, nseg));
    key_count_kernel<<<grid_for(nseg), kThreads, 0, s>>>(KO.flags, nseg, cnt);
    OPS_TRY(excl_scan(ctx, S, cnt, nseg, dense, &nkeys, s));
    KeyEmit KE{KO.flags, KO.ct, KO.ut, KO.dt, KO.kmeta, KO.win, KO.exp_t, KO.exp_meta, KO.del_t, KO.del_meta,
               ncbeg, nccnt, mcbeg, mccnt, nsum, dense, perm, seg_start, sk_d[O_KH], sk_d[O_KF], o_kh, o_kf, Ks};
    cdb_dev_rows R;
    std::memset(&R, 0, sizeof R);
    for (int c = 0; c < kKeyOutCols; ++c) R.col[c] = key_out[c];
    key_emit_kernel<<<grid_for(nseg), kThreads, 0, s>>>(KE, nseg, R);
    OPS_TRY(launch_check(ctx, s, "key_emit_kernel"));
  }
  OPS_TRY(hip_check(ctx, hipEventRecord(e1, s), "event"));
  unsigned long long hs[8];
  OPS_TRY(hip_check(ctx, hipMemcpyAsync(hs, dstats, 64, hipMemcpyDeviceToHost, s), "d2h"));
  OPS_TRY(hip_check(ctx, hipStreamSynchronize(s), "sync"));
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  // ---- download
  auto down = [&](ColVec* dst, int nc, uint64_t* const* src, uint64_t n) -> cdb_status {
    for (int c = 0; c < nc; ++c) {
      dst[c].resize(n);  // default-initialised
      advise_huge(dst[c].data(), n * 8);
      OPS_TRY(staged_d2h(ctx, dst[c].data(), src[c], n * 8, s));
    }
    return CDB_OK;
  };
  OPS_TRY(down(ok, kKeyOutCols, key_out, nkeys));
  OPS_TRY(down(on, kNodeCols, node_out, out_n[0]));
  OPS_TRY(down(om, kMemberCols, mem_out, out_n[1]));
  if (stats) {
    std::memset(stats, 0, sizeof *stats);
    stats->ops_in = Ko;
    stats->node_args_in = Nn;
    stats->member_args_in = Mm;
    stats->key_rows_in = Ks;
    stats->key_rows_out = nkeys;
    stats->node_rows_out = out_n[0];
    stats->member_rows_out = out_n[1];
    stats->type_errors = hs[0];
    stats->expired_on_query = hs[1];
    stats->device_ms = ms;
  }
  return CDB_OK;
}

}  // namespace cdb
