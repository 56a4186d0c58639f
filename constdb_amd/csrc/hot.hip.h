// Over-capacity buckets whose keys fit the workgroup tier but whose children do not (config C5:
// a few keys own up to millions of counter nodes or set/dict members; the per-key loops of
// type_counter.rs:59-87 and lwwhash.rs:319-323 are then the whole cost). The keys of such a
// bucket are sorted and folded by one workgroup (bucket_keys), and its children are spread over
// the whole chip instead:
//   hot_keys_kernel : one workgroup per hot bucket: the key phase; the bucket's output keys go to
//                     a global key table at hk_off[h] (G = hk_off[h] + rank is a chip-wide key id);
//   hot_tag_kernel  : one thread per child (flat order): finds its key (binary search of the
//                     bucket's table), copies the fields the fold reads into a 32-B record,
//                     decides whether it takes part (head type, element type, remote dels
//                     ignored, exactly as the wave tier) and tags it with
//                     W = G << g_shift | id-hash top (g_shift - 6) bits << 6 | pos (g_shift:
//                     40, or less where that saves a sort pass -- see chip_wide); a child that
//                     takes no part gets its bucket's marker (every W bit of the bucket's last key
//                     set: pos 63, which no row has, and an id field no child gets), so it sorts
//                     to the end of its bucket's children and every bucket's children keep their
//                     flat range;
//   radix sort of (W, child) pairs (radix.hip.h) on W's bits above pos, stable, so equal W >> 6
//                     keep (bucket, row) order: run order, which is fold order on the sorted-run
//                     path unless two ids share the hash bits;
//                     W orders the buckets, so bucket h's children (markers last) keep its flat
//                     range [c_off[h], c_off[h + 1]);
//   hot_fold_kernel : one thread per W-run (a (key, child id) group, ~ one row per replica):
//                     folds every exact child id of the run in (pos, src) order -- Counter::merge's
//                     head-t rule or LWWHash::set's later-wins rule -- counting outputs (pass 0)
//                     or writing them at their rank inside the bucket (pass 1, after a scan);
//   hot_finish_kernel: counter sums (cal_sum) and child ranges into the key rows, bucket counts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bucket.hip.h"
#include "common.h"
#include "runs.hip.h"

namespace cdb {

constexpr int kHotIdBits = 40;     // largest g_shift: W = G << 40 | (child-id hash >> 30) << 6 | pos
constexpr int kHotMinIdBits = 20;  // fewest id-hash bits chosen to save a sort pass

struct HotArgs {
  const uint32_t* ids;       // hot bucket of h
  const uint32_t* hk_off;    // first key-table slot of h (prefix of the key rows)
  const uint32_t* c_off;     // first flat child of h (prefix of nodes + members), H + 1 entries
  uint32_t H;
  // key table (G)
  uint64_t *hk_h, *hk_f, *hk_vm;
  unsigned long long* hk_sum;
  uint32_t *hk_tp, *hk_cnt, *hk_cb;
  uint32_t* hk_kout;         // per h
  // children
  uint64_t* w;               // W per flat child (then sorted)
  uint32_t* v;               // flat child index (then sorted)
  ulonglong2* rec;           // flat child j's fold fields: rec[2j] = (id1, id2), rec[2j + 1] = (t, meta)
  uint32_t* c_h;             // bucket h of flat child j, bit 31 = member
  uint32_t *emit_n, *emit_m; // per sorted position: outputs of the run starting there
  const uint32_t *rank_n, *rank_m;  // exclusive scans of emit_n / emit_m
  uint64_t n_children;
  int id_shift;              // W's id bits = id hash >> id_shift (64 + 6 - g_shift; larger in tests)
  int g_shift;               // W's key-id bits start here (kHotIdBits or less)
  uint32_t* run_list;        // sorted position of every run's first row, ascending
  const uint64_t* run_count; // runs in run_list (device)
  uint32_t* fold_q;          // per run start: the sorted position whose row is the output
                             // (members: the winner; nodes: the head), kNone: selection path
  uint64_t* fold_v;          // per run start: a counter node's folded value
  // runs mode (sorted-run input, buckets of at most MatArgs::runs_child_max children): the
  // tag pass reads the children from the runs' columns (the absolute run row), not from copies
  int runs;
  RunView V;
};

// A child's columns: its copied AoS row, or (runs mode) the runs' SoA columns.
__device__ __forceinline__ uint64_t hot_col(const BucketArgs& A, const HotArgs& H, bool isn, uint32_t row, int c) {
  if (H.runs) return row_field(isn ? H.V.nin : H.V.min, isn ? H.V.ns : H.V.ms, c, row);
  return (isn ? A.nr : A.mr)[(uint64_t)row * kChildStride + c];
}

__device__ __forceinline__ uint32_t hot_bucket_of(const HotArgs& H, uint64_t j) {  // last h: c_off[h] <= j
  uint32_t lo = 0, hi = H.H;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (H.c_off[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// The W of bucket h's children that take no part: above every W of the bucket (its last key id,
// every id bit, pos 63) and below every W of the next bucket.
__device__ __forceinline__ uint64_t hot_marker(const HotArgs& H, uint32_t h) {
  return ((uint64_t)H.hk_off[h + 1] << H.g_shift) - 1;
}
__device__ __forceinline__ bool hot_takes_part(uint64_t W) { return (W & 63) != 63; }

__global__ void __launch_bounds__(kBktThreads) hot_keys_kernel(BucketArgs A, HotArgs H) {
  __shared__ LdsPool L;
  Scratch S;
  S.kh = L.kh; S.kf = L.kf; S.meta = L.meta;
  S.idx = L.idx; S.rk = L.rk; S.flag = L.flag; S.rank = L.rank; S.cnt = L.cnt;
  S.okh = L.okh; S.okf = L.okf; S.ovm = L.ovm; S.osum = L.osum;
  S.otp = L.otp; S.ocb = L.ocb; S.occ = L.occ;
  S.c1 = L.c1; S.c2 = L.c2; S.cm = L.cm; S.rt = L.rt; S.rm = L.rm;
  S.ck = L.ck; S.cidx = L.cidx; S.crk = L.crk; S.cflag = L.cflag; S.crank = L.crank;
  S.st = L.st; S.misc = L.misc;
  const uint32_t h = blockIdx.x, b = H.ids[h];
  const uint32_t kout = bucket_keys(A, b, S);
  const uint32_t g0 = H.hk_off[h];
  for (uint32_t o = threadIdx.x; o < kout; o += blockDim.x) {
    H.hk_h[g0 + o] = S.okh[o];
    H.hk_f[g0 + o] = S.okf[o];
    H.hk_vm[g0 + o] = S.ovm[o];
    H.hk_sum[g0 + o] = S.osum[o];
    H.hk_tp[g0 + o] = S.otp[o];
    H.hk_cnt[g0 + o] = 0;
    H.hk_cb[g0 + o] = kNone;
  }
  if (threadIdx.x == 0) H.hk_kout[h] = kout;
  __syncthreads();
  for (int i = threadIdx.x; i < ST_COUNT; i += blockDim.x)
    if (S.st[i]) atomicAdd(&stat_shard(A.stats)[i], S.st[i]);
}

__global__ void __launch_bounds__(256) hot_tag_kernel(BucketArgs A, HotArgs H) {
  const int ks = A.key_shift;
  unsigned long long orph = 0;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < H.n_children;
       j += (uint64_t)gridDim.x * blockDim.x) {
    // the wave's children are consecutive: lane 0 (active whenever any lane is) searches the
    // bucket of the first, the others step forward from it (buckets here hold hundreds of rows)
    uint32_t h = lane == 0 ? hot_bucket_of(H, j) : 0;
    h = (uint32_t)__shfl((int)h, 0);
    while (h + 1 < H.H && H.c_off[h + 1] <= j) ++h;
    const uint32_t b = H.ids[h];
    const uint32_t i = (uint32_t)(j - H.c_off[h]), N = A.ncnt[b];
    const bool isn = i < N;
    uint32_t row;
    if (H.runs) {  // the bucket's slices of the family's runs, in run order (as mat_copy lays them)
      const int f = isn ? 1 : 2;
      uint32_t k = isn ? i : i - N, r = 0;
      for (;; ++r) {
        const uint32_t* d = H.V.rdir[f] + (uint64_t)r * H.V.nbp1 + b;
        const uint32_t len = d[1] - d[0];
        if (k < len || r + 1 >= H.V.nr) {
          row = d[0] + k;  // (absolute rows)
          break;
        }
        k -= len;
      }
    } else {
      row = isn ? A.np[A.nbase[b] + i] : A.mp[A.mbase[b] + (i - N)];
    }
    const uint64_t pkh = hot_col(A, H, isn, row, C_PKH), pkf = hot_col(A, H, isn, row, C_PKF);
    const uint64_t id1 = hot_col(A, H, isn, row, C_ID1), m = hot_col(A, H, isn, row, C_META);
    const uint64_t id2 = hot_col(A, H, isn, row, C_ID2), t = hot_col(A, H, isn, row, C_T);
    // lower bound over the bucket's sorted output keys on (kh << shift, kh, kf)
    const uint32_t g0 = H.hk_off[h], kout = H.hk_kout[h];
    uint32_t lo = 0, hi = kout;
    const uint64_t sp = pkh << ks;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint64_t kh = H.hk_h[g0 + mid], sm = kh << ks;
      const bool less = sm < sp || (sm == sp && (kh < pkh || (kh == pkh && H.hk_f[g0 + mid] < pkf)));
      lo = less ? mid + 1 : lo;
      hi = less ? hi : mid;
    }
    uint64_t w = hot_marker(H, h);
    if (lo < kout && H.hk_h[g0 + lo] == pkh && H.hk_f[g0 + lo] == pkf && (H.hk_tp[g0 + lo] & 0xFF) <= TAG_SET) {
      const uint32_t T = H.hk_tp[g0 + lo] & 0xFF, hp = H.hk_tp[g0 + lo] >> 8, p = meta_pos(m);
      const bool type_ok = isn ? T == TAG_COUNTER : (T == TAG_SET || T == TAG_DICT);
      const bool elem_ok = (H.hk_vm[g0 + lo] >> p) & 1;
      const bool cand = isn || meta_tag(m) == KIND_ADD || p == hp;  // remote dels ignored
      if (type_ok && elem_ok && cand) {
        // (the id field stops one below all ones: the marker is above every W of the bucket in
        // the sorted bits, which leave out the pos bits)
        const uint64_t ih = isn ? mix64(id1) : id1, top = (1ull << (H.g_shift - 6)) - 2;
        w = ((uint64_t)(g0 + lo) << H.g_shift) | (min(ih >> H.id_shift, top) << 6) | p;
      }
    } else {
      ++orph;
    }
    H.w[j] = w;
    H.v[j] = (uint32_t)j;
    // the fold reads a child's four fields as one 32-B record (flat order: written in sequence)
    H.rec[2 * j] = make_ulonglong2(id1, id2);
    H.rec[2 * j + 1] = make_ulonglong2(t, m);
    H.c_h[j] = h | (isn ? 0u : 0x80000000u);
  }
  if (orph) atomicAdd(&stat_shard(A.stats)[ST_ORPHANS], orph);
}

// One child of a W-run, by sorted position q (j: its flat index, the last tie-break).
struct HotChild {
  uint64_t id1, id2, t, meta;
  uint32_t j;
};
__device__ __forceinline__ HotChild hot_child(const HotArgs& H, uint64_t q) {
  const uint32_t j = H.v[q];
  const ulonglong2 a = H.rec[2 * (uint64_t)j], b = H.rec[2 * (uint64_t)j + 1];
  HotChild c;
  c.id1 = a.x;
  c.id2 = a.y;
  c.t = b.x;
  c.meta = b.y;
  c.j = j;
  return c;
}
// Total order of a run's rows: exact id (nodes: the node id alone), fold position (pos, src),
// flat index. The fold visits the rows in this order.
__device__ __forceinline__ bool hot_before(const HotChild& a, const HotChild& b, bool isn) {
  if (a.id1 != b.id1) return a.id1 < b.id1;
  if (!isn && a.id2 != b.id2) return a.id2 < b.id2;
  const uint64_t oa = meta_order(a.meta), ob = meta_order(b.meta);
  if (oa != ob) return oa < ob;
  return a.j < b.j;
}

// Run starts: flag per sorted position (then an exclusive scan gives each run its index).
__global__ void __launch_bounds__(256) hot_runflag_kernel(HotArgs H, uint32_t* __restrict__ flag) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < H.n_children;
       p += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t W = H.w[p];
    // a run: equal W but the pos bits (a marker never starts one; one before W belongs to an
    // earlier bucket, so it never hides a start either)
    flag[p] = hot_takes_part(W) && !(p > 0 && (H.w[p - 1] >> 6) == (W >> 6));
  }
}
__global__ void __launch_bounds__(256) hot_runlist_kernel(HotArgs H, const uint32_t* __restrict__ flag,
                                                          const uint32_t* __restrict__ idx) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < H.n_children;
       p += (uint64_t)gridDim.x * blockDim.x)
    if (flag[p]) H.run_list[idx[p]] = (uint32_t)p;
}

constexpr uint32_t kFoldFast = 8;  // runs up to this many rows: rows in registers, loads overlapped

// One thread per run. Pass 0: the run's output count (emit_n / emit_m at its first position)
// and, for a run of one exact id whose rows arrive in strictly increasing (pos, src) order (the
// tag's low bits are the position) and no longer than kFoldFast, the output row's position and
// value (fold_q / fold_v); pass 1 writes outputs at their rank. Other runs (ids sharing the
// tag's id-hash bits -- g_shift - 6 of them, 20 to 34 -- and long runs) fold by successor selection in both passes: each step selects the successor
// of the last visited row (O(run^2) over rows in L2, no per-thread arrays), so rows are folded
// in order whatever order the sort left them in. Loops have wave-uniform trip counts with
// per-lane predicates: a loop-carried row must not be a live-out of a loop with divergent exits
// (gfx950 compilers have produced the first candidate instead of the smallest there).
__global__ void __launch_bounds__(256) hot_fold_kernel(BucketArgs A, HotArgs H, int pass) {
  unsigned long long gcm = 0, nslow = 0;
  const uint64_t nruns = *H.run_count;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < nruns; base += stride) {  // wave-uniform
    const uint64_t i = base + threadIdx.x;
    const bool act = i < nruns;
    const uint64_t p = act ? H.run_list[i] : 0;
    const uint64_t W = H.w[p];
    uint32_t nrows = 0;
    if (act) {
      uint64_t e = p + 1;
      while (e < H.n_children && (H.w[e] >> 6) == (W >> 6) && hot_takes_part(H.w[e])) ++e;
      nrows = (uint32_t)(e - p);
    }
    uint32_t hc = 0, h = 0, b = 0, G = 0;
    bool isn = false;
    uint64_t obase = 0;
    if (act) {
      hc = H.c_h[H.v[p]];
      h = hc & 0x7FFFFFFFu;
      isn = (hc >> 31) == 0;
      b = H.ids[h];
      G = (uint32_t)(W >> H.g_shift);
      if (pass == 1) obase = (isn ? H.rank_n[p] - H.rank_n[H.c_off[h]] : H.rank_m[p] - H.rank_m[H.c_off[h]]);
    }
    uint32_t nout = 0;
    // this run's contribution to its key's row: outputs, first output slot, counter sum (one
    // atomic per key and wave below, not per output: a hot key owns up to millions of them)
    uint32_t k_cnt = 0, k_cb = kNone;
    unsigned long long k_sum = 0;
    auto put = [&](uint64_t id1, uint64_t id2, uint64_t t, uint64_t meta, uint64_t v) {
      const uint32_t o = (uint32_t)(obase + nout);
      uint64_t* row = (isn ? A.nos + (uint64_t)(A.nbase[b] + o) * kChildStride
                           : A.mos + (uint64_t)(A.mbase[b] + o) * kChildStride);
      row[C_PKH] = H.hk_h[G];
      row[C_PKF] = H.hk_f[G];
      row[C_ID1] = id1;
      row[C_ID2] = isn ? v : id2;
      row[C_T] = t;
      row[C_META] = isn ? meta_pack(0, meta_pos(meta), meta_src(meta)) : meta;
      k_cb = min(k_cb, o);
      ++k_cnt;
      k_sum += isn ? v : 0;
    };
    auto emit_id = [&](const HotChild& hd, uint64_t v, uint64_t tw, uint64_t wmeta) {
      if (!isn && (A.flags & F_GC_MEMBERS) && meta_tag(wmeta) == KIND_DEL && tw < A.gc_wm) {
        ++gcm;
        return;
      }
      if (pass == 1) put(hd.id1, hd.id2, isn ? hd.t : tw, isn ? hd.meta : wmeta, v);
      ++nout;
    };
    bool slow = act;
    if (pass == 0) {
      // fast path: up to kFoldFast rows, their loads issued together
      const bool fast = act && nrows <= kFoldFast;
      uint32_t rj[kFoldFast];
#pragma unroll
      for (uint32_t k = 0; k < kFoldFast; ++k) rj[k] = (fast && k < nrows) ? H.v[p + k] : 0;
      uint64_t xi1[kFoldFast], xi2[kFoldFast], xt[kFoldFast], xm[kFoldFast];
#pragma unroll
      for (uint32_t k = 0; k < kFoldFast; ++k) {
        if (fast && k < nrows) {
          const ulonglong2 a = H.rec[2 * (uint64_t)rj[k]], c = H.rec[2 * (uint64_t)rj[k] + 1];
          xi1[k] = a.x;
          xi2[k] = a.y;
          xt[k] = c.x;
          xm[k] = c.y;
        } else {
          xi1[k] = xi2[k] = xt[k] = xm[k] = 0;
        }
      }
      bool simple = fast;
      uint64_t v = xi2[0], tw = xt[0];
      uint32_t qw = 0;  // winner (members)
#pragma unroll
      for (uint32_t k = 1; k < kFoldFast; ++k) {
        if (k < nrows) {
          simple = simple && xi1[k] == xi1[0] && (isn || xi2[k] == xi2[0]) &&
                   meta_order(xm[k]) > meta_order(xm[k - 1]);
          if (isn) {  // Counter::merge (type_counter.rs:60-84): the head's t is kept
            v = xt[k] > xt[0] ? xi2[k] : (xt[k] == xt[0] ? imax64(v, xi2[k]) : v);
          } else if (!(tw > xt[k])) {  // LWWHash::set (lwwhash.rs:87-107): later wins ties
            tw = xt[k];
            qw = k;
          }
        }
      }
      if (simple) {
        uint64_t wm = xm[0];
#pragma unroll
        for (uint32_t k = 1; k < kFoldFast; ++k) wm = (k == qw) ? xm[k] : wm;
        HotChild hd;
        hd.id1 = xi1[0];
        hd.id2 = xi2[0];
        hd.t = xt[0];
        hd.meta = xm[0];
        hd.j = 0;
        emit_id(hd, v, tw, wm);
        H.fold_q[p] = (uint32_t)(p + (isn ? 0 : qw));
        H.fold_v[p] = v;
        slow = false;
      } else if (act) {
        H.fold_q[p] = kNone;
      }
    } else if (act) {  // pass 1, fold kept by pass 0
      const uint32_t q = H.fold_q[p];
      if (q != kNone) {
        slow = false;
        if ((isn ? H.emit_n : H.emit_m)[p]) {
          const HotChild x = hot_child(H, q);
          put(x.id1, x.id2, x.t, x.meta, H.fold_v[p]);
        }
      }
    }
    // selection path
    nslow += (pass == 0 && slow) ? 1 : 0;
    uint32_t kslow = slow ? nrows : 0;
    for (int off = 32; off > 0; off >>= 1) kslow = max(kslow, (uint32_t)__shfl_xor((int)kslow, off));
    HotChild last, head;  // last visited row; first row of the id being folded
    last.id1 = last.id2 = last.t = last.meta = 0;
    last.j = 0;
    head = last;
    uint64_t v = 0, tw = 0, wmeta = 0;  // the fold of head's id so far
    bool open = false;                  // head's id has rows not yet emitted
    for (uint32_t step = 0; step < kslow + 1 && kslow; ++step) {
      HotChild c = last;
      bool have = false;
      for (uint32_t k = 0; k < kslow; ++k) {
        if (slow && k < nrows && step < nrows) {
          const HotChild x = hot_child(H, p + k);
          const bool after = step == 0 || hot_before(last, x, isn);
          const bool take = after && (!have || hot_before(x, c, isn));
          c.id1 = take ? x.id1 : c.id1;
          c.id2 = take ? x.id2 : c.id2;
          c.t = take ? x.t : c.t;
          c.meta = take ? x.meta : c.meta;
          c.j = take ? x.j : c.j;
          have = have || take;
        }
      }
      const bool new_id = !have || !open || c.id1 != head.id1 || (!isn && c.id2 != head.id2);
      if (slow && open && new_id) {  // head's id is complete: emit it
        emit_id(head, v, tw, wmeta);
        open = false;
      }
      if (slow && have) {
        if (new_id) {  // c opens an id
          head = c;
          v = c.id2;
          tw = c.t;
          wmeta = c.meta;
          open = true;
        } else if (isn) {
          v = c.t > head.t ? c.id2 : (c.t == head.t ? imax64(v, c.id2) : v);
        } else if (!(tw > c.t)) {
          tw = c.t;
          wmeta = c.meta;
        }
        last = c;
      }
    }
    if (pass == 0 && act) (isn ? H.emit_n : H.emit_m)[p] = nout;
    if (pass == 1) {
      // runs are in sorted order, so the wave's active lanes hold non-decreasing keys G:
      // a segmented reduction per key, and the segment's last lane does the atomics
      const uint32_t key = act ? G : kNone;  // inactive lanes only at the tail: segments are contiguous
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t gk = (uint32_t)__shfl_up((int)key, d);
        const uint32_t c2 = (uint32_t)__shfl_up((int)k_cnt, d);
        const uint32_t b2 = (uint32_t)__shfl_up((int)k_cb, d);
        const unsigned long long s2 = __shfl_up(k_sum, d);
        if (lane >= (uint32_t)d && gk == key) {
          k_cnt += c2;
          k_cb = min(k_cb, b2);
          k_sum += s2;
        }
      }
      const uint32_t next = (uint32_t)__shfl_down((int)key, 1);
      if (key != kNone && k_cnt && (lane == 63 || next != key)) {
        atomicMin(&H.hk_cb[G], k_cb);
        atomicAdd(&H.hk_cnt[G], k_cnt);
        if (isn && (H.hk_vm[G] & kVmaskMerged)) atomicAdd(&H.hk_sum[G], k_sum);
      }
    }
  }
  if (pass == 0 && gcm) atomicAdd(&stat_shard(A.stats)[ST_MEMBERS_GCED], gcm);
  if (nslow) atomicAdd(&stat_shard(A.stats)[ST_HOT_SLOW], nslow);
}

// Key rows: counter sums and child ranges (bucket-relative, as every tier leaves them for the
// compaction); the bucket's output counts.
__global__ void __launch_bounds__(256) hot_finish_kernel(BucketArgs A, HotArgs H) {
  const uint32_t h = blockIdx.x, b = H.ids[h];
  const uint32_t g0 = H.hk_off[h], kout = H.hk_kout[h], kb = A.kbase[b];
  uint32_t nn = 0, nm = 0;
  for (uint32_t o = threadIdx.x; o < kout; o += blockDim.x) {
    const uint32_t G = g0 + o, T = H.hk_tp[G] & 0xFF, cnt = H.hk_cnt[G];
    if (T == TAG_COUNTER) {
      A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_WIN] = H.hk_sum[G];
      nn += cnt;
    } else if (T == TAG_SET || T == TAG_DICT) {
      nm += cnt;
    }
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_CREF] = cref_pack(cnt ? H.hk_cb[G] : 0, cnt);
  }
  __shared__ uint32_t tot[2];
  if (threadIdx.x == 0) tot[0] = tot[1] = 0;
  __syncthreads();
  if (nn) atomicAdd(&tot[0], nn);
  if (nm) atomicAdd(&tot[1], nm);
  __syncthreads();
  if (threadIdx.x == 0) {
    A.kout[b] = kout;
    A.nout[b] = tot[0];
    A.mout[b] = tot[1];
  }
}

// Row counts of the listed buckets, for the host's plan of the over-capacity path.
__global__ void hot_counts_kernel(BucketArgs A, const uint32_t* __restrict__ list, uint32_t n, uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = list[i];
  out[3 * i] = A.kcnt[b];
  out[3 * i + 1] = A.ncnt[b];
  out[3 * i + 2] = A.mcnt[b];
}

}  // namespace cdb
