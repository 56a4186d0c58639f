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
//                     W = G << g_shift | child_order(id1) top (g_shift - 6) bits << 6 | pos (g_shift:
//                     40, or less where that saves a sort pass -- see chip_wide); a child that
//                     takes no part gets its bucket's marker (every W bit of the bucket's last key
//                     set: pos 63, which no row has, and an id field no child gets), so it sorts
//                     to the end of its bucket's children and every bucket's children keep their
//                     flat range;
//   the sort: a merge of the buckets' sorted child lists when they arrive sorted (a merge result's
//                     child order: hot_merge_kernel below), else
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

constexpr int kHotIdBits = 40;     // largest g_shift: W = G << 40 | (child_order(id1) >> 30) << 6 | pos
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
  uint32_t *emit_n, *emit_m; // per run (global sort): its node / member outputs
  const uint32_t *rank_n, *rank_m;  // exclusive scans of emit_n / emit_m
  uint32_t* first_run;       // per bucket h: its first run (global sort)
  uint64_t n_children;
  int id_shift;              // W's id bits = id hash >> id_shift (64 + 6 - g_shift; larger in tests)
  int g_shift;               // W's key-id bits start here (kHotIdBits or less)
  uint32_t* run_list;        // sorted position of every run's first row, ascending
  const uint64_t* run_count; // runs in run_list (device)
  uint32_t* fold_q;          // per run: the row of the run (k from its start) that is the output
                             // (members: the winner; nodes: the head), kNone: selection path
  uint64_t* fold_v;          // per run: a counter node's folded value
  // the global sort's fold, per run folded by pass 0 (fold_q != kNone): its output row's fields
  // (fold_rec[2 i] = (id1, id2 | a node's value), [2 i + 1] = (t, meta)) and (c_h of its rows, key
  // G) in fold_hg[i], so that pass 1 writes it without re-reading the run's rows (null: re-read)
  ulonglong2* fold_rec;
  uint2* fold_hg;
  // runs mode (sorted-run input, buckets of at most MatArgs::runs_child_max children): the
  // tag pass reads the children from the runs' columns (the absolute run row), not from copies
  int runs;
  RunView V;
  unsigned long long* prof;  // test hook (CDB_HOT_PROF): hot_sortfold_kernel's phase clocks, or null
  int small_keys;            // every bucket of the batch has at most kTagKeys output keys: the tag
                             // kernel searches its buckets' key tables in LDS
  int flagged;               // the sorted tags may hold inline markers (v's kInlineMarker bit)
  int direct;                // global path: v = the child's row (| kMemberBit for a member row),
                             // the fold reads the row itself; no rec records, no c_h; a key's
                             // bucket from hk_bkt
  uint32_t* hk_bkt;          // per key G: its bucket h
  int inline_markers;        // tag: a child that takes no part keeps the W it would have (its list
                             // stays sorted for the merge) and is flagged in v (kInlineMarker)
                             // instead of getting the bucket's marker
  int orphans_counted;       // tag: a previous tag pass of this batch already counted its orphan
                             // children (the list merge's, before a fallback re-tag): not again
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
// v's top bit: a child that takes no part, tagged with its own W (HotArgs::inline_markers); the low
// 31 bits are the flat index.
constexpr uint32_t kInlineMarker = 0x80000000u;
constexpr uint32_t kMemberBit = 0x40000000u;  // (direct mode: v's family bit; rows below 2^30)
__device__ __forceinline__ bool hot_row_part(uint64_t W, uint32_t v) { return hot_takes_part(W) && !(v & kInlineMarker); }

// The key phase's LDS (bucket_keys touches no child arrays): sized for KC key rows, so that batches
// of buckets of at most 256 keys run several workgroups per CU.
template <uint32_t KC>
struct KeyLds {
  uint64_t kh[KC], kf[KC], meta[KC];
  uint64_t okh[KC], okf[KC], ovm[KC], osum[KC];
  uint32_t idx[KC], rk[KC], flag[KC], rank[KC];
  uint32_t otp[KC], ocb[KC], occ[KC];
  uint32_t cnt[(kDig > KC + 1 ? kDig : KC + 1) + 1];
  unsigned long long st[ST_COUNT];
  uint32_t misc[32];
};

template <uint32_t KC>
__global__ void __launch_bounds__(kBktThreads) hot_keys_kernel(BucketArgs A, HotArgs H) {
  __shared__ KeyLds<KC> L;
  Scratch S = {};
  S.kh = L.kh; S.kf = L.kf; S.meta = L.meta;
  S.idx = L.idx; S.rk = L.rk; S.flag = L.flag; S.rank = L.rank; S.cnt = L.cnt;
  S.okh = L.okh; S.okf = L.okf; S.ovm = L.ovm; S.osum = L.osum;
  S.otp = L.otp; S.ocb = L.ocb; S.occ = L.occ;
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
    H.hk_bkt[g0 + o] = h;
  }
  if (threadIdx.x == 0) H.hk_kout[h] = kout;
  __syncthreads();
  for (int i = threadIdx.x; i < ST_COUNT; i += blockDim.x)
    if (S.st[i]) atomicAdd(&stat_shard(A.stats)[i], S.st[i]);
}

// Bucket h's output keys: the global key table (from hk_off[h]), or a workgroup's copy in LDS.
struct HotKeyTab {
  const uint64_t *kh, *kf, *vm;
  const uint32_t* tp;
};
__device__ __forceinline__ HotKeyTab hot_key_tab(const HotArgs& H, uint32_t g0) {
  HotKeyTab T;
  T.kh = H.hk_h + g0;
  T.kf = H.hk_f + g0;
  T.vm = H.hk_vm + g0;
  T.tp = H.hk_tp + g0;
  return T;
}

// Row of child i (flat order: nodes, then members) of bucket b: the bucket's slices of the family's
// runs, in run order (as mat_copy lays them), or its partitioned row list.
__device__ __forceinline__ uint32_t hot_row(const BucketArgs& A, const HotArgs& H, uint32_t b, uint32_t i,
                                            uint32_t N) {
  const bool isn = i < N;
  if (!H.runs) return isn ? A.np[A.nbase[b] + i] : A.mp[A.mbase[b] + (i - N)];
  const int f = isn ? 1 : 2;
  uint32_t k = isn ? i : i - N;
  for (uint32_t r = 0;; ++r) {
    const uint32_t* d = H.V.rdir[f] + (uint64_t)r * H.V.nbp1 + b;
    const uint32_t len = d[1] - d[0];
    if (k < len || r + 1 >= H.V.nr) return d[0] + k;  // (absolute rows)
    k -= len;
  }
}

// The fields of a child row the tag and the fold read: 16-B loads where two are adjacent (records
// pkf id1 id2 t meta at 8-B alignment; copied rows pkh pkf id1 id2 t meta, 16-B aligned).
struct HotFields {
  uint64_t pkh, pkf, id1, id2, t, m;
};
__device__ __forceinline__ HotFields hot_fields(const BucketArgs& A, const HotArgs& H, bool isn, uint32_t row) {
  HotFields F;
  if (H.runs) {
    const uint64_t* const* col = isn ? H.V.nin : H.V.min;
    const uint32_t st = isn ? H.V.ns : H.V.ms;
    F.pkh = col[C_PKH][row];
    if (st > 1) {
      const uint64_t* r = col[1] + (uint64_t)row * st;
      const u64x2 a = *(const u64x2*)(r + 1), c = *(const u64x2*)(r + 3);
      F.pkf = r[0];
      F.id1 = a.x;
      F.id2 = a.y;
      F.t = c.x;
      F.m = c.y;
    } else {
      F.pkf = col[C_PKF][row];
      F.id1 = col[C_ID1][row];
      F.id2 = col[C_ID2][row];
      F.t = col[C_T][row];
      F.m = col[C_META][row];
    }
  } else {
    const ulonglong2* r = (const ulonglong2*)((isn ? A.nr : A.mr) + (uint64_t)row * kChildStride);
    const ulonglong2 a = r[0], b = r[1], c = r[2];
    F.pkh = a.x;
    F.pkf = a.y;
    F.id1 = b.x;
    F.id2 = b.y;
    F.t = c.x;
    F.m = c.y;
  }
  return F;
}

// Flat child j of hot bucket h (fields F, a node when isn): its fold fields into rec[j] and its tag
// W (when it takes no part: the bucket's marker; with inline_markers, when its key is in the bucket,
// the W it would have, and *inline_marker is set -- the tag kernel flags it in v's top bit; orph
// counts children whose key is not in the bucket). T: the bucket's kout output keys.
__device__ __forceinline__ uint64_t hot_tag_row(const BucketArgs& A, const HotArgs& H, uint32_t h, uint64_t j,
                                                bool isn, const HotFields& F, const HotKeyTab& T, uint32_t kout,
                                                unsigned long long& orph, bool* inline_marker = nullptr) {
  const int ks = A.key_shift;
  const uint64_t pkh = F.pkh, pkf = F.pkf, id1 = F.id1, id2 = F.id2, t = F.t, m = F.m;
  // lower bound over the bucket's sorted output keys on (kh << shift, kh, kf)
  const uint32_t g0 = H.hk_off[h];
  uint32_t lo = 0, hi = kout;
  const uint64_t sp = pkh << ks;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint64_t kh = T.kh[mid], sm = kh << ks;
    const bool less = sm < sp || (sm == sp && (kh < pkh || (kh == pkh && T.kf[mid] < pkf)));
    lo = less ? mid + 1 : lo;
    hi = less ? hi : mid;
  }
  uint64_t w = hot_marker(H, h);
  const bool found = lo < kout && T.kh[lo] == pkh && T.kf[lo] == pkf;
  // (the id field stops one below all ones: the bucket's marker is above every W of the bucket in
  // the sorted bits, which leave out the pos bits)
  const uint64_t ih = child_order(id1), top = (1ull << (H.g_shift - 6)) - 2;
  const uint64_t wk = ((uint64_t)(g0 + lo) << H.g_shift) | (min(ih >> H.id_shift, top) << 6);
  if (found && (T.tp[lo] & 0xFF) <= TAG_SET) {
    const uint32_t TT = T.tp[lo] & 0xFF, hp = T.tp[lo] >> 8, p = meta_pos(m);
    const bool type_ok = isn ? TT == TAG_COUNTER : (TT == TAG_SET || TT == TAG_DICT);
    const bool elem_ok = (T.vm[lo] >> p) & 1;
    const bool cand = isn || meta_tag(m) == KIND_ADD || p == hp;  // remote dels ignored
    if (type_ok && elem_ok && cand) {
      w = wk | p;
    } else if (H.inline_markers) {
      w = wk | p;
      *inline_marker = true;
    }
  } else {
    ++orph;
    if (found && H.inline_markers) {
      w = wk | meta_pos(m);
      *inline_marker = true;
    }
  }
  // the fold reads a child's four fields as one 32-B record (flat order: written in sequence)
  if (!H.direct) {
    H.rec[2 * j] = make_ulonglong2(id1, id2);
    H.rec[2 * j + 1] = make_ulonglong2(t, m);
  }
  return w;
}

__device__ __forceinline__ uint64_t hot_tag_child(const BucketArgs& A, const HotArgs& H, uint32_t h, uint64_t j,
                                                  unsigned long long& orph) {
  const uint32_t b = H.ids[h];
  const uint32_t i = (uint32_t)(j - H.c_off[h]), N = A.ncnt[b];
  const bool isn = i < N;
  return hot_tag_row(A, H, h, j, isn, hot_fields(A, H, isn, hot_row(A, H, b, i, N)), hot_key_tab(H, H.hk_off[h]),
                     H.hk_kout[h], orph);
}

// One block per kTagChunk consecutive flat children: its first bucket is searched once, and the
// run slices of that bucket and the next (a chunk of a big bucket spans at most two) come from LDS.
constexpr uint32_t kTagChunk = 4096;
constexpr uint32_t kTagKeys = 256;
__global__ void __launch_bounds__(256) hot_tag_kernel(BucketArgs A, HotArgs H) {
  __shared__ uint32_t sl[2][4 * kMaxRuns];  // bucket h0 + slot: [family][run] first row, rows before
  __shared__ uint64_t tk[2][3][kTagKeys];   // (small_keys) bucket h0 + slot's keys: kh, kf, vm
  __shared__ uint32_t ttp[2][kTagKeys];     // ... and tag / pos words
  __shared__ uint32_t h_first;
  unsigned long long orph = 0;
  const uint32_t tid = threadIdx.x;
  const uint64_t j0 = (uint64_t)blockIdx.x * kTagChunk;
  if (tid == 0) h_first = hot_bucket_of(H, j0);
  __syncthreads();
  const uint32_t h0 = h_first;
  const uint32_t nr = H.runs ? H.V.nr : 0;
  if (H.small_keys) {
    for (uint32_t slot = 0; slot < 2 && h0 + slot < H.H; ++slot) {
      const uint32_t g0 = H.hk_off[h0 + slot], ko = H.hk_kout[h0 + slot];
      for (uint32_t o = tid; o < ko; o += blockDim.x) {
        tk[slot][0][o] = H.hk_h[g0 + o];
        tk[slot][1][o] = H.hk_f[g0 + o];
        tk[slot][2][o] = H.hk_vm[g0 + o];
        ttp[slot][o] = H.hk_tp[g0 + o];
      }
    }
  }
  for (uint32_t t = tid; t < 4 * nr; t += blockDim.x) {
    const uint32_t slot = t / (2 * nr), f = (t / nr) & 1, r = t % nr;
    if (h0 + slot < H.H) {
      const uint32_t* d = H.V.rdir[1 + f] + (uint64_t)r * H.V.nbp1 + H.ids[h0 + slot];
      sl[slot][f * 2 * kMaxRuns + r] = d[0];
      sl[slot][f * 2 * kMaxRuns + kMaxRuns + r] = d[1] - d[0];
    }
  }
  __syncthreads();
  if (tid < 4 && nr) {  // lengths -> exclusive prefix
    uint32_t* len = &sl[tid >> 1][(tid & 1) * 2 * kMaxRuns + kMaxRuns];
    uint32_t acc = 0;
    for (uint32_t r = 0; r < nr; ++r) {
      const uint32_t l = len[r];
      len[r] = acc;
      acc += l;
    }
  }
  __syncthreads();
  uint32_t h = h0;
  for (uint32_t it = 0; it < kTagChunk / 256; ++it) {
    const uint64_t j = j0 + it * 256 + tid;
    if (j >= H.n_children) break;
    while (h + 1 < H.H && H.c_off[h + 1] <= j) ++h;
    const uint32_t b = H.ids[h];
    const uint32_t i = (uint32_t)(j - H.c_off[h]), N = A.ncnt[b];
    const bool isn = i < N;
    uint32_t row;
    if (nr && h - h0 < 2) {
      const uint32_t k = isn ? i : i - N, *fs = &sl[h - h0][isn ? 0 : 2 * kMaxRuns];
      uint32_t r = 0;
      while (r + 1 < nr && fs[kMaxRuns + r + 1] <= k) ++r;
      row = fs[r] + (k - fs[kMaxRuns + r]);
    } else {
      row = hot_row(A, H, b, i, N);
    }
    HotKeyTab T;
    if (H.small_keys && h - h0 < 2) {
      const uint32_t slot = h - h0;
      T.kh = tk[slot][0];
      T.kf = tk[slot][1];
      T.vm = tk[slot][2];
      T.tp = ttp[slot];
    } else {
      T = hot_key_tab(H, H.hk_off[h]);
    }
    bool mk = false;
    H.w[j] = hot_tag_row(A, H, h, j, isn, hot_fields(A, H, isn, row), T, H.hk_kout[h], orph, &mk);
    if (H.direct) {
      H.v[j] = row | (isn ? 0u : kMemberBit) | (mk ? kInlineMarker : 0u);
    } else {
      H.v[j] = (uint32_t)j | (mk ? kInlineMarker : 0u);
      H.c_h[j] = h | (isn ? 0u : 0x80000000u);
    }
  }
  if (orph && !H.orphans_counted) atomicAdd(&stat_shard(A.stats)[ST_ORPHANS], orph);
}

// One child of a W-run, by flat index j (the last tie-break).
struct HotChild {
  uint64_t id1, id2, t, meta;
  uint32_t j;
};
// A child's fold fields (id1, id2) and (t, meta): its 32-B record, or (direct) its row.
__device__ __forceinline__ void hot_rec(const BucketArgs& A, const HotArgs& H, uint32_t j, ulonglong2& a,
                                        ulonglong2& c) {
  if (!H.direct) {
    a = H.rec[2 * (uint64_t)j];
    c = H.rec[2 * (uint64_t)j + 1];
    return;
  }
  const bool isn = !(j & kMemberBit);
  const uint32_t row = j & (kMemberBit - 1);
  if (H.runs) {
    const uint64_t* const* col = isn ? H.V.nin : H.V.min;
    const uint32_t st = isn ? H.V.ns : H.V.ms;
    if (st > 1) {  // records: pkf id1 id2 t meta
      const uint64_t* r = col[1] + (uint64_t)row * st;
      a = make_ulonglong2(r[1], r[2]);
      c = make_ulonglong2(r[3], r[4]);
    } else {
      a = make_ulonglong2(col[C_ID1][row], col[C_ID2][row]);
      c = make_ulonglong2(col[C_T][row], col[C_META][row]);
    }
  } else {
    const ulonglong2* r = (const ulonglong2*)((isn ? A.nr : A.mr) + (uint64_t)row * kChildStride);
    a = r[1];
    c = r[2];
  }
}
__device__ __forceinline__ HotChild hot_child(const BucketArgs& A, const HotArgs& H, uint32_t j) {
  ulonglong2 a, b;
  hot_rec(A, H, j, a, b);
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
  if (a.id1 != b.id1) return child_order(a.id1) < child_order(b.id1);
  if (!isn && a.id2 != b.id2) return a.id2 < b.id2;
  const uint64_t oa = meta_order(a.meta), ob = meta_order(b.meta);
  if (oa != ob) return oa < ob;
  return a.j < b.j;
}

// Does sorted position p start a run?
__device__ __forceinline__ bool hot_run_start(const HotArgs& H, uint64_t p) {
  const uint64_t W = H.w[p];
  // a run: equal W but the pos bits, from its first row that takes part (a bucket's marker never
  // starts one; one before W belongs to an earlier bucket, so it never hides a start either;
  // inline markers sit inside runs)
  bool start = H.flagged ? hot_row_part(W, H.v[p]) : hot_takes_part(W);
  if (!H.flagged) start = start && !(p > 0 && (H.w[p - 1] >> 6) == (W >> 6));
  for (uint64_t q = p; H.flagged && start && q > 0;) {
    --q;
    const uint64_t X = H.w[q];
    if ((X >> 6) != (W >> 6)) break;
    if (hot_row_part(X, H.v[q])) start = false;
  }
  return start;
}
// hot_run_start for the wave's 64 consecutive positions p (lane order; inb: p is a position): in
// flagged mode the nearest earlier row that takes part, when the wave holds one, decides by its key
// alone (sorted W: an equal key means p is not the first, a smaller one that it is); only a wave's
// first such row scans back through memory.
__device__ __forceinline__ bool hot_run_start_wave(const HotArgs& H, uint64_t p, bool inb, int lane) {
  if (!H.flagged) return inb && hot_run_start(H, p);
  const uint64_t W = inb ? H.w[p] : 0;
  const bool part = inb && hot_row_part(W, H.v[p]);
  const uint64_t below = __ballot(part) & ((1ull << lane) - 1);
  const int src = below ? 63 - __builtin_clzll(below) : lane;
  const uint32_t klo = (uint32_t)__shfl((int)(uint32_t)(W >> 6), src, 64);
  const uint32_t khi = (uint32_t)__shfl((int)(uint32_t)(W >> 38), src, 64);
  if (!part) return false;
  if (below) return (((uint64_t)khi << 32) | klo) != (W >> 6);
  return hot_run_start(H, p);
}
// Run starts -> run list, in two passes over tiles of kRunTile sorted positions (one workgroup of
// 256 each): count each tile's starts, scan the counts, then write each tile's starts at its
// offset in position order. (Replaces a flag per position and a scan over all of them: 24 B per
// child read instead of 36 B read and written.)
constexpr uint32_t kRunTile = 4096;
__global__ void __launch_bounds__(256) hot_runcount_kernel(HotArgs H, uint32_t* __restrict__ tile_n) {
  __shared__ uint32_t tot;
  if (threadIdx.x == 0) tot = 0;
  __syncthreads();
  const uint64_t p0 = (uint64_t)blockIdx.x * kRunTile;
  const uint64_t p1 = min<uint64_t>(p0 + kRunTile, H.n_children);
  uint32_t n = 0;  // (wave-uniform)
  for (uint64_t p = p0 + threadIdx.x; p - threadIdx.x < p1; p += 256)
    n += (uint32_t)__popcll(__ballot(hot_run_start_wave(H, p, p < p1, (int)(threadIdx.x & 63))));
  if ((threadIdx.x & 63) == 0) atomicAdd(&tot, n);
  __syncthreads();
  if (threadIdx.x == 0) tile_n[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(256) hot_runlist_kernel(HotArgs H, const uint32_t* __restrict__ tile_off) {
  __shared__ uint32_t wn[2][4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t p0 = (uint64_t)blockIdx.x * kRunTile;
  const uint64_t p1 = min<uint64_t>(p0 + kRunTile, H.n_children);
  uint32_t base = tile_off[blockIdx.x];
  int par = 0;
  for (uint64_t p = p0 + threadIdx.x; p - threadIdx.x < p1; p += 256, par ^= 1) {
    const bool s = hot_run_start_wave(H, p, p < p1, lane);
    const uint64_t m = __ballot(s);
    if (lane == 0) wn[par][wv] = (uint32_t)__popcll(m);
    __syncthreads();  // (two count buffers: the next round writes the other one)
    uint32_t before = 0, all = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t c = wn[par][k];
      before += k < wv ? c : 0u;
      all += c;
    }
    if (s) H.run_list[base + before + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint32_t)p;
    base += all;
  }
}
__global__ void __launch_bounds__(256) hot_runlist_kernel(HotArgs H, const uint32_t* __restrict__ flag,
                                                          const uint32_t* __restrict__ idx) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < H.n_children;
       p += (uint64_t)gridDim.x * blockDim.x)
    if (flag[p]) H.run_list[idx[p]] = (uint32_t)p;
}
// The first run of every bucket: the first run start at or after the bucket's first position.
__global__ void __launch_bounds__(256) hot_first_run_kernel(HotArgs H) {
  const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H.H) return;
  const uint32_t x = H.c_off[h];
  uint32_t lo = 0, hi = (uint32_t)*H.run_count;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (H.run_list[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  H.first_run[h] = lo;
}

// ---- The chip-wide sort as a merge of sorted lists. Every merge tier writes a key's children in
// child_order (common.h), so in a merge result -- and so in a position-0 state, or a snapshot this
// engine encoded from one and decoded again -- bucket h's flat children are 2 nr lists (the node
// runs, then the member runs: hot_row's order) that are each non-decreasing in W: the key id G
// follows the run's key-hash order and the id bits are a prefix of child_order(id1). A child that
// takes no part keeps the W it would have (inline_markers) and is flagged in v instead, so it stays
// in place in its sorted list; after the merge it sits inside its W-run, where run detection and
// the fold skip it. The sort is then log2(L) rounds of stable pairwise merges of
// neighbouring lists (L = 2 nr rounded up to a power of two; on equal W the lower list first,
// i.e. flat order -- what the stable radix sort keeps), each one read and one write of the
// (W, child) pairs instead of the radix sort's six passes and their histograms. Round 0 verifies
// that every list is sorted; an input that is not (a reference snapshot's HashMap order, or a
// producer that is not a merge) sets *unsorted and the caller re-tags and radix-sorts.
constexpr uint32_t kMergeItems = 8;
constexpr uint32_t kMergeTile = 256 * kMergeItems;  // outputs per workgroup tile

// List bounds of every bucket: bounds[h * (L + 1) + l] = flat start of list l (l < 2 nr: family
// l / nr, run l % nr), padding lists empty, bounds[h * (L + 1) + L] = the bucket's end. Lists that
// do not tile the bucket's flat children exactly (its copied rows laid out otherwise than the run
// directory says) set *unsorted: the batch takes the radix sort, which needs no lists.
__global__ void __launch_bounds__(256) hot_lists_kernel(HotArgs H, uint32_t L, uint32_t* __restrict__ bounds,
                                                        uint32_t* __restrict__ unsorted) {
  const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H.H) return;
  const uint32_t b = H.ids[h], nr = H.V.nr;
  uint32_t* o = bounds + (uint64_t)h * (L + 1);
  uint32_t x = H.c_off[h];
  for (uint32_t f = 0; f < 2; ++f)
    for (uint32_t r = 0; r < nr; ++r) {
      o[f * nr + r] = x;
      const uint32_t* d = H.V.rdir[1 + f] + (uint64_t)r * H.V.nbp1 + b;
      x += d[1] - d[0];
    }
  for (uint32_t l = 2 * nr; l <= L; ++l) o[l] = x;
  if (x != H.c_off[h + 1]) atomicOr(unsorted, 1u);
}

// A cheap early look at whether the lists are sorted, before anything is tagged: 256 sampled pairs
// of neighbouring children of one list, tagged here (the tag kernel rewrites the same records) and
// compared. An input whose children are not in child order (a reference snapshot's HashMap order)
// fails here at once and goes straight to the radix sort; a pass is no proof -- the merge's round
// 0 checks every element.
__global__ void __launch_bounds__(256) hot_sample_kernel(BucketArgs A, HotArgs H, uint32_t L,
                                                         const uint32_t* __restrict__ bounds, uint32_t* unsorted) {
  if (H.n_children < 2) return;
  const uint64_t j = 1 + mix64(0x51ED27A3C4B1F00Dull + threadIdx.x) % (H.n_children - 1);
  const uint32_t h = hot_bucket_of(H, j);
  const uint32_t* o = bounds + (uint64_t)h * (L + 1);
  bool first = false;  // j opens its list: no pair
  for (uint32_t l = 0; l <= L; ++l) first |= o[l] == j;
  if (first || j <= H.c_off[h]) return;
  unsigned long long orph = 0;
  const uint32_t b = H.ids[h], N = A.ncnt[b];
  uint64_t w[2];
  for (int k = 0; k < 2; ++k) {
    const uint64_t x = j - 1 + k;
    const uint32_t i = (uint32_t)(x - H.c_off[h]);
    const bool isn = i < N;
    bool mk = false;
    w[k] = hot_tag_row(A, H, h, x, isn, hot_fields(A, H, isn, hot_row(A, H, b, i, N)), hot_key_tab(H, H.hk_off[h]),
                       H.hk_kout[h], orph, &mk);
  }
  if (w[1] < w[0]) atomicOr(unsorted, 1u);
}

struct MergeArgs {
  const uint32_t* bounds;    // hot_lists_kernel
  uint32_t L, span;          // this round merges list groups [2 span m, 2 span m + span) and [.. + span, 2 span (m + 1))
  uint32_t n_jobs;           // H * L / (2 span): job J = bucket J / (L / 2 span), pair J % (L / 2 span)
  uint32_t* tiles;           // per job: its tiles, then (scanned) its first tile
  const uint64_t* n_tiles;   // total tiles (device)
  const uint64_t* wi;
  const uint32_t* vi;
  uint64_t* wo;
  uint32_t* vo;
  uint32_t* unsorted;        // check: a list decreases somewhere
  int check;
};
__device__ __forceinline__ void merge_job(const MergeArgs& M, uint32_t J, uint32_t& a0, uint32_t& a1, uint32_t& b1) {
  const uint32_t per = M.L / (2 * M.span), h = J / per, m = J % per;
  const uint32_t* o = M.bounds + (uint64_t)h * (M.L + 1) + 2 * M.span * m;
  a0 = o[0];
  a1 = o[M.span];
  b1 = o[2 * M.span];
}
__global__ void __launch_bounds__(256) hot_merge_count_kernel(MergeArgs M) {
  const uint32_t J = blockIdx.x * blockDim.x + threadIdx.x;
  if (J >= M.n_jobs) return;
  uint32_t a0, a1, b1;
  merge_job(M, J, a0, a1, b1);
  M.tiles[J] = (b1 - a0 + kMergeTile - 1) / kMergeTile;
}
// A's elements before output position d of the stable merge of A[0, na) and B[0, nb) (A first on
// equal keys).
template <class KA, class KB>
__device__ __forceinline__ uint32_t merge_path(KA a, uint32_t na, KB bk, uint32_t nb, uint32_t d) {
  uint32_t lo = d > nb ? d - nb : 0, hi = min(d, na);
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a(mid) <= bk(d - 1 - mid)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// Each tile's job and its first A element (merge path at the tile's first output), one thread per
// tile, so that the merge's workgroups start with their split in hand instead of a chain of global
// loads.
__global__ void __launch_bounds__(256) hot_merge_split_kernel(MergeArgs M, uint2* __restrict__ split) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= *M.n_tiles) return;
  uint32_t lo = 0, hi = M.n_jobs;  // the last job whose first tile is at or before t
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (M.tiles[mid] <= t) lo = mid;
    else hi = mid;
  }
  const uint32_t J = lo;
  uint32_t a0, a1, b1;
  merge_job(M, J, a0, a1, b1);
  const uint64_t* A = M.wi + a0;
  const uint64_t* B = M.wi + a1;
  const uint32_t d0 = (uint32_t)(t - M.tiles[J]) * kMergeTile;
  split[t] = make_uint2(merge_path([&](uint32_t i) { return A[i]; }, a1 - a0, [&](uint32_t i) { return B[i]; },
                                   b1 - a1, d0), J);
}
// One tile of kMergeTile outputs per workgroup: the tile's two input slices (from its split and
// the next tile's) are staged in LDS with coalesced loads, and each thread merges kMergeItems
// outputs from LDS.
__global__ void __launch_bounds__(256) hot_merge_kernel(MergeArgs M, const uint2* __restrict__ split) {
  __shared__ uint64_t sw[kMergeTile];
  __shared__ uint32_t sv[kMergeTile];
  const uint32_t tid = threadIdx.x;
  const uint64_t nt = *M.n_tiles;
  const uint64_t t = blockIdx.x;
  if (t >= nt) return;
  const uint2 sp = split[t];
  const uint32_t J = sp.y;
  uint32_t a0, a1, b1;
  merge_job(M, J, a0, a1, b1);
  const uint32_t na = a1 - a0, nb = b1 - a1;
  const uint32_t d0 = (uint32_t)(t - M.tiles[J]) * kMergeTile, d1 = min(d0 + kMergeTile, na + nb);
  uint32_t ia1 = na;  // (the job's last tile ends at the job's end)
  if (t + 1 < nt) {
    const uint2 nx = split[t + 1];
    if (nx.y == J) ia1 = nx.x;
  }
  const uint32_t ia0 = sp.x, ib0 = d0 - ia0, ib1 = d1 - ia1;
  const uint32_t la = ia1 - ia0, lb = ib1 - ib0;
  const uint64_t* A = M.wi + a0;
  const uint64_t* B = M.wi + a1;
  for (uint32_t x = tid; x < la + lb; x += blockDim.x) {
    const uint32_t src = x < la ? a0 + ia0 + x : a1 + ib0 + (x - la);
    sw[x] = M.wi[src];
    sv[x] = M.vi[src];
  }
  __syncthreads();
  if (M.check) {  // every element against its list predecessor (the first one's from global memory)
    bool bad = false;
    for (uint32_t x = tid; x < la + lb; x += blockDim.x) {
      const bool ina = x < la;
      const uint32_t k = ina ? ia0 + x : ib0 + (x - la);  // index inside its list
      if (k == 0) continue;
      const uint64_t prev = (x != 0 && x != la) ? sw[x - 1] : (ina ? A[k - 1] : B[k - 1]);
      bad |= sw[x] < prev;
    }
    if (__ballot(bad) && (tid & 63) == 0) atomicOr(M.unsorted, 1u);
  }
  // each thread merges its kMergeItems outputs into registers, then they go back through LDS so
  // that the global stores are coalesced
  const uint32_t d = tid * kMergeItems, n = la + lb;
  uint64_t ow[kMergeItems];
  uint32_t ov[kMergeItems];
  if (d < n) {
    uint32_t i = merge_path([&](uint32_t k) { return sw[k]; }, la, [&](uint32_t k) { return sw[la + k]; }, lb, d);
    uint32_t j = d - i;
#pragma unroll
    for (uint32_t q = 0; q < kMergeItems; ++q) {
      const bool takea = j >= lb || (i < la && sw[i] <= sw[la + j]);
      const uint32_t x = takea ? i : la + j;
      ow[q] = sw[x];
      ov[q] = sv[x];
      i += takea ? 1 : 0;
      j += takea ? 0 : 1;
    }
  }
  __syncthreads();
  if (d < n) {
#pragma unroll
    for (uint32_t q = 0; q < kMergeItems; ++q) {
      if (d + q < n) {
        sw[d + q] = ow[q];
        sv[d + q] = ov[q];
      }
    }
  }
  __syncthreads();
  for (uint32_t x = tid; x < n; x += blockDim.x) {
    M.wo[a0 + d0 + x] = sw[x];
    M.vo[a0 + d0 + x] = sv[x];
  }
}

constexpr uint32_t kFoldFast = 8;  // runs up to this many rows: rows in registers, loads overlapped

// One run's contribution to its key's row: outputs, first output slot, counter sum.
struct HotAcc {
  uint32_t nout = 0, k_cnt = 0, k_cb = kNone;
  unsigned long long k_sum = 0;
};

// The fold of one W-run: its rows k = 0 .. nrows - 1 in sorted order, flat index jat(k), key G,
// bucket b. Pass 0 counts the run's outputs (acc.nout) and, for a run of one exact id whose rows
// arrive in strictly increasing (pos, src) order (the tag's low bits are the position) and no
// longer than kFoldFast, keeps the fold: *fq = the output row's k (members: the winner; nodes: the
// head), *fv = a counter node's folded value; *fq = kNone sends the run to the selection path.
// Pass 1 (emitted: pass 0 counted outputs) writes the outputs at rows obase.. of the bucket's
// family and sums them into acc. Other runs (ids sharing the tag's id-hash bits, and long runs)
// fold by successor selection in both passes: each step selects the successor of the last visited
// row (O(run^2) over rows in L2, no per-thread arrays), so rows are folded in order whatever order
// the sort left them in. Every lane of the wave calls this (act false for idle lanes): loops have
// wave-uniform trip counts with per-lane predicates -- a loop-carried row must not be a live-out
// of a loop with divergent exits (gfx950 compilers have produced the first candidate instead of
// the smallest there). Rows k with !part(k) take no part (inline markers, after the run's first
// row): they are skipped.
template <class JAt, class Part>
__device__ __forceinline__ void hot_fold_run(const BucketArgs& A, const HotArgs& H, int pass, bool act, bool isn,
                                             uint32_t b, uint32_t G, uint32_t nrows, JAt jat, Part part, uint64_t obase,
                                             bool emitted, uint32_t* fq, uint64_t* fv, ulonglong2* fs, HotAcc& acc,
                                             unsigned long long& gcm, unsigned long long& nslow) {
  auto put = [&](uint64_t id1, uint64_t id2, uint64_t t, uint64_t meta, uint64_t v) {
    const uint32_t o = (uint32_t)(obase + acc.nout);
    // (one whole 48-B row as three 16-B stores: pkh pkf | id1 id2 | t meta)
    ulonglong2* row = (ulonglong2*)(isn ? A.nos + (uint64_t)(A.nbase[b] + o) * kChildStride
                                        : A.mos + (uint64_t)(A.mbase[b] + o) * kChildStride);
    row[0] = make_ulonglong2(H.hk_h[G], H.hk_f[G]);
    row[1] = make_ulonglong2(id1, isn ? v : id2);
    row[2] = make_ulonglong2(t, isn ? meta_pack(0, meta_pos(meta), meta_src(meta)) : meta);
    acc.k_cb = min(acc.k_cb, o);
    ++acc.k_cnt;
    acc.k_sum += isn ? v : 0;
  };
  auto emit_id = [&](const HotChild& hd, uint64_t v, uint64_t tw, uint64_t wmeta) {
    if (!isn && (A.flags & F_GC_MEMBERS) && meta_tag(wmeta) == KIND_DEL && tw < A.gc_wm) {
      ++gcm;
      return;
    }
    if (pass == 1) put(hd.id1, hd.id2, isn ? hd.t : tw, isn ? hd.meta : wmeta, v);
    ++acc.nout;
  };
  bool slow = act;
  if (pass == 0) {
    // fast path: up to kFoldFast rows, their loads issued together
    const bool fast = act && nrows <= kFoldFast;
    uint32_t rj[kFoldFast];
    bool pk[kFoldFast];
#pragma unroll
    for (uint32_t k = 0; k < kFoldFast; ++k) {
      pk[k] = fast && k < nrows && (k == 0 || part(k));
      rj[k] = pk[k] ? jat(k) : 0;
    }
    uint64_t xi1[kFoldFast], xi2[kFoldFast], xt[kFoldFast], xm[kFoldFast];
#pragma unroll
    for (uint32_t k = 0; k < kFoldFast; ++k) {
      if (pk[k]) {
        ulonglong2 a, c;
        hot_rec(A, H, rj[k], a, c);
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
    uint64_t last_order = meta_order(xm[0]);
    uint32_t qw = 0;  // winner (members)
#pragma unroll
    for (uint32_t k = 1; k < kFoldFast; ++k) {
      if (pk[k]) {
        simple = simple && xi1[k] == xi1[0] && (isn || xi2[k] == xi2[0]) && meta_order(xm[k]) > last_order;
        last_order = meta_order(xm[k]);
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
      *fq = isn ? 0u : qw;
      if (fs) {  // the output row's fields (nodes: the head row, the folded value; members: the winner)
        uint64_t i2 = xi2[0], i1 = xi1[0];
#pragma unroll
        for (uint32_t k = 1; k < kFoldFast; ++k) {
          i1 = (k == qw) ? xi1[k] : i1;
          i2 = (k == qw) ? xi2[k] : i2;
        }
        fs[0] = make_ulonglong2(isn ? xi1[0] : i1, isn ? v : i2);
        fs[1] = make_ulonglong2(isn ? xt[0] : tw, isn ? xm[0] : wm);
      } else {
        *fv = v;
      }
      slow = false;
    } else if (act) {
      *fq = kNone;
    }
  } else if (act) {  // pass 1, fold kept by pass 0
    const uint32_t q = *fq;
    if (q != kNone) {
      slow = false;
      if (emitted && fs) {
        const ulonglong2 a = fs[0], c = fs[1];
        put(a.x, a.y, c.x, c.y, a.y);
      } else if (emitted) {
        const HotChild x = hot_child(A, H, jat(q));
        put(x.id1, x.id2, x.t, x.meta, *fv);
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
      if (slow && k < nrows && step < nrows && (k == 0 || part(k))) {
        const HotChild x = hot_child(A, H, jat(k));
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
}

// One thread per W-run of the global sort (a (key, child id) group, ~ one row per replica): pass
// 0 counts (emit_n / emit_m at the run's index), pass 1 writes at the run's rank in its
// bucket (after scans of the counts) and adds the run to its key row.
__global__ void __launch_bounds__(256) hot_fold_kernel(BucketArgs A, HotArgs H, int pass) {
  unsigned long long gcm = 0, nslow = 0;
  const uint64_t nruns = *H.run_count;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < nruns; base += stride) {  // wave-uniform
    const uint64_t i = base + threadIdx.x;
    const bool act = i < nruns;
    // pass 1: a run pass 0 folded (fold_q != kNone) is written from the stash alone; the others
    // (the selection path) find their rows again
    const bool kept = act && pass == 1 && H.fold_q[i] != kNone;
    const bool rows = act && !kept;
    const uint64_t p = rows ? H.run_list[i] : 0;
    uint64_t W = 0;
    uint32_t nrows = 0, hc = 0, G = 0;
    if (rows) {
      W = H.w[p];
      uint64_t e = p + 1;  // (inline markers inside the run are rows of it; the fold skips them)
      while (e < H.n_children && (H.w[e] >> 6) == (W >> 6) && hot_takes_part(H.w[e])) ++e;
      nrows = (uint32_t)(e - p);
      G = (uint32_t)(W >> H.g_shift);
      if (H.direct)
        hc = H.hk_bkt[G] | ((H.v[p] & kMemberBit) ? 0x80000000u : 0u);
      else
        hc = H.c_h[H.v[p] & ~kInlineMarker];
    } else if (kept) {
      const uint2 hg = H.fold_hg[i];
      hc = hg.x;
      G = hg.y;
    }
    uint32_t h = 0, b = 0;
    bool isn = false;
    uint64_t obase = 0;
    if (act) {
      h = hc & 0x7FFFFFFFu;
      isn = (hc >> 31) == 0;
      b = H.ids[h];
      if (pass == 0) H.fold_hg[i] = make_uint2(hc, G);
      if (pass == 1) {
        const uint32_t f = H.first_run[h];
        obase = isn ? H.rank_n[i] - H.rank_n[f] : H.rank_m[i] - H.rank_m[f];
      }
    }
    const bool emitted = act && pass == 1 && (isn ? H.emit_n : H.emit_m)[i] != 0;
    HotAcc acc;
    hot_fold_run(A, H, pass, act, isn, b, G, nrows, [&](uint32_t k) { return H.v[p + k] & ~kInlineMarker; },
                 [&](uint32_t k) { return !(H.v[p + k] & kInlineMarker); }, obase, emitted,
                 &H.fold_q[i], &H.fold_v[i], H.fold_rec + 2 * i, acc, gcm, nslow);
    if (pass == 0 && act) {
      H.emit_n[i] = isn ? acc.nout : 0;
      H.emit_m[i] = isn ? 0 : acc.nout;
    }
    if (pass == 1) {
      // runs are in sorted order, so the wave's active lanes hold non-decreasing keys G:
      // a segmented reduction per key, and the segment's last lane does the atomics (one per key
      // and wave, not per output: a hot key owns up to millions of them)
      const uint32_t key = act ? G : kNone;  // inactive lanes only at the tail: segments are contiguous
      uint32_t k_cnt = acc.k_cnt, k_cb = acc.k_cb;
      unsigned long long k_sum = acc.k_sum;
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

// ---- Run-order batches of buckets of at most kSortCap children: one workgroup per bucket does the
// whole child path in LDS (hot_sortfold_kernel) instead of the global tag sort and its scans. The
// tag of a child is key32 = W >> 6 less the bucket's first key id: (G - hk_off[h]) << id_bits | id
// bits (G - hk_off[h] < kCapK = 2^10, id_bits <= kSortIdBits, so it fits 32 bits; the bucket's
// marker is the largest, (K << id_bits) - 1). A stable LDS radix sort of (key32, flat index) is
// then the global sort's permutation restricted to the bucket (the global one sorts W's bits from
// 6 on and keeps buckets apart), so runs, their fold order and the outputs' order are the ones
// the global path gives for the same id_bits. Runs are folded by hot_fold_run, ranked by a
// workgroup scan, and the key rows finished from LDS accumulators.
constexpr uint32_t kSortCap = 8192;
constexpr int kSortIdBits = 22;
// Two shapes: buckets of at most 8192 children (1024 threads, one workgroup per CU), and buckets
// of at most 2048 children and 256 keys (256 threads, four workgroups per CU).
template <uint32_t CAP, int THREADS, uint32_t KCAP>
struct SortCfg {
  static constexpr uint32_t Cap = CAP, KCap = KCAP;
  static constexpr int Threads = THREADS, Waves = THREADS / 64, It = CAP / THREADS;
};
using SortBig = SortCfg<kSortCap, 1024, kCapK>;
using SortSmall = SortCfg<2048, 256, 256>;

template <class C>
struct SortLds {
  uint32_t key[2][C::Cap];          // key32 (ping-pong); after the sort: run list, then run offsets
  uint16_t ix[2][C::Cap];           // flat index - c_off[h] (ping-pong); then outputs per run
  uint16_t wc[C::Waves][256];       // a tile's digit counts per wave, then their prefixes
  uint32_t dbase[256];              // wave totals of the digit scan
  uint32_t kcnt[C::KCap], kcb[C::KCap];  // per output key: children out, first child slot
  unsigned long long ksum[C::KCap];      // per output key: counter sum
  uint64_t tab[3 * C::KCap];        // the bucket's output keys: kh, kf, vm
  uint32_t ttp[C::KCap];            // ... and tag / pos words
  uint32_t sl[4 * kMaxRuns];        // [family][run]: first row, rows before the run
  uint32_t wsum[C::Waves];
  uint32_t misc[8];                 // AND / OR of the keys, first marker position, totals
};

// Exclusive scan of one value per thread over the workgroup (total in *total).
template <int WAVES>
__device__ __forceinline__ uint32_t sort_block_scan(uint32_t x, uint32_t* wsum, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)inc, d);
    if (lane >= (uint32_t)d) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < WAVES; ++k) {
    const uint32_t v = wsum[k];
    pre += (uint32_t)k < wv ? v : 0;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return pre + inc - x;
}

// One stable pass of the LDS radix sort on key bits [sh, sh + 8): key[s] / ix[s] -> key[s ^ 1] /
// ix[s ^ 1]. Wave w ranks the consecutive chunk w of the elements, 64 at a time with ballots, in
// its own digit counters; one scan over (digit, wave) then places every wave's run of each digit.
template <class C>
__device__ __forceinline__ void sort_pass(SortLds<C>& L, int s, int sh, uint32_t n) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint16_t* wcf = &L.wc[0][0];
  for (uint32_t k = tid; k < C::Waves * 256; k += C::Threads) wcf[k] = 0;
  __syncthreads();
  const uint32_t chunk = (n + C::Waves * 64 - 1) / (C::Waves * 64) * 64;  // per wave, whole sub-tiles
  const uint32_t base = wv * chunk;
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t kk[C::It], rr[C::It];
  uint16_t xx[C::It];
#pragma unroll
  for (int it = 0; it < C::It; ++it) {
    kk[it] = rr[it] = 0;
    xx[it] = 0;
    if ((uint32_t)it * 64 < chunk) {  // (uniform)
      const uint32_t i = base + it * 64 + lane;
      const bool valid = i < n;
      const uint32_t key = valid ? L.key[s][i] : 0;
      xx[it] = valid ? L.ix[s][i] : 0;
      kk[it] = key;
      const uint32_t d = (key >> sh) & 255;
      uint64_t peers = __ballot(valid);  // the wave's valid lanes with this lane's digit
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const uint64_t bb = __ballot((d >> bit) & 1);
        peers &= ((d >> bit) & 1) ? bb : ~bb;
      }
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      const uint32_t cur = L.wc[wv][d];  // (one wave's LDS accesses stay in order)
      rr[it] = cur + below;
      if (valid && below == 0) L.wc[wv][d] = (uint16_t)(cur + __popcll(peers));
    }
  }
  __syncthreads();
  // digit d: prefix over the waves, then the digits' totals scanned (wave totals in dbase[0..3])
  uint32_t tot = 0, inc = 0;
  if (tid < 256) {
#pragma unroll
    for (int w = 0; w < C::Waves; ++w) {
      const uint32_t c = L.wc[w][tid];
      L.wc[w][tid] = (uint16_t)tot;
      tot += c;
    }
    inc = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, d);
      if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) L.dbase[wv] = inc;
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t dbase = inc - tot;
    for (uint32_t k = 0; k < wv; ++k) dbase += L.dbase[k];
#pragma unroll
    for (int w = 0; w < C::Waves; ++w) L.wc[w][tid] = (uint16_t)(L.wc[w][tid] + dbase);
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < C::It; ++it) {
    const uint32_t i = base + it * 64 + lane;
    if ((uint32_t)it * 64 < chunk && i < n) {
      const uint32_t dst = L.wc[wv][(kk[it] >> sh) & 255] + rr[it];
      L.key[s ^ 1][dst] = kk[it];
      L.ix[s ^ 1][dst] = xx[it];
    }
  }
  __syncthreads();
}

template <class C>
__global__ void __launch_bounds__(C::Threads) hot_sortfold_kernel(BucketArgs A, HotArgs H, int id_bits) {
  __shared__ SortLds<C> L;
  const uint32_t h = blockIdx.x, b = H.ids[h], tid = threadIdx.x;
  const uint32_t c0 = H.c_off[h], n = H.c_off[h + 1] - c0, g0 = H.hk_off[h];
  const uint32_t K = H.hk_off[h + 1] - g0, kout = H.hk_kout[h], N = A.ncnt[b];
  const uint32_t mk = (K << id_bits) - 1;  // the marker's key32
  unsigned long long orph = 0, gcm = 0, nslow = 0;
  uint64_t clk = H.prof ? wall_clock64() : 0;
  auto phase = [&](int i) {  // (after a barrier)
    if (H.prof && tid == 0) {
      const uint64_t now = wall_clock64();
      atomicAdd(&H.prof[i], (unsigned long long)(now - clk));
      clk = now;
    }
  };
  for (uint32_t o = tid; o < kout; o += C::Threads) {
    L.kcnt[o] = 0;
    L.kcb[o] = kNone;
    L.ksum[o] = H.hk_sum[g0 + o];
  }
  if (tid == 0) {
    L.misc[0] = ~0u;  // AND of the keys
    L.misc[1] = 0;    // OR of the keys
    L.misc[2] = n;    // first marker position after the sort
    L.misc[3] = L.misc[4] = 0;
  }
  // the bucket's key table and run slices
  HotKeyTab T;
  T.kh = L.tab;
  T.kf = L.tab + C::KCap;
  T.vm = L.tab + 2 * C::KCap;
  T.tp = L.ttp;
  for (uint32_t o = tid; o < kout; o += C::Threads) {
    L.tab[o] = H.hk_h[g0 + o];
    L.tab[C::KCap + o] = H.hk_f[g0 + o];
    L.tab[2 * C::KCap + o] = H.hk_vm[g0 + o];
    L.ttp[o] = H.hk_tp[g0 + o];
  }
  uint32_t* sl = L.sl;  // [family 0/1][run]: first row, then rows before the run
  const uint32_t nr = H.runs ? H.V.nr : 0;
  if (tid < 2 * nr) {
    const uint32_t f = tid / nr, r = tid % nr;
    const uint32_t* d = H.V.rdir[1 + f] + (uint64_t)r * H.V.nbp1 + b;
    sl[f * 2 * kMaxRuns + r] = d[0];
    sl[f * 2 * kMaxRuns + kMaxRuns + r] = d[1] - d[0];
  }
  __syncthreads();
  if (tid < 2) {  // lengths -> exclusive prefix
    uint32_t acc = 0;
    for (uint32_t r = 0; r < nr; ++r) {
      const uint32_t len = sl[tid * 2 * kMaxRuns + kMaxRuns + r];
      sl[tid * 2 * kMaxRuns + kMaxRuns + r] = acc;
      acc += len;
    }
  }
  __syncthreads();
  // 1. tags (rec[j] written as on the global path)
  uint32_t kand = ~0u, kor = 0;
  auto row_of = [&](uint32_t i) -> uint32_t {
    const bool isn = i < N;
    if (!nr) return hot_row(A, H, b, i, N);
    const uint32_t k = isn ? i : i - N, *fs = sl + (isn ? 0 : 2 * kMaxRuns);
    uint32_t r = 0;
    while (r + 1 < nr && fs[kMaxRuns + r + 1] <= k) ++r;
    return fs[r] + (k - fs[kMaxRuns + r]);
  };
  auto tag = [&](uint32_t i, const HotFields& F) {
    const uint64_t W = hot_tag_row(A, H, h, (uint64_t)c0 + i, i < N, F, T, kout, orph);
    const uint32_t k32 = (uint32_t)((W >> 6) - ((uint64_t)g0 << id_bits));
    L.key[0][i] = k32;
    L.ix[0][i] = (uint16_t)i;
    kand &= k32;
    kor |= k32;
  };
  for (uint32_t i = tid; i < n; i += 2 * C::Threads) {  // two children per step, their loads first
    const uint32_t i2 = i + C::Threads;
    const HotFields F1 = hot_fields(A, H, i < N, row_of(i));
    HotFields F2;
    if (i2 < n) F2 = hot_fields(A, H, i2 < N, row_of(i2));
    tag(i, F1);
    if (i2 < n) tag(i2, F2);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    kand &= (uint32_t)__shfl_xor((int)kand, off);
    kor |= (uint32_t)__shfl_xor((int)kor, off);
  }
  if ((tid & 63) == 0) {
    atomicAnd(&L.misc[0], kand);
    atomicOr(&L.misc[1], kor);
  }
  __syncthreads();
  phase(0);
  // 2. stable LDS radix sort; digits equal in every key are skipped
  const uint32_t vary = L.misc[0] ^ L.misc[1];
  int s = 0;
  for (int sh = 0; sh < 32; sh += 8) {
    if (((vary >> sh) & 255) == 0) continue;
    sort_pass<C>(L, s, sh, n);
    s ^= 1;
  }
  phase(1);
  const uint32_t* sk = L.key[s];
  const uint16_t* sx = L.ix[s];
  // 3. runs (equal key32; markers, sorted last, start none): list in key[s ^ 1] as
  //    start | (G - g0) << 16, in chunks of consecutive positions per thread
  uint32_t* rl = L.key[s ^ 1];
  const uint32_t per = (n + C::Threads - 1) / C::Threads;
  const uint32_t q0 = min(n, tid * per), q1 = min(n, q0 + per);
  uint32_t cnt = 0;
  for (uint32_t q = q0; q < q1; ++q) {
    const uint32_t k = sk[q];
    const bool prev_same = q > 0 && sk[q - 1] == k;
    cnt += (k != mk && !prev_same) ? 1 : 0;
    if (k == mk && !prev_same) L.misc[2] = q;
  }
  uint32_t nruns = 0;
  uint32_t ex = sort_block_scan<C::Waves>(cnt, L.wsum, &nruns);
  for (uint32_t q = q0; q < q1; ++q) {
    const uint32_t k = sk[q];
    if (k != mk && !(q > 0 && sk[q - 1] == k)) rl[ex++] = q | ((k >> id_bits) << 16);
  }
  __syncthreads();
  const uint32_t m = L.misc[2];  // rows taking part
  phase(2);
  // the fold reads a child by its flat index (its 32-B record from the tag pass) or, direct, by its
  // row in the runs / the copied rows (no records written: the rows were just read by the tag pass)
  auto jat_of = [&](uint32_t i) -> uint32_t {
    if (!H.direct) return c0 + i;
    return row_of(i) | (i < N ? 0u : kMemberBit);
  };
  // 4. fold, pass 0: outputs per run into ix[s ^ 1]
  uint16_t* no = L.ix[s ^ 1];
  uint32_t* fq = H.fold_q + c0;
  uint64_t* fv = H.fold_v + c0;
  for (uint32_t base = 0; base < nruns; base += C::Threads) {  // (uniform)
    const uint32_t r = base + tid;
    const bool act = r < nruns;
    const uint32_t e = act ? rl[r] : 0, q = e & 0xFFFF;
    const uint32_t nrows = act ? (r + 1 < nruns ? (rl[r + 1] & 0xFFFF) : m) - q : 0;
    const bool isn = act && sx[q] < N;
    HotAcc acc;
    hot_fold_run(A, H, 0, act, isn, b, g0 + (e >> 16), nrows, [&](uint32_t k) { return jat_of(sx[q + k]); },
                 [](uint32_t) { return true; }, 0,
                 false, fq + r, fv + r, nullptr, acc, gcm, nslow);
    if (act) no[r] = (uint16_t)acc.nout;
  }
  __syncthreads();
  // ranks: one scan of (member outputs << 16 | node outputs) over the runs, into key[s]
  uint32_t* ro = L.key[s];
  const uint32_t pr = (nruns + C::Threads - 1) / C::Threads;
  const uint32_t r0 = min(nruns, tid * pr), r1 = min(nruns, r0 + pr);
  uint32_t c = 0;
  for (uint32_t r = r0; r < r1; ++r) c += sx[rl[r] & 0xFFFF] < N ? (uint32_t)no[r] : (uint32_t)no[r] << 16;
  uint32_t tot = 0;
  ex = sort_block_scan<C::Waves>(c, L.wsum, &tot);
  for (uint32_t r = r0; r < r1; ++r) {
    ro[r] = ex;
    ex += sx[rl[r] & 0xFFFF] < N ? (uint32_t)no[r] : (uint32_t)no[r] << 16;
  }
  __syncthreads();
  phase(3);
  // 5. fold, pass 1: outputs at their rank, their key rows' counts, first slots and sums in LDS
  for (uint32_t base = 0; base < nruns; base += C::Threads) {  // (uniform)
    const uint32_t r = base + tid;
    const bool act = r < nruns;
    const uint32_t e = act ? rl[r] : 0, q = e & 0xFFFF, gr = e >> 16;
    const uint32_t nrows = act ? (r + 1 < nruns ? (rl[r + 1] & 0xFFFF) : m) - q : 0;
    const bool isn = act && sx[q] < N;
    const uint32_t off = act ? ro[r] : 0;
    HotAcc acc;
    hot_fold_run(A, H, 1, act, isn, b, g0 + gr, nrows, [&](uint32_t k) { return jat_of(sx[q + k]); },
                 [](uint32_t) { return true; },
                 isn ? (off & 0xFFFF) : (off >> 16), act && no[r] != 0, fq + r, fv + r, nullptr, acc, gcm, nslow);
    if (act && acc.k_cnt) {
      atomicAdd(&L.kcnt[gr], acc.k_cnt);
      atomicMin(&L.kcb[gr], acc.k_cb);
      if (isn && (H.hk_vm[g0 + gr] & kVmaskMerged)) atomicAdd(&L.ksum[gr], acc.k_sum);
    }
  }
  __syncthreads();
  phase(4);
  // 6. key rows (as hot_finish_kernel)
  const uint32_t kb = A.kbase[b];
  uint32_t nn = 0, nm = 0;
  for (uint32_t o = tid; o < kout; o += C::Threads) {
    const uint32_t tk = H.hk_tp[g0 + o] & 0xFF, kc = L.kcnt[o];
    if (tk == TAG_COUNTER) {
      A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_WIN] = L.ksum[o];
      nn += kc;
    } else if (tk == TAG_SET || tk == TAG_DICT) {
      nm += kc;
    }
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_CREF] = cref_pack(kc ? L.kcb[o] : 0, kc);
  }
  if (nn) atomicAdd(&L.misc[3], nn);
  if (nm) atomicAdd(&L.misc[4], nm);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    orph += __shfl_xor(orph, off);
    gcm += __shfl_xor(gcm, off);
    nslow += __shfl_xor(nslow, off);
  }
  if ((tid & 63) == 0) {
    if (orph) atomicAdd(&stat_shard(A.stats)[ST_ORPHANS], orph);
    if (gcm) atomicAdd(&stat_shard(A.stats)[ST_MEMBERS_GCED], gcm);
    if (nslow) atomicAdd(&stat_shard(A.stats)[ST_HOT_SLOW], nslow);
  }
  __syncthreads();
  if (tid == 0) {
    A.kout[b] = kout;
    A.nout[b] = L.misc[3];
    A.mout[b] = L.misc[4];
  }
  phase(5);
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
