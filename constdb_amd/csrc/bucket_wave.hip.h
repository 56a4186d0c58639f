// Wave-per-bucket merge kernels (gfx950, wave64) — the hot path of the merge.
//
// One 64-lane wave owns one bucket and never synchronises with another wave.
//   0. every global load of the bucket is issued up front: the row indices (the final
//      partition level is index-only), then all key columns and all child columns, so a
//      bucket costs one dependent pair of round trips instead of one pair per family;
//   1. keys: each row gets ONE 64-bit sort word (kh low 44 bits | family | pos | slot); a
//      lane's rank is the number of smaller words (a K-step loop over LDS broadcasts — for
//      ~40 rows cheaper than a bitonic network and proportional to the bucket, not to 64),
//      and rows are scattered to their rank. Words equal in the kh part but different in
//      (kh, kf) (a 2^-44 event per pair) and two rows of one (key, family, pos) (duplicate
//      keys in one snapshot) hand the bucket to the exact-comparator workgroup tier before
//      anything is written, so the order (kh, family, pos, src) is exact here;
//   2. key folds: the tail slot of each (key, family) segment replays the reference's
//      sequential fold over its segment (<= R rows, already in sorted order in LDS):
//        data     DB::merge_entry / Object::merge   (db.rs:31-43, object.rs:63-83)
//        expires / deletes: last (pos, src) wins   (db.rs:68-76), DB::gc (db.rs:82-95);
//   3. children: counter nodes and set/dict members share the slots (a key has one type);
//      each finds its key by binary search over the wave's sorted output keys (LDS), is
//      kept if its element has the key's head type (object.rs:80) and, for members of a
//      non-head position, only if it is an add (SetIter/DictIter, lwwhash.rs:319-323);
//      ranked by one word (key rank | id hash low 42 bits | pos | slot), folded per
//      (key, node) with Counter::merge's head-t rule (type_counter.rs:59-87) or per
//      (key, member) with LWWHash::set's later-wins-ties rule (lwwhash.rs:87-107);
//   4. counter sums (cal_sum, type_counter.rs:89-91) and child ranges; outputs are
//      written by the tail slots (ballot + mbcnt ranks).
// bucket_wave_kernel (KE = 1: 64 key rows, 128 child rows) runs every bucket; one over that
// goes to bucket_wide_kernel (KE = 2: 128 key rows, 256 child rows), and anything beyond
// that, collisions, duplicates and forced tiers go to the workgroup tier (bucket.hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bucket.hip.h"
#include "common.h"

namespace cdb {

constexpr int kWavesPerWG = 4;
// Profiling builds only (-DCDB_WAVE_STOP=n, scripts/wave_phases.sh): stop a bucket after phase n
// and sink what it computed into a spare statistics word, to time the phases of the wave kernel.
#ifndef CDB_WAVE_STOP
#define CDB_WAVE_STOP 99
#endif
constexpr uint64_t kM44 = (1ull << 44) - 1, kM42 = (1ull << 42) - 1;

// Output rows are written once and not read again by this kernel: streaming (non-temporal)
// stores keep them from displacing the input lines neighbouring buckets still read from L2.
#ifndef CDB_NT_OUT
#define CDB_NT_OUT 1
#endif
typedef unsigned long long u64x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_row16(ulonglong2* p, unsigned long long x, unsigned long long y) {
  if (CDB_NT_OUT) {
    u64x2v v = {x, y};
    __builtin_nontemporal_store(v, reinterpret_cast<u64x2v*>(p));
  } else {
    *p = make_ulonglong2(x, y);
  }
}


// Per-wave LDS. KE = key rows per lane (1 or 2); child rows per lane CE = 2 KE.
template <int KE>
struct WaveLds {
  static constexpr int KC = 64 * KE;       // key-row capacity
  static constexpr int CC = 128 * KE;      // child-row capacity
  uint64_t okh[KC], okf[KC], ovm[KC], osum[KC];  // output keys, sorted
  uint32_t otp[KC], ocnt[KC], ocb[KC];
  uint64_t sw[CC + 2];                     // sort words (keys, then children), sorted in place
  union __attribute__((aligned(16))) {     // rows in sorted order (and the load staging area)
    uint64_t col[7][KC];                   // key rows: KS_*
    uint64_t ccol[4][CC];                  // child rows: CS_*
  };
};
enum { KS_KH = 0, KS_KF, KS_CT, KS_UT, KS_DT, KS_AUX, KS_META };
enum { CS_ID1 = 0, CS_C2, CS_T, CS_META };  // C2 = node value | member id2

__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits of mask below my lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint64_t upto(int lane) { return lane == 63 ? ~0ull : ((2ull << lane) - 1); }

// Position of the segment head for slot (lane, e): the highest head bit at or below it
// (the slot itself is live, so position 0 is a head and the search always succeeds).
template <int E>
__device__ __forceinline__ int seg_head(const uint64_t (&H)[E], int e, int lane) {
  const uint64_t m = H[e] & upto(lane);
  if (m) return 64 * e + 63 - __clzll(m);
#pragma unroll
  for (int f = E - 1; f >= 0; --f)
    if (f < e && H[f]) return 64 * f + 63 - __clzll(H[f]);
  return 0;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}
// Sum over the wave of per-lane values below 2^BITS: one ballot + popcount per bit.
template <int BITS>
__device__ __forceinline__ uint32_t wave_sum_bits(uint32_t x) {
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < BITS; ++k) s += (uint32_t)__popcll(__ballot((x >> k) & 1u)) << k;
  return s;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x = max(x, (uint64_t)__shfl_xor((unsigned long long)x, d, 64));
  return x;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x = min(x, (uint64_t)__shfl_xor((unsigned long long)x, d, 64));
  return x;
}

// rk[e] = #{j < n : sw[j] < w[e]} for the first EA of my words; sw[n] must be ~0 when n is
// odd (the loop reads pairs). Words are distinct, so ranks are a permutation of [0, n).
template <int EA, int E>
__device__ __forceinline__ void rank_count(const uint64_t* sw, uint32_t n, const uint64_t (&w)[E],
                                           uint32_t (&rk)[E]) {
#pragma unroll
  for (int e = 0; e < EA; ++e) rk[e] = 0;
  const uint32_t n2 = (n + 1) & ~1u;
#pragma unroll 4
  for (uint32_t j = 0; j < n2; j += 2) {
    const uint64_t a = sw[j], b = sw[j + 1];  // same address in every lane: LDS broadcast
#pragma unroll
    for (int e = 0; e < EA; ++e) rk[e] += (uint32_t)(a < w[e]) + (uint32_t)(b < w[e]);
  }
}

// Sorted-run input (cdb_dev_input.n_runs > 0): the rows of every family are nr runs, each
// non-decreasing in (parent) key hash, left where the caller put them (SoA columns). Bucket b's
// rows in run r of family f are run rows [rdir[f][r * (nb + 1) + b], rdir[f][r * (nb + 1) + b + 1])
// (run-relative), i.e. a few consecutive rows per run: the wave kernels read them column by
// column with no partition pass and no row permutation (runs.hip.h).
struct RunView {
  const uint32_t* rdir[3];
  const uint64_t* rbase;      // absolute first row of run r of family f at rbase[f * 65 + r]
  uint32_t nr;
  uint32_t nbp1;              // nb + 1: one run's directory row
  const uint64_t* kin[kKeyCols];
  const uint64_t* nin[kNodeCols];
  const uint64_t* min[kMemberCols];
  uint32_t ks, ns, ms;        // record strides of the families (1: plain columns; common.h row_field)
  uint32_t rs_sum[3];         // per family, the sum of the runs' first rows (mod 2^32): a bucket's
                              // dense base is the sum of its slices' first rows minus this
  const uint32_t* bdir;       // at most 8 runs: the bucket-major directory (run_reduce3_kernel), else null
};

struct WaveArgs {
  BucketArgs A;
  uint32_t nbuckets;
  uint32_t blo, bhi;    // this launch's bucket range (the bucket phase runs in chunks)
  uint32_t* big_list;   // buckets for the workgroup tier
  uint32_t* big_count;
  RunView V;            // sorted-run path only
  uint32_t* wide_next;  // the wide tier's next group of 64 buckets (one counter per range)
  uint32_t* pipe_next;  // the persistent wave tier's next chunk, one counter per XCD slab (8)
  const uint32_t* units;  // the persistent wave tier's unit starts: bit b of the bitmap (pipe_units_kernel)
};

// A bucket's directory entry (row counts and first row of each family).
struct WaveDir {
  uint32_t K = 0, N = 0, M = 0, kb = 0, nb0 = 0, mb0 = 0;
  // Buckets of the unit: the persistent wave tier merges G consecutive buckets whose rows fit one
  // wave as one (their rows are consecutive rows of every run, their hash span fits the sort word)
  // and counts every output to the first: bucket b then holds the group's rows in hash order in its
  // slots, buckets b + 1 .. b + G - 1 none -- the bucket layout's contract (cdb_dev_buckets: each
  // bucket's rows in its slot range, in key-hash order, ascending over buckets) holds as it is.
  uint32_t G = 1;
};
__device__ __forceinline__ WaveDir load_dir(const BucketArgs& A, uint32_t b) {
  WaveDir d;
  d.K = A.kcnt[b];
  d.N = A.ncnt[b];
  d.M = A.mcnt[b];
  d.kb = A.kbase[b];
  d.nb0 = A.nbase[b];
  d.mb0 = A.mbase[b];
  return d;
}

// Row indices of a bucket's rows (the last partition level is index-only).
template <int KE>
struct WavePerm {
  uint32_t krow[KE], crow[2 * KE];
};
template <int KE>
__device__ __forceinline__ void load_perm(const BucketArgs& A, const WaveDir& d, int lane, WavePerm<KE>& p) {
  const uint32_t C = d.N + d.M;
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const uint32_t c = lane + 64 * e;
    p.krow[e] = c < d.K ? A.kp[d.kb + c] : 0;
  }
#pragma unroll
  for (int e = 0; e < 2 * KE; ++e) {
    const uint32_t c = lane + 64 * e;
    p.crow[e] = c < d.N ? A.np[d.nb0 + c] : (c < C ? A.mp[d.mb0 + (c - d.N)] : 0);
  }
}

// Every input column of a bucket: KE key rows and CE child rows per lane (CE = 1 for the
// buckets of at most 64 child rows, the common case: the child phases then run once per lane).
template <int KE, int CE = 2 * KE>
struct WaveIn {
  WaveDir d;
  uint64_t kh[KE], kf[KE], kct[KE], kut[KE], kdt[KE], kaux[KE], kmeta[KE];
  uint64_t cpkh[CE], cpkf[CE], cid1[CE], cid2[CE], ct[CE], cm[CE];
};
template <int KE>
__device__ __forceinline__ void load_cols(const BucketArgs& A, const WaveDir& d, const WavePerm<KE>& p, int lane,
                                          WaveIn<KE>& in) {
  // A lane reads its own row: three 16-B pieces (+ one 8-B word for a key row's meta), all
  // from the row's one (key) or two (child) cache lines.
  in.d = d;
  const uint32_t C = d.N + d.M;
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const uint32_t c = lane + 64 * e;
    in.kh[e] = in.kf[e] = in.kct[e] = in.kut[e] = in.kdt[e] = in.kaux[e] = in.kmeta[e] = 0;
    if (c < d.K) {
      const uint64_t* row = A.kr + (uint64_t)p.krow[e] * kKeyStride;
      const ulonglong2 q0 = reinterpret_cast<const ulonglong2*>(row)[0];
      const ulonglong2 q1 = reinterpret_cast<const ulonglong2*>(row)[1];
      const ulonglong2 q2 = reinterpret_cast<const ulonglong2*>(row)[2];
      in.kh[e] = q0.x;
      in.kf[e] = q0.y;
      in.kct[e] = q1.x;
      in.kut[e] = q1.y;
      in.kdt[e] = q2.x;
      in.kaux[e] = q2.y;
      in.kmeta[e] = row[K_META];
    }
  }
#pragma unroll
  for (int e = 0; e < 2 * KE; ++e) {
    const uint32_t c = lane + 64 * e;
    in.cpkh[e] = in.cpkf[e] = in.cid1[e] = in.cid2[e] = in.ct[e] = in.cm[e] = 0;
    if (c < C) {
      const uint64_t* row = (c < d.N ? A.nr : A.mr) + (uint64_t)p.crow[e] * kChildStride;
      const ulonglong2 q0 = reinterpret_cast<const ulonglong2*>(row)[0];
      const ulonglong2 q1 = reinterpret_cast<const ulonglong2*>(row)[1];
      const ulonglong2 q2 = reinterpret_cast<const ulonglong2*>(row)[2];
      in.cpkh[e] = q0.x;
      in.cpkf[e] = q0.y;
      in.cid1[e] = q1.x;
      in.cid2[e] = q1.y;
      in.ct[e] = q2.x;
      in.cm[e] = q2.y;
    }
  }
}

// A bucket is merged in two halves. The first (phases 0-3) consumes the bucket's input registers:
// keys ranked and folded, children found, ranked and staged in LDS. The second (phases 4-5) folds
// the children and writes every output from LDS and the key state below. Between them the input
// registers are dead, which is where a streaming kernel issues the next bucket's loads (one
// program point: wave_bucket's `next()`).
template <int KE>
struct WaveMid {
  uint32_t K, N, M, kb, nb0, mb0, kout, nlive, G;  // (wave-uniform)
  uint64_t kh[KE], kf[KE], o_ct[KE], o_ut[KE], o_dt[KE], o_meta[KE], o_win[KE];
  uint32_t o_T[KE], orank[KE], fam[KE];
  bool emit[KE];
  uint32_t st_conf, st_dict, st_gcd, orph;
};
enum { WAVE_GO = 0, WAVE_DONE = 1, WAVE_PUSH = 2 };  // first half: second half / nothing more / exact tier

// Hands buckets b .. b + G - 1 to the workgroup tier (no outputs until that tier's: a pipelined
// compaction may read them first).
__device__ __forceinline__ void wave_push(const WaveArgs& W, uint32_t b, int lane, uint32_t G = 1) {
  if ((uint32_t)lane < G) {
    W.A.kout[b + lane] = W.A.nout[b + lane] = W.A.mout[b + lane] = 0;
    W.big_list[atomicAdd(W.big_count, 1u)] = b + lane;
  }
}

// One bucket on one wave, up to 64*KE key rows and 128*KE child rows, from the columns in
// `in`. KE = 1 leaves buckets over that capacity to bucket_wide_kernel and lists those over
// ITS capacity (and forced tiers) for the workgroup tier (WAVE_PUSH).
template <int KE, int CE>
__device__ __forceinline__ int wave_phase_a(const WaveArgs& W, WaveLds<KE>& L, uint32_t b, int lane,
                                            const WaveIn<KE, CE>& in, WaveMid<KE>& mid) {
  static_assert(CE <= 2 * KE, "child slots per lane");
  constexpr uint32_t KC = WaveLds<KE>::KC, CC = WaveLds<KE>::CC;
  const BucketArgs& A = W.A;
  const uint32_t K = in.d.K, N = in.d.N, M = in.d.M;
  if (KE == 1) {  // the wide kernel finds its buckets itself (wide_bucket_candidate)
    if (A.force_tier == 1 || A.force_tier == 2 || A.force_tier == 4 || N + M > WaveLds<2>::CC || K > WaveLds<2>::KC)
      return WAVE_PUSH;
    if (K > KC || N + M > CC || A.force_tier == 3) return WAVE_DONE;
  }
  const uint32_t kb = in.d.kb, nb0 = in.d.nb0, mb0 = in.d.mb0;
  const uint32_t C = N + M;

  // ------------------------------------------------------------ 0. the bucket's columns
  uint64_t kh[KE], kf[KE], kct[KE], kut[KE], kdt[KE], kaux[KE], kmeta[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    kh[e] = in.kh[e];
    kf[e] = in.kf[e];
    kct[e] = in.kct[e];
    kut[e] = in.kut[e];
    kdt[e] = in.kdt[e];
    kaux[e] = in.kaux[e];
    kmeta[e] = in.kmeta[e];
  }
  uint64_t cpkh[CE], cpkf[CE], cid1[CE], cid2[CE], ct_[CE], cm[CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    cpkh[e] = in.cpkh[e];
    cpkf[e] = in.cpkf[e];
    cid1[e] = in.cid1[e];
    cid2[e] = in.cid2[e];
    ct_[e] = in.ct[e];
    cm[e] = in.cm[e];
  }

  if (CDB_WAVE_STOP <= 0) {
    const unsigned long long sk = wave_sum_u64((unsigned long long)(in.kh[0] ^ in.kf[0] ^ in.kct[0] ^ in.kut[0] ^ in.kdt[0] ^ in.kaux[0] ^ in.kmeta[0] ^ in.cpkh[0] ^ in.cpkf[0] ^ in.cid1[0] ^ in.cid2[0] ^ in.ct[0] ^ in.cm[0] ^ in.cpkh[CE-1] ^ in.cm[CE-1]));
    if (lane == 0) {
      A.kout[b] = A.nout[b] = A.mout[b] = 0;
      atomicAdd(&stat_shard(A.stats)[kStatStride - 1], sk);
    }
    return WAVE_DONE;
  }
  // ------------------------------------------------------------ 1. keys: rank + scatter
  // word = rel << 20 | family << 18 | pos << 12 | slot   (pos < 64, slot < 4096), where rel is
  // the 44 leading bits of (kh << shift) - b * bw (BucketArgs): monotone in the key hash, so the
  // output keys leave in exact key-hash order whenever rel_shift == 0 (a merge result is then a
  // sorted run for the next merge, runs.hip.h); two hashes that share rel go to the exact tier
  const int ks = A.key_shift, rsh = A.rel_shift;
  const uint64_t lo = (uint64_t)b * A.bw;
  auto rel44 = [&](uint64_t h) { return (((h << ks) - lo) >> rsh) & kM44; };
  uint64_t w[KE];
  uint32_t rk[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const uint32_t c = lane + 64 * e;
    w[e] = (rel44(kh[e]) << 20) | ((uint64_t)tag_family(meta_tag(kmeta[e])) << 18) |
           ((uint64_t)meta_pos(kmeta[e]) << 12) | c;
    if (c < K) L.sw[c] = w[e];
  }
  if (lane == 0) L.sw[K] = ~0ull;
  wave_sync();
  rank_count<KE>(L.sw, K, w, rk);
  wave_sync();
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    if (lane + 64 * e < K) {
      const uint32_t s = rk[e];
      L.sw[s] = w[e];
      L.col[KS_KH][s] = kh[e];
      L.col[KS_KF][s] = kf[e];
      L.col[KS_CT][s] = kct[e];
      L.col[KS_UT][s] = kut[e];
      L.col[KS_DT][s] = kdt[e];
      L.col[KS_AUX][s] = kaux[e];
      L.col[KS_META][s] = kmeta[e];
    }
  }
  wave_sync();
  // sorted slot s = lane + 64 e from here on
  uint32_t fam[KE];
  uint64_t Hk[KE];
  bool kin[KE], coll = false;
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const uint32_t s = lane + 64 * e;
    kin[e] = s < K;
    const uint32_t sp = s > 0 ? s - 1 : 0;
    w[e] = kin[e] ? L.sw[s] : ~0ull;
    kh[e] = L.col[KS_KH][s];
    kf[e] = L.col[KS_KF][s];
    const uint64_t pw = L.sw[sp], pkh = L.col[KS_KH][sp], pkf = L.col[KS_KF][sp];
    fam[e] = (uint32_t)(w[e] >> 18) & 3;
    const bool same_key = kin[e] && s > 0 && (pw >> 20) == (w[e] >> 20);
    // equal kh bits but another identity: a 2^-44 event (or a real 64-bit kh collision);
    // equal (key, family, pos): duplicate keys in one snapshot, folded in src order there
    coll |= same_key && (pkh != kh[e] || pkf != kf[e] || (pw >> 12) == (w[e] >> 12));
    Hk[e] = __ballot(kin[e] && (s == 0 || (pw >> 18) != (w[e] >> 18)));
  }
  if (__ballot(coll)) return WAVE_PUSH;

  if (CDB_WAVE_STOP <= 1) {
    const unsigned long long sk = wave_sum_u64((unsigned long long)(w[0] ^ kh[0] ^ (uint64_t)Hk[0]));
    if (lane == 0) {
      A.kout[b] = A.nout[b] = A.mout[b] = 0;
      atomicAdd(&stat_shard(A.stats)[kStatStride - 1], sk);
    }
    return WAVE_DONE;
  }
  // ------------------------------------------------------------ 2. key folds (tail slots)
  const uint64_t last_bad = (A.flags & F_GC_DELETES) ? *A.last_bad : 0;
  uint64_t o_ct[KE], o_ut[KE], o_dt[KE], o_meta[KE], o_win[KE];
  uint32_t o_T[KE], orank[KE];
  bool emit[KE];
  uint32_t st_conf = 0, st_dict = 0, st_gcd = 0;
  uint32_t kout = 0;
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const int pos = lane + 64 * e;
    const int en = e + 1 < KE ? e + 1 : e;
    const bool nxt_head = lane < 63 ? ((Hk[e] >> (lane + 1)) & 1) : (e + 1 < KE && (Hk[en] & 1));
    const bool ktail = kin[e] && (pos == (int)K - 1 || nxt_head);
    const uint32_t fm = fam[e];
    uint64_t vm = 0, sum = 0;
    uint32_t hp = 0;
    o_ct[e] = o_ut[e] = o_dt[e] = o_meta[e] = o_win[e] = 0;
    o_T[e] = 0;
    emit[e] = false;
    if (ktail) {
      const int hl = seg_head<KE>(Hk, e, lane);
      const uint64_t m0 = L.col[KS_META][hl];
      const uint32_t T = meta_tag(m0);
      hp = meta_pos(m0);
      const uint64_t ct0 = L.col[KS_CT][hl], ut0 = L.col[KS_UT][hl], dt0 = L.col[KS_DT][hl];
      uint64_t ct = ct0, ut = ut0, dt = dt0;
      uint64_t win = meta_order(m0), lastm = m0;
      uint32_t nvalid = 1, conflicts = 0;
      vm = 1ull << hp;
      const uint64_t tl_ct = L.col[KS_CT][pos];  // the segment's last row (side maps)
      bool gc_hit = fm == 2 && meta_order(m0) + 1 > last_bad && ct0 == tl_ct;
      for (int q = hl + 1; q <= pos; ++q) {
        const uint64_t m = L.col[KS_META][q];
        lastm = m;
        if (fm != 0) {
          gc_hit |= fm == 2 && meta_order(m) + 1 > last_bad && L.col[KS_CT][q] == tl_ct;
          continue;
        }
        if (meta_tag(m) != T) {  // object.rs:80: type conflict, local kept
          ++conflicts;
          continue;
        }
        ++nvalid;
        vm |= 1ull << meta_pos(m);
        if (T == TAG_BYTES) {  // object.rs:69-77
          const uint64_t c2 = L.col[KS_CT][q];
          if (ct < c2) win = meta_order(m);
          ct = max(ct, c2);
          dt = max(dt, L.col[KS_DT][q]);
          ut = max(ut, L.col[KS_UT][q]);
        }
      }
      if (fm == 0) {
        st_conf += conflicts;
        if (T == TAG_DICT) st_dict += nvalid - 1;
        o_T[e] = T;
        // non-Bytes objects keep the head's times (object.rs:68,78-79)
        o_ct[e] = T == TAG_BYTES ? ct : ct0;
        o_ut[e] = T == TAG_BYTES ? ut : ut0;
        o_dt[e] = T == TAG_BYTES ? dt : dt0;
        o_meta[e] = m0;
        o_win[e] = T == TAG_BYTES ? win : 0;
        vm |= (T == TAG_COUNTER && nvalid >= 2) ? kVmaskMerged : 0;
        // a counter that was never merged keeps its load-time total (aux, head row)
        // (sorted-run path, W.V.nr > 0: the aux slot holds the head row's index, its aux word is
        // read from the runs only here)
        if (T == TAG_COUNTER && nvalid < 2) {
          const uint64_t a = L.col[KS_AUX][hl];
          sum = W.V.nr ? row_field(W.V.kin, W.V.ks, K_AUX, a) : a;
        }
        emit[e] = true;
      } else {  // expires / deletes: plain overwrite, the last (pos, src) wins
        const bool removed = fm == 2 && (A.flags & F_GC_DELETES) && gc_hit;
        o_T[e] = meta_tag(lastm);
        hp = meta_pos(lastm);
        o_ct[e] = tl_ct;
        o_meta[e] = lastm;
        o_win[e] = meta_order(lastm);
        emit[e] = !removed;
        st_gcd += removed ? 1 : 0;
      }
    }
    const uint64_t Ek = __ballot(emit[e]);
    orank[e] = kout + lane_rank(Ek);
    kout += __popcll(Ek);
    if (emit[e]) {
      const uint32_t o = orank[e];
      L.okh[o] = kh[e];
      L.okf[o] = kf[e];
      L.ovm[o] = vm;
      L.otp[o] = o_T[e] | (hp << 8);
      L.osum[o] = sum;
      L.ocnt[o] = 0;
      L.ocb[o] = kNone;
    }
  }
  wave_sync();

  if (CDB_WAVE_STOP <= 2) {
    const unsigned long long sk = wave_sum_u64((unsigned long long)((uint64_t)kout ^ o_ct[0] ^ o_win[0]));
    if (lane == 0) {
      A.kout[b] = A.nout[b] = A.mout[b] = 0;
      atomicAdd(&stat_shard(A.stats)[kStatStride - 1], sk);
    }
    return WAVE_DONE;
  }
  // ------------------------------------------------------------ 3. children: key lookup
  // word = key rank << 56 | child_order(id1)[63:22] << 14 | pos << 8 | slot   (rank < 128, slot < 256)
  uint32_t orph = 0;
  uint32_t ckey[CE];
  bool clive[CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const uint32_t c = lane + 64 * e;
    clive[e] = false;
    ckey[e] = 0;
    if (c < C) {
      const bool isn = c < N;
      uint32_t ql = 0, qh = kout;  // lower bound (output keys are in word order)
      if (rsh == 0) {   // word order is (hash << shift) order: compare those directly
        const uint64_t t = cpkh[e] << ks;
        while (ql < qh) {
          const uint32_t mid = (ql + qh) >> 1;
          const bool less = (L.okh[mid] << ks) < t;
          ql = less ? mid + 1 : ql;
          qh = less ? qh : mid;
        }
      } else {
        const uint64_t t44 = rel44(cpkh[e]);
        while (ql < qh) {
          const uint32_t mid = (ql + qh) >> 1;
          const bool less = rel44(L.okh[mid]) < t44;
          ql = less ? mid + 1 : ql;
          qh = less ? qh : mid;
        }
      }
      if (ql < kout && L.okh[ql] == cpkh[e] && L.okf[ql] == cpkf[e] && (L.otp[ql] & 0xFF) <= TAG_SET) {
        const uint32_t KT = L.otp[ql] & 0xFF, khp = L.otp[ql] >> 8, p = meta_pos(cm[e]);
        const bool type_ok = isn ? KT == TAG_COUNTER : (KT == TAG_SET || KT == TAG_DICT);
        const bool elem_ok = (L.ovm[ql] >> p) & 1;
        const bool cand = isn || meta_tag(cm[e]) == KIND_ADD || p == khp;  // remote dels ignored
        clive[e] = type_ok && elem_ok && cand;
        ckey[e] = ql;
      } else {
        ++orph;
      }
    }
  }
  // live children -> compact list of words, then rank
  uint64_t cw[CE];
  uint32_t crk[CE];
  uint32_t nlive = 0;
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const uint32_t c = lane + 64 * e;
    const bool isn = c < N;
    cw[e] = ~0ull;
    if (clive[e]) {
      // ranked by the leading 42 bits of child_order(id1) (ids that share them are caught below
      // and go to the exact tier)
      cw[e] = ((uint64_t)ckey[e] << 56) | ((child_order(cid1[e]) >> 22) << 14) | ((uint64_t)meta_pos(cm[e]) << 8) | c;
    }
    const uint64_t Lm = __ballot(clive[e]);
    if (clive[e]) L.sw[nlive + lane_rank(Lm)] = cw[e];
    nlive += __popcll(Lm);
  }
  if (lane == 0) L.sw[nlive] = ~0ull;
  wave_sync();
  // a lane's live words sit at its input slots lane + 64 e, so rank the first ceil(C / 64)
  if (CE >= 4 && C > 192)
    rank_count<(CE >= 4 ? 4 : CE)>(L.sw, nlive, cw, crk);
  else if (CE >= 3 && C > 128)
    rank_count<(CE >= 3 ? 3 : CE)>(L.sw, nlive, cw, crk);
  else if (CE >= 2 && C > 64)
    rank_count<(CE >= 2 ? 2 : CE)>(L.sw, nlive, cw, crk);
  else
    rank_count<1>(L.sw, nlive, cw, crk);
  wave_sync();
  // node rows keep id2 = value; for the identity check a node compares only its id
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    if (clive[e]) {
      const uint32_t s = crk[e];
      L.sw[s] = cw[e];
      L.ccol[CS_ID1][s] = cid1[e];
      L.ccol[CS_C2][s] = cid2[e];
      L.ccol[CS_T][s] = ct_[e];
      L.ccol[CS_META][s] = cm[e];
    }
  }
  wave_sync();
  // this bucket's input registers are dead from here on
  mid.K = K;
  mid.N = N;
  mid.M = M;
  mid.kb = kb;
  mid.nb0 = nb0;
  mid.mb0 = mb0;
  mid.kout = kout;
  mid.nlive = nlive;
  mid.G = in.d.G;
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    mid.kh[e] = kh[e];
    mid.kf[e] = kf[e];
    mid.o_ct[e] = o_ct[e];
    mid.o_ut[e] = o_ut[e];
    mid.o_dt[e] = o_dt[e];
    mid.o_meta[e] = o_meta[e];
    mid.o_win[e] = o_win[e];
    mid.o_T[e] = o_T[e];
    mid.orank[e] = orank[e];
    mid.fam[e] = fam[e];
    mid.emit[e] = emit[e];
  }
  mid.st_conf = st_conf;
  mid.st_dict = st_dict;
  mid.st_gcd = st_gcd;
  mid.orph = orph;
  return WAVE_GO;
}

template <int KE, int CE>
__device__ __forceinline__ void wave_phase_b(const WaveArgs& W, WaveLds<KE>& L, uint32_t b, int lane,
                                             const WaveMid<KE>& mid) {
  constexpr uint32_t KC = WaveLds<KE>::KC;
  const BucketArgs& A = W.A;
  const uint32_t kb = mid.kb, nb0 = mid.nb0, mb0 = mid.mb0, kout = mid.kout, nlive = mid.nlive;
  const uint32_t st_conf = mid.st_conf, st_dict = mid.st_dict, st_gcd = mid.st_gcd, orph = mid.orph;
  const auto& kh = mid.kh;
  const auto& kf = mid.kf;
  const auto& o_ct = mid.o_ct;
  const auto& o_ut = mid.o_ut;
  const auto& o_dt = mid.o_dt;
  const auto& o_meta = mid.o_meta;
  const auto& o_win = mid.o_win;
  const auto& o_T = mid.o_T;
  const auto& orank = mid.orank;
  const auto& fam = mid.fam;
  const auto& emit = mid.emit;
  uint32_t gcm = 0;
  if (CDB_WAVE_STOP <= 3) {
    const unsigned long long sk = wave_sum_u64((unsigned long long)((uint64_t)nlive ^ orph));
    if (lane == 0) {
      A.kout[b] = A.nout[b] = A.mout[b] = 0;
      atomicAdd(&stat_shard(A.stats)[kStatStride - 1], sk);
    }
    return;
  }
  // ------------------------------------------------------------ 4. child folds + outputs
  bool live[CE], knode[CE], coll2 = false;
  uint64_t H[CE], Lv[CE], sw_[CE], sid1[CE], sid2[CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const uint32_t s = lane + 64 * e;
    live[e] = s < nlive;
    const uint32_t sp = s > 0 ? s - 1 : 0;
    sw_[e] = live[e] ? L.sw[s] : ~0ull;
    const uint32_t k = (uint32_t)(sw_[e] >> 56) & (KC - 1);
    knode[e] = live[e] && (L.otp[k] & 0xFF) == TAG_COUNTER;
    sid1[e] = L.ccol[CS_ID1][s];
    sid2[e] = knode[e] ? 0 : L.ccol[CS_C2][s];
    const uint64_t pw = L.sw[sp], p1 = L.ccol[CS_ID1][sp], p2 = knode[e] ? 0 : L.ccol[CS_C2][sp];
    const bool same = live[e] && s > 0 && (pw >> 14) == (sw_[e] >> 14);
    coll2 |= same && (p1 != sid1[e] || p2 != sid2[e] || (pw >> 8) == (sw_[e] >> 8));
    H[e] = __ballot(live[e] && (s == 0 || !same));
    Lv[e] = __ballot(live[e]);
  }
  if (__ballot(coll2)) {  // id-hash collision or duplicate: exact tier (nothing written yet)
    wave_push(W, b, lane, mid.G);
    return;
  }
  uint64_t En[CE], Em[CE], c_v[CE], c_t[CE], c_m[CE];
  bool cemit[CE];
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const int en = e + 1 < CE ? e + 1 : e;
    const bool nxt_head = lane < 63 ? ((H[e] >> (lane + 1)) & 1) : (e + 1 < CE && (H[en] & 1));
    const bool nxt_live = lane < 63 ? ((Lv[e] >> (lane + 1)) & 1) : (e + 1 < CE && (Lv[en] & 1));
    const bool ctail = live[e] && (nxt_head || !nxt_live);
    const int pos = lane + 64 * e;
    c_v[e] = c_t[e] = c_m[e] = 0;
    cemit[e] = false;
    if (ctail) {
      const int hl = seg_head<CE>(H, e, lane);
      if (knode[e]) {  // Counter::merge per node (type_counter.rs:60-84): the head's t is kept
        const uint64_t t0 = L.ccol[CS_T][hl];
        uint64_t v = L.ccol[CS_C2][hl];
        for (int q = hl + 1; q <= pos; ++q) {
          const uint64_t tt = L.ccol[CS_T][q], vv = L.ccol[CS_C2][q];
          v = tt > t0 ? vv : (tt == t0 ? imax64(v, vv) : v);
        }
        c_v[e] = v;
        c_t[e] = t0;
        const uint64_t mh = L.ccol[CS_META][hl];
        c_m[e] = meta_pack(0, meta_pos(mh), meta_src(mh));
        cemit[e] = true;
      } else {  // LWWHash::set chain (lwwhash.rs:87-107): the later candidate wins ties
        int wq = hl;
        uint64_t tw = L.ccol[CS_T][hl];
        for (int q = hl + 1; q <= pos; ++q) {
          const uint64_t tr = L.ccol[CS_T][q];
          const bool later = !(tw > tr);
          wq = later ? q : wq;
          tw = later ? tr : tw;
        }
        c_t[e] = tw;
        c_m[e] = L.ccol[CS_META][wq];
        cemit[e] = true;
        if ((A.flags & F_GC_MEMBERS) && meta_tag(c_m[e]) == KIND_DEL && tw < A.gc_wm) {
          cemit[e] = false;
          ++gcm;
        }
      }
    }
    En[e] = __ballot(cemit[e] && knode[e]);
    Em[e] = __ballot(cemit[e] && !knode[e]);
  }
  // output positions: the bucket's row slots (its input offsets); each lane stores its rows whole
  // (16-B pieces). Staging the rows in LDS for wave-contiguous stores was measured slower (C4:
  // 20.5 -> 21.3 ms with per-lane record loads, the extra LDS round trip and VALU outweigh it).
  const uint64_t xk = kb, xn = nb0, xm = mb0;
  uint32_t nbase = 0, mbase = 0;
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    if (cemit[e]) {
      const uint32_t crank = (knode[e] ? nbase : mbase) + lane_rank(knode[e] ? En[e] : Em[e]);
      const uint32_t k = (uint32_t)(sw_[e] >> 56) & (KC - 1);
      const uint64_t id2 = knode[e] ? c_v[e] : sid2[e];
      {  // one whole 48-B AoS row
        ulonglong2* row = (ulonglong2*)((knode[e] ? A.nos : A.mos) + ((knode[e] ? xn : xm) + crank) * kChildStride);
        st_row16(row + 0, L.okh[k], L.okf[k]);
        st_row16(row + 1, sid1[e], id2);
        st_row16(row + 2, c_t[e], c_m[e]);
      }
      if (knode[e] && (L.ovm[k] & kVmaskMerged))
        atomicAdd((unsigned long long*)&L.osum[k], (unsigned long long)c_v[e]);
      atomicMin(&L.ocb[k], crank);
      atomicAdd(&L.ocnt[k], 1u);
    }
    nbase += __popcll(En[e]);
    mbase += __popcll(Em[e]);
  }
  wave_sync();

  // ------------------------------------------------------------ 5. key outputs
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    if (emit[e]) {
      const uint32_t r = orank[e];
      const uint64_t win = (fam[e] == 0 && o_T[e] == TAG_COUNTER) ? L.osum[r] : o_win[e];
      // child ranges: bucket-relative (compaction makes them absolute)
      const uint64_t cref = cref_pack(L.ocnt[r] ? L.ocb[r] : 0, L.ocnt[r]);
      {  // one whole 64-B AoS row
        ulonglong2* row = (ulonglong2*)(A.kos + (xk + r) * kKeyOutCols);
        st_row16(row + 0, kh[e], kf[e]);
        st_row16(row + 1, o_ct[e], o_ut[e]);
        st_row16(row + 2, o_dt[e], o_meta[e]);
        st_row16(row + 3, win, cref);
      }
    }
  }
  if ((uint32_t)lane < mid.G) {  // (a group: every output counted to its first bucket)
    A.kout[b + lane] = lane == 0 ? kout : 0u;
    A.nout[b + lane] = lane == 0 ? nbase : 0u;
    A.mout[b + lane] = lane == 0 ? mbase : 0u;
  }
  unsigned long long* st = stat_shard(A.stats);
  // per-lane counts are small (<= 64 KE segment rows, <= CE children): summed by bit slices
  if (__ballot(st_conf)) {
    const unsigned long long v = wave_sum_bits<8>(st_conf);
    if (lane == 0) atomicAdd(&st[ST_TYPE_CONFLICTS], v);
  }
  if (__ballot(st_dict)) {
    const unsigned long long v = wave_sum_bits<8>(st_dict);
    if (lane == 0) atomicAdd(&st[ST_DICT_MERGES], v);
  }
  if (__ballot(orph)) {
    const unsigned long long v = wave_sum_bits<3>(orph);
    if (lane == 0) atomicAdd(&st[ST_ORPHANS], v);
  }
  if (__ballot(st_gcd)) {
    const unsigned long long v = wave_sum_bits<2>(st_gcd);
    if (lane == 0) atomicAdd(&st[ST_DELETES_GCED], v);
  }
  if (__ballot(gcm)) {
    const unsigned long long v = wave_sum_bits<3>(gcm);
    if (lane == 0) atomicAdd(&st[ST_MEMBERS_GCED], v);
  }
}


// The whole bucket: first half, `next()` (exactly once per bucket, at this one point), second half.
template <int KE, int CE, typename Next>
__device__ __forceinline__ void wave_bucket(const WaveArgs& W, WaveLds<KE>& L, uint32_t b, int lane,
                                            const WaveIn<KE, CE>& in, Next&& next) {
  WaveMid<KE> mid;
  const int act = wave_phase_a<KE, CE>(W, L, b, lane, in, mid);
  next();
  if (act == WAVE_PUSH)
    wave_push(W, b, lane);
  else if (act == WAVE_GO)
    wave_phase_b<KE, CE>(W, L, b, lane, mid);
}

constexpr uint32_t kXcds = 8;

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2). Remap so
// that XCD x runs one contiguous range of blocks: neighbouring buckets share a final
// partition segment, whose rows then stay in one L2.
__device__ __forceinline__ uint32_t xcd_block(uint32_t i, uint32_t G) {
  const uint32_t q = G / kXcds, r = G % kXcds, x = i % kXcds, j = i / kXcds;
  return x * q + min(x, r) + j;
}

// One bucket per wave, no loop: the fewest live registers and so the most resident waves
// (5 per SIMD), which is what hides the bucket's memory round trips best (software-pipelined
// variants that prefetched the next bucket lost more to their lower occupancy than they gained;
// DESIGN.md §4a').
__global__ void __launch_bounds__(kWavesPerWG * 64) bucket_wave_kernel(WaveArgs W) {
  __shared__ WaveLds<1> lds_all[kWavesPerWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // buckets in dispatch order (an XCD remap measured no faster with whole-row reads)
  const uint32_t b = W.blo + blockIdx.x * kWavesPerWG + wv;
  if (b >= W.bhi) return;
  const WaveDir d = load_dir(W.A, b);
  WavePerm<1> p;
  WaveIn<1> in;
  load_perm<1>(W.A, d, lane, p);
  load_cols<1>(W.A, d, p, lane, in);
  wave_bucket<1>(W, lds_all[wv], b, lane, in, []() {});
}

// Buckets over bucket_wave_kernel's capacity but within this kernel's.
__device__ __forceinline__ bool wide_bucket_candidate(const BucketArgs& A, uint32_t b) {
  const uint32_t K = A.kcnt[b], C = A.ncnt[b] + A.mcnt[b];
  if (A.force_tier == 1 || A.force_tier == 2 || A.force_tier == 4 || C > WaveLds<2>::CC || K > WaveLds<2>::KC) return false;
  return K > WaveLds<1>::KC || C > WaveLds<1>::CC || A.force_tier == 3;
}

// The wide tier's next group of 64 buckets: one atomic per group on a counter of the range, so
// that a second, wider launch queued behind the wave tier joins the one running beside it and
// takes the groups left when the wave tier ends (C5's wide tier ran 0.7 ms past it at one wave
// per SIMD).
// A claim takes kWideClaim groups (one atomic per 512 buckets: claiming single groups cost C4's
// 105K-group wide tier ~0.4 ms of contention).
constexpr uint32_t kWideClaim = 8;
__device__ __forceinline__ uint32_t wide_group(const WaveArgs& W, int lane, uint32_t& next, uint32_t& end) {
  if (next < end) return next++;  // (wave-uniform)
  uint32_t c = 0;
  if (lane == 0) c = atomicAdd(W.wide_next, 1u);
  c = (uint32_t)__shfl((int)c, 0);
  next = c * kWideClaim + 1;
  end = (c + 1) * kWideClaim;
  return c * kWideClaim;
}

// Persistent: each wave takes the bucket directory 64 buckets at a time and merges the
// candidates one by one.
__global__ void __launch_bounds__(kWavesPerWG * 64) bucket_wide_kernel(WaveArgs W) {
  __shared__ WaveLds<2> lds_all[kWavesPerWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t groups = (W.bhi - W.blo + 63) / 64;
  unsigned long long found = 0;
  (void)wv;
  uint32_t nx = 0, en = 0;
  for (uint32_t g = wide_group(W, lane, nx, en); g < groups; g = wide_group(W, lane, nx, en)) {
    const uint32_t b = W.blo + g * 64 + lane;
    uint64_t m = __ballot(b < W.bhi && wide_bucket_candidate(W.A, b));
    found += __popcll(m);
    while (m) {
      const int i = __builtin_ctzll(m);
      m &= m - 1;
      const uint32_t bb = W.blo + g * 64 + i;
      const WaveDir d = load_dir(W.A, bb);
      WavePerm<2> p;
      WaveIn<2> in;
      load_perm<2>(W.A, d, lane, p);
      load_cols<2>(W.A, d, p, lane, in);
      wave_bucket<2>(W, lds_all[wv], bb, lane, in, []() {});
    }
  }
  if (lane == 0 && found) atomicAdd(&stat_shard(W.A.stats)[ST_WIDE], found);
}

// Sums the statistic shards into out[0 .. ST_COUNT).
__global__ void stats_reduce_kernel(const unsigned long long* __restrict__ shards, unsigned long long* out) {
  for (int i = threadIdx.x; i < ST_COUNT; i += blockDim.x) {
    unsigned long long s = 0;
    for (int k = 0; k < kStatShards; ++k) s += shards[(size_t)k * kStatStride + i];
    out[i] = s;
  }
}

}  // namespace cdb
