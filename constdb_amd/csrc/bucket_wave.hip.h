// Wave-per-bucket merge kernels (gfx950, wave64) — the hot path of the merge.
//
// One 64-lane wave owns one bucket and never synchronises with another wave. Rows sit in
// registers, E per lane (row i = lane + 64 e):
//   1. keys: each lane loads its rows (coalesced); a register bitonic network over
//      __shfl_xor sorts (kh, family|pos|src|idx); equal kh with different kf (a 64-bit
//      collision) hands the bucket to the exact-comparator workgroup tier before anything
//      is written;
//   2. key folds: the tail slot of each (key, family) segment replays the reference's
//      sequential fold over its segment (<= R rows, read from LDS in sorted order):
//        data     DB::merge_entry / Object::merge   (db.rs:31-43, object.rs:63-83)
//        expires / deletes: last (pos, src) wins   (db.rs:68-76), DB::gc (db.rs:82-95);
//   3. children: counter nodes and set/dict members share the slots (a key has one type);
//      each finds its key by binary search over the wave's sorted output keys (LDS), is
//      kept if its element has the key's head type (object.rs:80) and, for members of a
//      non-head position, only if it is an add (SetIter/DictIter, lwwhash.rs:319-323);
//      sorted by (key rank, id hash, pos|src), folded per (key, node) with
//      Counter::merge's head-t rule (type_counter.rs:59-87) or per (key, member) with
//      LWWHash::set's later-wins-ties rule (lwwhash.rs:87-107);
//   4. counter sums (cal_sum, type_counter.rs:89-91) and child ranges; outputs are
//      written by the tail slots (ballot + mbcnt ranks).
// bucket_wave_kernel (KE = 1: 64 key rows, 128 child rows) runs every bucket; one over that
// goes to bucket_wide_kernel (KE = 2: 128 key rows, 256 child rows; fewer waves per CU for
// its larger LDS), and anything beyond that, collisions and forced tiers go to the
// workgroup tier (bucket.hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bucket.hip.h"
#include "common.h"

namespace cdb {

constexpr int kWavesPerWG = 4;

// Per-wave LDS. KE = key rows per lane (1 or 2); child rows per lane: 2 (KE = 1) or 4.
template <int KE>
struct WaveLds {
  static constexpr int KC = 64 * KE;                // key-row capacity
  static constexpr int CC = KE == 1 ? 128 : 256;    // child-row capacity
  uint64_t okh[KC], okf[KC], ovm[KC], osum[KC];
  uint32_t otp[KC], ocnt[KC], ocb[KC];
  uint32_t sidx[KC > CC ? KC : CC];
  union {  // per-row staging, gathered through sidx after each sort
    uint64_t col[5][KC];   // key rows (KC_*)
    uint64_t ccol[4][CC];  // child rows (CC_*)
  };
};

__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  return (uint64_t)__shfl_xor((unsigned long long)v, m, 64);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  return (uint64_t)__shfl_up((unsigned long long)v, d, 64);
}
__device__ __forceinline__ uint64_t bcast63(uint64_t v) {
  return (uint64_t)__shfl((unsigned long long)v, 63, 64);
}

// Branch-free lexicographic (a0, a1) < (b0, b1).
__device__ __forceinline__ bool lt2(uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1) {
  return (a0 < b0) | ((a0 == b0) & (a1 < b1));
}

// Ascending bitonic sort of 64*E two-word elements, element i = (lane, e), i = lane + 64 e.
// Stages with j >= 64 compare two elements of the same lane (no data movement); the rest
// exchange over __shfl_xor. Rows carry their staging index in the low bits of w1, so a
// compare-exchange moves two words. Sentinels are all-ones.
template <int E>
__device__ __forceinline__ void wave_bitonic(uint64_t (&w0)[E], uint64_t (&w1)[E]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int kk = 2; kk <= 64 * E; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int je = j / 64;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (e & je) continue;
          const int f = e | je;
          const bool up = ((64 * e) & kk) == 0;  // lower element keeps the min when ascending
          const bool sw = up ? lt2(w0[f], w1[f], w0[e], w1[e]) : lt2(w0[e], w1[e], w0[f], w1[f]);
          const uint64_t a0 = w0[e], a1 = w1[e];
          w0[e] = sw ? w0[f] : w0[e];
          w1[e] = sw ? w1[f] : w1[e];
          w0[f] = sw ? a0 : w0[f];
          w1[f] = sw ? a1 : w1[f];
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint64_t o0 = shfl_xor64(w0[e], j), o1 = shfl_xor64(w1[e], j);
          const bool keep_min = ((lane & j) == 0) == (((lane + 64 * e) & kk) == 0);
          const bool take = keep_min ? lt2(o0, o1, w0[e], w1[e]) : lt2(w0[e], w1[e], o0, o1);
          w0[e] = take ? o0 : w0[e];
          w1[e] = take ? o1 : w1[e];
        }
      }
    }
  }
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

struct WaveArgs {
  BucketArgs A;
  uint32_t nbuckets;
  uint32_t* wide_list;  // buckets over the main kernel's capacity (bucket_wide_kernel)
  uint32_t* wide_count;
  uint32_t* big_list;   // buckets for the workgroup tier
  uint32_t* big_count;
};

enum { KC_CT = 0, KC_UT, KC_DT, KC_META, KC_KF };  // key staging columns
enum { CC_ID1 = 0, CC_C2, CC_T, CC_META };        // child staging: C2 = node value | member id2

struct ChildOut {
  uint32_t nout, mout;
  unsigned long long orph, gcm;  // per-lane counts
};

// Stages 3-4 for up to 64*E child rows (nodes in [0, N), members in [N, N+M)); E <= CC/64. Returns
// false on a 64-bit id-hash collision (the bucket then goes to the exact tier; nothing has
// been written).
template <int E, int KE>
__device__ __forceinline__ bool children_stage(const BucketArgs& A, WaveLds<KE>& L, int lane, uint32_t N,
                                               uint32_t M, uint32_t nb0, uint32_t mb0, uint32_t kout,
                                               ChildOut& co) {
  uint64_t w0[E], w1[E];
  unsigned long long orph = 0, gcm = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t c = lane + 64 * e;
    w0[e] = ~0ull;
    w1[e] = ~0ull;
    if (c < N + M) {
      const bool isn = c < N;
      const uint64_t* const* C = isn ? A.nd : A.mb;
      const uint32_t row = isn ? A.np[nb0 + c] : A.mp[mb0 + (c - N)];
      const uint64_t cpkh = C[C_PKH][row], cpkf = C[C_PKF][row];
      const uint64_t id1 = C[C_ID1][row], m = C[C_META][row];
      L.ccol[CC_ID1][c] = id1;
      L.ccol[CC_C2][c] = C[C_ID2][row];
      L.ccol[CC_T][c] = C[C_T][row];
      L.ccol[CC_META][c] = m;
      uint32_t lo = 0, hi = kout;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const bool less = lt2(L.okh[mid], L.okf[mid], cpkh, cpkf);
        lo = less ? mid + 1 : lo;
        hi = less ? hi : mid;
      }
      uint32_t key = 255;
      if (lo < kout && L.okh[lo] == cpkh && L.okf[lo] == cpkf && (L.otp[lo] & 0xFF) <= TAG_SET) {
        const uint32_t KT = L.otp[lo] & 0xFF, khp = L.otp[lo] >> 8, p = meta_pos(m);
        const bool type_ok = isn ? KT == TAG_COUNTER : (KT == TAG_SET || KT == TAG_DICT);
        const bool elem_ok = (L.ovm[lo] >> p) & 1;
        const bool cand = isn || meta_tag(m) == KIND_ADD || p == khp;  // remote dels ignored
        if (type_ok && elem_ok && cand) key = lo;
      } else {
        ++orph;
      }
      if (key != 255) {
        const uint64_t ih = isn ? mix64(id1) : id1;
        w0[e] = ((uint64_t)key << 56) | (ih >> 8);
        w1[e] = (meta_order(m) << 8) | c;
      }
    }
  }
  wave_bitonic<E>(w0, w1);
  bool live[E], knode[E];
  uint32_t idx[E], ckey[E];
  uint64_t cid1[E], cid2[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    live[e] = (w0[e] >> 56) < 255u;  // valid rows sort before invalid and empty slots
    idx[e] = (uint32_t)(w1[e] & 0xFF);
    L.sidx[lane + 64 * e] = idx[e];
  }
  wave_sync();
  bool coll = false;
  uint64_t H[E], Lv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    ckey[e] = (uint32_t)(w0[e] >> 56) & (WaveLds<KE>::KC - 1);
    knode[e] = live[e] && (L.otp[ckey[e]] & 0xFF) == TAG_COUNTER;
    cid1[e] = live[e] ? L.ccol[CC_ID1][idx[e]] : 0;
    cid2[e] = (live[e] && !knode[e]) ? L.ccol[CC_C2][idx[e]] : 0;
    uint64_t p0 = shfl_up64(w0[e], 1), pid1 = shfl_up64(cid1[e], 1), pid2 = shfl_up64(cid2[e], 1);
    if (e > 0) {  // position 64e - 1 is lane 63's previous element
      const int ep = e > 0 ? e - 1 : 0;
      const uint64_t x0 = bcast63(w0[ep]), x1 = bcast63(cid1[ep]), x2 = bcast63(cid2[ep]);
      p0 = lane == 0 ? x0 : p0;
      pid1 = lane == 0 ? x1 : pid1;
      pid2 = lane == 0 ? x2 : pid2;
    }
    const bool first = lane == 0 && e == 0;
    coll |= live[e] && !first && p0 == w0[e] && (pid1 != cid1[e] || pid2 != cid2[e]);
    H[e] = __ballot(live[e] && (first || p0 != w0[e]));
    Lv[e] = __ballot(live[e]);
  }
  if (__ballot(coll)) return false;

  uint64_t En[E], Em[E], c_v[E], c_t[E], c_m[E];
  bool cemit[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int en = e + 1 < E ? e + 1 : e;
    const bool nxt_head = lane < 63 ? ((H[e] >> (lane + 1)) & 1) : (e + 1 < E && (H[en] & 1));
    const bool nxt_live = lane < 63 ? ((Lv[e] >> (lane + 1)) & 1) : (e + 1 < E && (Lv[en] & 1));
    const bool ctail = live[e] && (nxt_head || !nxt_live);
    const int pos = lane + 64 * e;
    c_v[e] = c_t[e] = c_m[e] = 0;
    cemit[e] = false;
    if (ctail) {
      const int hl = seg_head<E>(H, e, lane);
      const uint32_t r0 = L.sidx[hl];
      if (knode[e]) {  // Counter::merge per node (type_counter.rs:60-84): the head's t is kept
        const uint64_t t0 = L.ccol[CC_T][r0];
        uint64_t v = L.ccol[CC_C2][r0];
        for (int q = hl + 1; q <= pos; ++q) {
          const uint32_t r = L.sidx[q];
          const uint64_t tt = L.ccol[CC_T][r], vv = L.ccol[CC_C2][r];
          v = tt > t0 ? vv : (tt == t0 ? imax64(v, vv) : v);
        }
        c_v[e] = v;
        c_t[e] = t0;
        const uint64_t mh = L.ccol[CC_META][r0];
        c_m[e] = meta_pack(0, meta_pos(mh), meta_src(mh));
        cemit[e] = true;
      } else {  // LWWHash::set chain (lwwhash.rs:87-107): the later candidate wins ties
        uint32_t w = r0;
        uint64_t tw = L.ccol[CC_T][r0];
        for (int q = hl + 1; q <= pos; ++q) {
          const uint32_t r = L.sidx[q];
          const uint64_t tr = L.ccol[CC_T][r];
          const bool later = !(tw > tr);
          w = later ? r : w;
          tw = later ? tr : tw;
        }
        c_t[e] = tw;
        c_m[e] = L.ccol[CC_META][w];
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
  uint32_t nbase = 0, mbase = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (cemit[e]) {
      const uint32_t crank = (knode[e] ? nbase : mbase) + lane_rank(knode[e] ? En[e] : Em[e]);
      const uint32_t o = (knode[e] ? nb0 : mb0) + crank;
      uint64_t* const* O = knode[e] ? A.no : A.mo;
      const uint32_t k = ckey[e];
      O[C_PKH][o] = L.okh[k];
      O[C_PKF][o] = L.okf[k];
      O[C_ID1][o] = cid1[e];
      O[C_ID2][o] = knode[e] ? c_v[e] : cid2[e];
      O[C_T][o] = c_t[e];
      O[C_META][o] = c_m[e];
      if (knode[e] && (L.ovm[k] & kVmaskMerged))
        atomicAdd((unsigned long long*)&L.osum[k], (unsigned long long)c_v[e]);
      atomicMin(&L.ocb[k], crank);
      atomicAdd(&L.ocnt[k], 1u);
    }
    nbase += __popcll(En[e]);
    mbase += __popcll(Em[e]);
  }
  wave_sync();
  co.nout = nbase;
  co.mout = mbase;
  co.orph = orph;
  co.gcm = gcm;
  return true;
}

// One bucket on one wave, up to 64*KE key rows. `spill` receives buckets over the key
// capacity (KE = 1: the wide kernel; KE = 2: the workgroup tier).
template <int KE>
__device__ __forceinline__ void wave_bucket(const WaveArgs& W, WaveLds<KE>& L, uint32_t b, int lane,
                                            uint32_t* spill_list, uint32_t* spill_count) {
  const BucketArgs& A = W.A;
  const uint32_t K = A.kcnt[b], N = A.ncnt[b], M = A.mcnt[b];
  auto push = [&](uint32_t* list, uint32_t* count) {
    if (lane == 0) list[atomicAdd(count, 1u)] = b;
  };
  constexpr uint32_t KC = WaveLds<KE>::KC, CC = WaveLds<KE>::CC;
  if (A.force_tier == 1 || A.force_tier == 2 || N + M > WaveLds<2>::CC || K > WaveLds<2>::KC) {
    push(W.big_list, W.big_count);
    return;
  }
  if (K > KC || N + M > CC || (KE == 1 && A.force_tier == 3)) {
    push(spill_list, spill_count);
    return;
  }
  const uint32_t kb = A.kbase[b], nb0 = A.nbase[b], mb0 = A.mbase[b];

  // ------------------------------------------------------------ 1. keys: load + sort
  // w1 = family:2 | pos:6 | src:48 | idx:7 (pos < 64, kMaxPos)
  uint64_t w0[KE], w1[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const uint32_t c = lane + 64 * e;
    w0[e] = ~0ull;
    w1[e] = ~0ull;
    if (c < K) {
      const uint32_t row = A.kp[kb + c];
      const uint64_t meta = A.k[K_META][row];
      w0[e] = A.k[K_KH][row];
      w1[e] = ((uint64_t)tag_family(meta_tag(meta)) << 61) | (meta_order(meta) << 7) | c;
      L.col[KC_CT][c] = A.k[K_CT][row];
      L.col[KC_UT][c] = A.k[K_UT][row];
      L.col[KC_DT][c] = A.k[K_DT][row];
      L.col[KC_META][c] = meta;
      L.col[KC_KF][c] = A.k[K_KF][row];
    }
  }
  wave_bitonic<KE>(w0, w1);
  uint32_t idx[KE], fam[KE];
  uint64_t kh[KE], kf[KE], Hk[KE];
  bool kin[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    idx[e] = (uint32_t)(w1[e] & 127);
    L.sidx[lane + 64 * e] = idx[e];
  }
  wave_sync();
  bool coll = false;
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const uint32_t pos = lane + 64 * e;
    kin[e] = pos < K;
    kh[e] = w0[e];
    fam[e] = (uint32_t)(w1[e] >> 61) & 3;
    kf[e] = kin[e] ? L.col[KC_KF][idx[e]] : 0;
    uint64_t pkh = shfl_up64(kh[e], 1), pkf = shfl_up64(kf[e], 1);
    uint32_t pfam = __shfl_up(fam[e], 1, 64);
    if (e > 0) {
      const int ep = e > 0 ? e - 1 : 0;
      const uint64_t x0 = bcast63(kh[ep]), x1 = bcast63(kf[ep]);
      const uint32_t x2 = __shfl(fam[ep], 63, 64);
      pkh = lane == 0 ? x0 : pkh;
      pkf = lane == 0 ? x1 : pkf;
      pfam = lane == 0 ? x2 : pfam;
    }
    coll |= kin[e] && pos > 0 && pkh == kh[e] && pkf != kf[e];  // 64-bit kh collision
    Hk[e] = __ballot(kin[e] && (pos == 0 || pkh != kh[e] || pfam != fam[e]));
  }
  if (__ballot(coll)) {
    push(W.big_list, W.big_count);
    return;
  }

  // ------------------------------------------------------------ 2. key folds (tail slots)
  const uint64_t last_bad = (A.flags & F_GC_DELETES) ? *A.last_bad : 0;
  uint64_t o_ct[KE], o_ut[KE], o_dt[KE], o_meta[KE], o_win[KE];
  uint32_t o_T[KE], orank[KE];
  bool emit[KE];
  unsigned long long st_conf = 0, st_dict = 0, st_dup = 0, st_gcd = 0;
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
      const uint32_t r0 = L.sidx[hl];
      const uint64_t m0 = L.col[KC_META][r0];
      const uint32_t T = meta_tag(m0);
      hp = meta_pos(m0);
      const uint64_t ct0 = L.col[KC_CT][r0], ut0 = L.col[KC_UT][r0], dt0 = L.col[KC_DT][r0];
      uint64_t ct = ct0, ut = ut0, dt = dt0;
      uint64_t win = meta_order(m0), lastm = m0;
      uint32_t nvalid = 1, conflicts = 0, dups = 0, prevpos = hp;
      vm = 1ull << hp;
      const uint64_t tl_ct = L.col[KC_CT][idx[e]];  // the segment's last row (side maps)
      bool gc_hit = fm == 2 && meta_order(m0) + 1 > last_bad && ct0 == tl_ct;
      for (int q = hl + 1; q <= pos; ++q) {
        const uint32_t r = L.sidx[q];
        const uint64_t m = L.col[KC_META][r];
        const uint32_t p = meta_pos(m);
        dups += p == prevpos;
        prevpos = p;
        lastm = m;
        if (fm != 0) {
          gc_hit |= fm == 2 && meta_order(m) + 1 > last_bad && L.col[KC_CT][r] == tl_ct;
          continue;
        }
        if (meta_tag(m) != T) {  // object.rs:80: type conflict, local kept
          ++conflicts;
          continue;
        }
        ++nvalid;
        vm |= 1ull << p;
        if (T == TAG_BYTES) {  // object.rs:69-77
          const uint64_t c2 = L.col[KC_CT][r];
          if (ct < c2) win = meta_order(m);
          ct = max(ct, c2);
          dt = max(dt, L.col[KC_DT][r]);
          ut = max(ut, L.col[KC_UT][r]);
        }
      }
      st_dup += dups;
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
        sum = (T == TAG_COUNTER && nvalid < 2) ? A.k[K_AUX][A.kp[kb + r0]] : 0;
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

  // ------------------------------------------------------------ 3-4. children
  ChildOut co;
  bool ok;
  if (N + M <= 64)
    ok = children_stage<1, KE>(A, L, lane, N, M, nb0, mb0, kout, co);
  else if (KE == 1 || N + M <= 128)
    ok = children_stage<2, KE>(A, L, lane, N, M, nb0, mb0, kout, co);
  else
    ok = children_stage<(KE == 1 ? 2 : 4), KE>(A, L, lane, N, M, nb0, mb0, kout, co);
  if (!ok) {  // id-hash collision: exact tier
    push(W.big_list, W.big_count);
    return;
  }

  // ------------------------------------------------------------ 5. key outputs
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    if (emit[e]) {
      const uint32_t r = orank[e], o = kb + r;
      A.ko[O_KH][o] = kh[e];
      A.ko[O_KF][o] = kf[e];
      A.ko[O_CT][o] = o_ct[e];
      A.ko[O_UT][o] = o_ut[e];
      A.ko[O_DT][o] = o_dt[e];
      A.ko[O_META][o] = o_meta[e];
      A.ko[O_WIN][o] = (fam[e] == 0 && o_T[e] == TAG_COUNTER) ? L.osum[r] : o_win[e];
      A.ko[O_CREF][o] = cref_pack(L.ocnt[r] ? L.ocb[r] : 0, L.ocnt[r]);
    }
  }
  if (lane == 0) {
    A.kout[b] = kout;
    A.nout[b] = co.nout;
    A.mout[b] = co.mout;
  }
  const unsigned long long s0 = wave_sum_u64(st_conf), s1 = wave_sum_u64(st_dict), s2 = wave_sum_u64(st_dup),
                           s3 = wave_sum_u64(co.orph), s4 = wave_sum_u64(st_gcd), s5 = wave_sum_u64(co.gcm);
  if (lane == 0) {
    if (s0) atomicAdd(&A.stats[ST_TYPE_CONFLICTS], s0);
    if (s1) atomicAdd(&A.stats[ST_DICT_MERGES], s1);
    if (s2) atomicAdd(&A.stats[ST_DUP_ROWS], s2);
    if (s3) atomicAdd(&A.stats[ST_ORPHANS], s3);
    if (s4) atomicAdd(&A.stats[ST_DELETES_GCED], s4);
    if (s5) atomicAdd(&A.stats[ST_MEMBERS_GCED], s5);
  }
}

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2). Remap so
// that XCD x runs one contiguous range of blocks: neighbouring buckets share a final
// partition segment, whose rows then stay in one L2.
__device__ __forceinline__ uint32_t xcd_block(uint32_t i, uint32_t G) {
  constexpr uint32_t kXcd = 8;
  const uint32_t q = G / kXcd, r = G % kXcd, x = i % kXcd, j = i / kXcd;
  return x * q + min(x, r) + j;
}

// Every bucket, one wave each (<= 64 key rows per wave).
__global__ void __launch_bounds__(kWavesPerWG * 64) bucket_wave_kernel(WaveArgs W) {
  __shared__ WaveLds<1> lds_all[kWavesPerWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t b = xcd_block(blockIdx.x, gridDim.x) * kWavesPerWG + wv;
  if (b >= W.nbuckets) return;
  wave_bucket<1>(W, lds_all[wv], b, lane, W.wide_list, W.wide_count);
}

// Buckets over bucket_wave_kernel's capacity (listed by it), persistent over the list.
__global__ void __launch_bounds__(kWavesPerWG * 64) bucket_wide_kernel(WaveArgs W) {
  __shared__ WaveLds<2> lds_all[kWavesPerWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t total = *W.wide_count;
  for (uint32_t i = blockIdx.x * kWavesPerWG + wv; i < total; i += gridDim.x * kWavesPerWG)
    wave_bucket<2>(W, lds_all[wv], W.wide_list[i], lane, W.big_list, W.big_count);
}

}  // namespace cdb
