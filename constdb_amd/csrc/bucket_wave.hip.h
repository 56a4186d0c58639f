// Wave-per-bucket merge kernel (gfx950, wave64) — the hot path of the merge.
//
// One 64-lane wave owns one bucket (<= 64 key rows and <= 64 child rows, one row per
// lane) and never synchronises with another wave:
//   1. keys: lane i loads row i (coalesced); a register bitonic network over __shfl_xor
//      sorts (kh, family|pos|src); equal kh with different kf (a 64-bit collision) hands
//      the bucket to the exact-comparator workgroup tier before anything is written;
//   2. key folds: the tail lane of each (key, family) segment replays the reference's
//      sequential fold over its segment (<= R rows, read from LDS in sorted order):
//        data     DB::merge_entry / Object::merge   (db.rs:31-43, object.rs:63-83)
//        expires / deletes: last (pos, src) wins   (db.rs:68-76), DB::gc (db.rs:82-95);
//   3. children: counter nodes and set/dict members share the lanes (a key has one type);
//      each finds its key by binary search over the wave's sorted output keys (LDS), is
//      kept if its element has the key's head type (object.rs:80) and, for members of a
//      non-head position, only if it is an add (SetIter/DictIter, lwwhash.rs:319-323);
//      sorted by (key rank, id hash, pos|src), folded per (key, node) with
//      Counter::merge's head-t rule (type_counter.rs:59-87) or per (key, member) with
//      LWWHash::set's later-wins-ties rule (lwwhash.rs:87-107);
//   4. counter sums (cal_sum, type_counter.rs:89-91) and child ranges; outputs are
//      written by the tail lanes (ballot + mbcnt ranks).
// Buckets over a wave's capacity go to the workgroup tier (bucket.hip.h) via a list.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bucket.hip.h"
#include "common.h"

namespace cdb {

constexpr int kWaveCap = 64;
constexpr int kWavesPerWG = 4;

struct WaveLds {
  uint64_t okh[kWaveCap], okf[kWaveCap], ovm[kWaveCap], osum[kWaveCap];
  uint32_t otp[kWaveCap], ocnt[kWaveCap], ocb[kWaveCap], sidx[kWaveCap];
  uint64_t col[6][kWaveCap];  // per-row staging, gathered through sidx after the sort
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

// Branch-free lexicographic (a0, a1) < (b0, b1).
__device__ __forceinline__ bool lt2(uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1) {
  return (a0 < b0) | ((a0 == b0) & (a1 < b1));
}

// Ascending bitonic sort of one (w0, w1, idx) element per lane; sentinels are all-ones.
__device__ __forceinline__ void wave_bitonic2(uint64_t& w0, uint64_t& w1, uint32_t& idx) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
      const uint64_t o0 = shfl_xor64(w0, j), o1 = shfl_xor64(w1, j);
      const uint32_t oi = __shfl_xor(idx, j, 64);
      const bool keep_min = ((lane & j) == 0) == ((lane & kk) == 0);
      const bool other_lt = lt2(o0, o1, w0, w1), mine_lt = lt2(w0, w1, o0, o1);
      const bool take = keep_min ? other_lt : mine_lt;
      w0 = take ? o0 : w0;
      w1 = take ? o1 : w1;
      idx = take ? oi : idx;
    }
  }
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits of mask below my lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
// Highest set bit of `mask` at or below `lane` (mask must have one there).
__device__ __forceinline__ int head_of(uint64_t mask, int lane) {
  const uint64_t m = mask & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
  return 63 - __clzll(m);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

struct WaveArgs {
  BucketArgs A;
  uint32_t nbuckets;
  uint32_t* big_list;   // buckets for the workgroup tier
  uint32_t* big_count;
};

enum { KC_CT = 0, KC_UT, KC_DT, KC_AUX, KC_META, KC_KF };  // key staging columns
enum { CC_ID1 = 0, CC_ID2, CC_V, CC_T, CC_META };           // child staging columns

__global__ void __launch_bounds__(kWavesPerWG * 64) bucket_wave_kernel(WaveArgs W) {
  __shared__ WaveLds lds_all[kWavesPerWG];
  const BucketArgs& A = W.A;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * kWavesPerWG + wv;
  if (b >= W.nbuckets) return;
  WaveLds& L = lds_all[wv];
  const uint32_t K = A.kcnt[b], N = A.ncnt[b], M = A.mcnt[b];
  auto bail = [&]() {
    if (lane == 0) W.big_list[atomicAdd(W.big_count, 1u)] = b;
  };
  if (K > kWaveCap || N + M > kWaveCap || A.force_tier >= 1) {
    bail();
    return;
  }
  const uint32_t kb = A.kbase[b], nb0 = A.nbase[b], mb0 = A.mbase[b];

  // ------------------------------------------------------------ 1. keys: load + sort
  const bool kin = lane < (int)K;
  uint64_t w0 = ~0ull, w1 = ~0ull;
  uint32_t idx = lane;
  if (kin) {
    const uint64_t meta = A.k[K_META][kb + lane];
    w0 = A.k[K_KH][kb + lane];
    w1 = ((uint64_t)tag_family(meta_tag(meta)) << 56) | meta_order(meta);
    L.col[KC_CT][lane] = A.k[K_CT][kb + lane];
    L.col[KC_UT][lane] = A.k[K_UT][kb + lane];
    L.col[KC_DT][lane] = A.k[K_DT][kb + lane];
    L.col[KC_AUX][lane] = A.k[K_AUX][kb + lane];
    L.col[KC_META][lane] = meta;
    L.col[KC_KF][lane] = A.k[K_KF][kb + lane];
  }
  wave_bitonic2(w0, w1, idx);
  L.sidx[lane] = idx;
  wave_sync();
  const uint64_t kh = w0;
  const uint32_t fam = (uint32_t)(w1 >> 56);
  const uint64_t kf = kin ? L.col[KC_KF][idx] : 0;
  const uint64_t pkh = shfl_up64(kh, 1), pkf = shfl_up64(kf, 1);
  const uint32_t pfam = __shfl_up(fam, 1, 64);
  if (__ballot(kin && lane > 0 && pkh == kh && pkf != kf)) {  // 64-bit kh collision
    bail();
    return;
  }
  const bool khead = kin && (lane == 0 || pkh != kh || pfam != fam);
  const uint64_t Hk = __ballot(khead);
  const bool ktail = kin && (lane == (int)K - 1 || ((Hk >> (lane + 1)) & 1));

  // ------------------------------------------------------------ 2. key folds (tail lanes)
  const uint64_t last_bad = (A.flags & F_GC_DELETES) ? *A.last_bad : 0;
  uint64_t o_ct = 0, o_ut = 0, o_dt = 0, o_meta = 0, o_win = 0, o_vm = 0, o_sum = 0;
  uint32_t o_T = 0, o_hp = 0;
  bool emit = false;
  unsigned long long st_conf = 0, st_dict = 0, st_dup = 0, st_orph = 0, st_gcd = 0, st_gcm = 0;
  if (ktail) {
    const int hl = head_of(Hk, lane);
    const uint32_t r0 = L.sidx[hl];
    const uint64_t m0 = L.col[KC_META][r0];
    const uint32_t T = meta_tag(m0), hp = meta_pos(m0);
    const uint64_t ct0 = L.col[KC_CT][r0], ut0 = L.col[KC_UT][r0], dt0 = L.col[KC_DT][r0];
    uint64_t ct = ct0, ut = ut0, dt = dt0;
    uint64_t win = meta_order(m0), vm = 1ull << hp, lastm = m0;
    uint32_t nvalid = 1, conflicts = 0, dups = 0, prevpos = hp;
    const uint64_t tl_ct = L.col[KC_CT][L.sidx[lane]];  // the segment's last row (side maps)
    bool gc_hit = fam == 2 && meta_order(m0) + 1 > last_bad && ct0 == tl_ct;
    for (int q = hl + 1; q <= lane; ++q) {
      const uint32_t r = L.sidx[q];
      const uint64_t m = L.col[KC_META][r];
      const uint32_t p = meta_pos(m);
      dups += p == prevpos;
      prevpos = p;
      lastm = m;
      if (fam != 0) {
        gc_hit |= fam == 2 && meta_order(m) + 1 > last_bad && L.col[KC_CT][r] == tl_ct;
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
    st_dup = dups;
    if (fam == 0) {
      st_conf = conflicts;
      if (T == TAG_DICT) st_dict = nvalid - 1;
      o_T = T;
      o_hp = hp;
      // non-Bytes objects keep the head's times (object.rs:68,78-79)
      o_ct = T == TAG_BYTES ? ct : ct0;
      o_ut = T == TAG_BYTES ? ut : ut0;
      o_dt = T == TAG_BYTES ? dt : dt0;
      o_meta = m0;
      o_win = T == TAG_BYTES ? win : 0;
      o_vm = vm | ((T == TAG_COUNTER && nvalid >= 2) ? kVmaskMerged : 0);
      o_sum = (T == TAG_COUNTER && nvalid < 2) ? L.col[KC_AUX][r0] : 0;  // load-time total
      emit = true;
    } else {  // expires / deletes: plain overwrite, the last (pos, src) wins
      const bool removed = fam == 2 && (A.flags & F_GC_DELETES) && gc_hit;
      o_T = meta_tag(lastm);
      o_hp = meta_pos(lastm);
      o_ct = tl_ct;
      o_meta = lastm;
      o_win = meta_order(lastm);
      emit = !removed;
      st_gcd = removed ? 1 : 0;
    }
  }
  const uint64_t Ek = __ballot(emit);
  const uint32_t kout = __popcll(Ek);
  const uint32_t orank = lane_rank(Ek);
  if (emit) {
    L.okh[orank] = kh;
    L.okf[orank] = kf;
    L.ovm[orank] = o_vm;
    L.otp[orank] = o_T | (o_hp << 8);
    L.osum[orank] = o_sum;
    L.ocnt[orank] = 0;
    L.ocb[orank] = kNone;
  }
  wave_sync();

  // ------------------------------------------------------------ 3. children: load, find key, sort
  const bool cin = lane < (int)(N + M);
  const bool isnode_row = lane < (int)N;
  w0 = ~0ull;
  w1 = ~0ull;
  idx = lane;
  if (cin) {
    const uint64_t* const* C = isnode_row ? A.nd : A.mb;
    const uint32_t row = isnode_row ? nb0 + lane : mb0 + (lane - N);
    const uint64_t cpkh = C[C_PKH][row], cpkf = C[C_PKF][row];
    const uint64_t id1 = C[C_ID1][row], c2 = C[C_ID2][row], t = C[C_T][row], m = C[C_META][row];
    L.col[CC_ID1][lane] = id1;
    L.col[CC_ID2][lane] = isnode_row ? 0 : c2;
    L.col[CC_V][lane] = isnode_row ? c2 : 0;
    L.col[CC_T][lane] = t;
    L.col[CC_META][lane] = m;
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
      const bool type_ok = isnode_row ? KT == TAG_COUNTER : (KT == TAG_SET || KT == TAG_DICT);
      const bool elem_ok = (L.ovm[lo] >> p) & 1;
      const bool cand = isnode_row || meta_tag(m) == KIND_ADD || p == khp;  // remote dels ignored
      if (type_ok && elem_ok && cand) key = lo;
    } else {
      st_orph = 1;
    }
    if (key != 255) {
      const uint64_t ih = isnode_row ? mix64(id1) : id1;
      w0 = ((uint64_t)key << 56) | (ih >> 8);
      w1 = meta_order(m);
    }
  }
  wave_bitonic2(w0, w1, idx);
  L.sidx[lane] = idx;
  wave_sync();
  const bool live = (w0 >> 56) < 255u;  // valid rows sort before invalid and empty lanes
  const uint64_t cid1 = live ? L.col[CC_ID1][idx] : 0, cid2 = live ? L.col[CC_ID2][idx] : 0;
  const uint64_t p0 = shfl_up64(w0, 1), pid1 = shfl_up64(cid1, 1), pid2 = shfl_up64(cid2, 1);
  if (__ballot(live && lane > 0 && p0 == w0 && (pid1 != cid1 || pid2 != cid2))) {  // id-hash collision
    bail();
    return;
  }
  const bool chead = live && (lane == 0 || p0 != w0);
  const uint64_t Hc = __ballot(chead), Lv = __ballot(live);
  const bool ctail = live && (lane == 63 || ((Hc >> (lane + 1)) & 1) || !((Lv >> (lane + 1)) & 1));

  // ------------------------------------------------------------ 4. child folds (tail lanes)
  const uint32_t ckey = (uint32_t)(w0 >> 56) & 63;
  const bool knode = live && (L.otp[ckey] & 0xFF) == TAG_COUNTER;
  uint64_t c_v = 0, c_t = 0, c_m = 0;
  bool cemit = false;
  if (ctail) {
    const int hl = head_of(Hc, lane);
    const uint32_t r0 = L.sidx[hl];
    if (knode) {  // Counter::merge per node (type_counter.rs:60-84): the head's t is kept
      const uint64_t t0 = L.col[CC_T][r0];
      uint64_t v = L.col[CC_V][r0];
      for (int q = hl + 1; q <= lane; ++q) {
        const uint32_t r = L.sidx[q];
        const uint64_t tt = L.col[CC_T][r], vv = L.col[CC_V][r];
        v = tt > t0 ? vv : (tt == t0 ? imax64(v, vv) : v);
      }
      c_v = v;
      c_t = t0;
      const uint64_t mh = L.col[CC_META][r0];
      c_m = meta_pack(0, meta_pos(mh), meta_src(mh));
      cemit = true;
    } else {  // LWWHash::set chain (lwwhash.rs:87-107): the later candidate wins ties
      uint32_t w = r0;
      uint64_t tw = L.col[CC_T][r0];
      for (int q = hl + 1; q <= lane; ++q) {
        const uint32_t r = L.sidx[q];
        const uint64_t tr = L.col[CC_T][r];
        const bool later = !(tw > tr);
        w = later ? r : w;
        tw = later ? tr : tw;
      }
      c_t = tw;
      c_m = L.col[CC_META][w];
      cemit = true;
      if ((A.flags & F_GC_MEMBERS) && meta_tag(c_m) == KIND_DEL && tw < A.gc_wm) {
        cemit = false;
        st_gcm = 1;
      }
    }
  }
  const uint64_t En = __ballot(cemit && knode), Em = __ballot(cemit && !knode);
  const uint32_t nout = __popcll(En), mout = __popcll(Em);
  if (cemit) {
    const uint32_t crank = lane_rank(knode ? En : Em);
    const uint32_t o = (knode ? nb0 : mb0) + crank;
    uint64_t* const* O = knode ? A.no : A.mo;
    O[C_PKH][o] = L.okh[ckey];
    O[C_PKF][o] = L.okf[ckey];
    O[C_ID1][o] = cid1;
    O[C_ID2][o] = knode ? c_v : cid2;
    O[C_T][o] = c_t;
    O[C_META][o] = c_m;
    if (knode && (L.ovm[ckey] & kVmaskMerged)) atomicAdd((unsigned long long*)&L.osum[ckey], (unsigned long long)c_v);
    atomicMin(&L.ocb[ckey], crank);
    atomicAdd(&L.ocnt[ckey], 1u);
  }
  wave_sync();

  // ------------------------------------------------------------ 5. key outputs
  if (emit) {
    const uint32_t o = kb + orank;
    A.ko[O_KH][o] = kh;
    A.ko[O_KF][o] = kf;
    A.ko[O_CT][o] = o_ct;
    A.ko[O_UT][o] = o_ut;
    A.ko[O_DT][o] = o_dt;
    A.ko[O_META][o] = o_meta;
    A.ko[O_WIN][o] = (fam == 0 && o_T == TAG_COUNTER) ? L.osum[orank] : o_win;
    A.ko[O_CREF][o] = cref_pack(L.ocnt[orank] ? L.ocb[orank] : 0, L.ocnt[orank]);
  }
  if (lane == 0) {
    A.kout[b] = kout;
    A.nout[b] = nout;
    A.mout[b] = mout;
  }
  const unsigned long long s0 = wave_sum_u64(st_conf), s1 = wave_sum_u64(st_dict), s2 = wave_sum_u64(st_dup),
                           s3 = wave_sum_u64(st_orph), s4 = wave_sum_u64(st_gcd), s5 = wave_sum_u64(st_gcm);
  if (lane == 0) {
    if (s0) atomicAdd(&A.stats[ST_TYPE_CONFLICTS], s0);
    if (s1) atomicAdd(&A.stats[ST_DICT_MERGES], s1);
    if (s2) atomicAdd(&A.stats[ST_DUP_ROWS], s2);
    if (s3) atomicAdd(&A.stats[ST_ORPHANS], s3);
    if (s4) atomicAdd(&A.stats[ST_DELETES_GCED], s4);
    if (s5) atomicAdd(&A.stats[ST_MEMBERS_GCED], s5);
  }
}

}  // namespace cdb
