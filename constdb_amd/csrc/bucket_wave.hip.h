// Wave-per-bucket merge kernel (gfx950, wave64) — the hot path of the merge.
//
// One 64-lane wave owns one small bucket (<= 64 key rows, <= 64 counter-node rows,
// <= 64 set/dict-member rows; one row per lane) and never synchronises with another
// wave. Per family:
//   load  : lane i loads row i of every column (coalesced within the bucket);
//   sort  : register bitonic network over __shfl_xor (21 compare-exchange stages) on a
//           multi-word key — keys by (kh, kf, family|pos|src), nodes by (key rank, node,
//           pos|src), members by (key rank, mh, mf, pos|src);
//   fold  : segmented inclusive wave scans (6 shuffle steps) implement the reference's
//           sequential folds as associative operators:
//             Bytes  (object.rs:69-77)      (ct, winner) <- later strictly-greater ct wins,
//                                            max ut, max dt;
//             Counter node (type_counter.rs:60-84) element -> {ID, SET(v), MAX(v)} monoid
//                                            relative to the head's t, applied to v0;
//             Set/Dict member (lwwhash.rs:87-107) (t, winner) <- later greater-or-equal t;
//             expires/deletes (db.rs:68-76) last (pos, src) wins; DB::gc (db.rs:82-95);
//   emit  : the tail lane of each segment writes the output row (ballot + mbcnt ranks).
// Buckets that exceed a wave's capacity are appended to a list for the workgroup kernel.
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
  uint32_t otp[kWaveCap], ocnt[kWaveCap], ocb[kWaveCap];
  uint64_t col[kKeyCols][kWaveCap];  // staging for the gather after the sort
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
__device__ __forceinline__ uint64_t shfl_down64(uint64_t v, int d) {
  return (uint64_t)__shfl_down((unsigned long long)v, d, 64);
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int l) { return (uint64_t)__shfl((unsigned long long)v, l, 64); }

template <int NW>
__device__ __forceinline__ bool lex_less(const uint64_t (&a)[NW], const uint64_t (&b)[NW]) {
#pragma unroll
  for (int w = 0; w < NW; ++w)
    if (a[w] != b[w]) return a[w] < b[w];
  return false;
}

// Ascending bitonic sort of one element per lane (sentinel lanes carry all-ones keys).
template <int NW>
__device__ __forceinline__ void wave_bitonic(uint64_t (&k)[NW], uint32_t& idx) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
      uint64_t o[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) o[w] = shfl_xor64(k[w], j);
      const uint32_t oi = __shfl_xor(idx, j, 64);
      const bool lower = (lane & j) == 0, up = (lane & kk) == 0;
      const bool take = (lower == up) ? lex_less<NW>(o, k) : lex_less<NW>(k, o);
      if (take) {
#pragma unroll
        for (int w = 0; w < NW; ++w) k[w] = o[w];
        idx = oi;
      }
    }
  }
}

// Lane index of my segment's head (inclusive max-scan of head ? lane : 0).
__device__ __forceinline__ int seg_head_lane(bool head) {
  const int lane = threadIdx.x & 63;
  int x = head ? lane : 0;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) x = max(x, __shfl_up(x, d, 64));
  return x;
}
// Lane index of my segment's tail (suffix min-scan of tail ? lane : 63).
__device__ __forceinline__ int seg_tail_lane(bool tail) {
  const int lane = threadIdx.x & 63;
  int x = tail ? lane : 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_down(x, d, 64);
    if (lane + d < 64) x = min(x, y);
  }
  return x;
}

// Segmented inclusive scans within [hl, lane].
__device__ __forceinline__ uint64_t seg_max_u64(uint64_t x, int hl) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = shfl_up64(x, d);
    if (lane - d >= hl) x = max(x, y);
  }
  return x;
}
__device__ __forceinline__ uint64_t seg_or_u64(uint64_t x, int hl) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = shfl_up64(x, d);
    if (lane - d >= hl) x |= y;
  }
  return x;
}
__device__ __forceinline__ uint32_t seg_sum_u32(uint32_t x, int hl) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane - d >= hl) x += y;
  }
  return x;
}
// (value, winner) pairs: later element replaces when its value is > (strict) or >= (ge).
template <bool GE>
__device__ __forceinline__ void seg_argmax(uint64_t& v, uint32_t& w, int hl) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t yv = shfl_up64(v, d);
    const uint32_t yw = __shfl_up(w, d, 64);
    if (lane - d >= hl) {
      // combine(left = y, right = mine): right wins iff right beats left
      const bool right_wins = GE ? (v >= yv) : (v > yv);
      if (!right_wins) { v = yv; w = yw; }
    }
  }
}
// Counter element functions {ID=0, SET=1, MAX=2} with constant c; compose left then right.
__device__ __forceinline__ void seg_counter(uint32_t& kind, uint64_t& c, int hl) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t yk = __shfl_up(kind, d, 64);
    const uint64_t yc = shfl_up64(c, d);
    if (lane - d >= hl) {
      if (kind == 0) { kind = yk; c = yc; }                      // ID after y = y
      else if (kind == 2 && yk != 0) { kind = yk; c = imax64(yc, c); }  // MAX after SET/MAX
      // SET after anything = SET (unchanged)
    }
  }
}

__device__ __forceinline__ uint32_t lane_rank(bool pred) {  // exclusive ballot rank
  const uint64_t m = __ballot(pred);
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

struct WaveArgs {
  BucketArgs A;
  uint32_t nbuckets;
  uint32_t* big_list;   // buckets for the workgroup kernel
  uint32_t* big_count;
};

__global__ void __launch_bounds__(kWavesPerWG * 64) bucket_wave_kernel(WaveArgs W) {
  __shared__ WaveLds lds_all[kWavesPerWG];
  const BucketArgs& A = W.A;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * kWavesPerWG + wv;
  if (b >= W.nbuckets) return;
  WaveLds& L = lds_all[wv];
  const uint32_t K = A.kcnt[b], N = A.ncnt[b], M = A.mcnt[b];
  if (K > kWaveCap || N > kWaveCap || M > kWaveCap || A.force_tier >= 1) {
    if (lane == 0) W.big_list[atomicAdd(W.big_count, 1u)] = b;
    return;
  }
  const uint32_t kb = A.kbase[b];
  unsigned long long st_conf = 0, st_dict = 0, st_dup = 0, st_orph = 0, st_gcd = 0, st_gcm = 0;

  // ------------------------------------------------------------ keys
  const bool kin = lane < (int)K;
  uint64_t w3[3];
  uint32_t idx = lane;
  {
    uint64_t kh = ~0ull, kf = ~0ull, meta = ~0ull;
    if (kin) {
      kh = A.k[K_KH][kb + lane];
      kf = A.k[K_KF][kb + lane];
      meta = A.k[K_META][kb + lane];
      L.col[K_CT][lane] = A.k[K_CT][kb + lane];
      L.col[K_UT][lane] = A.k[K_UT][kb + lane];
      L.col[K_DT][lane] = A.k[K_DT][kb + lane];
      L.col[K_AUX][lane] = A.k[K_AUX][kb + lane];
      L.col[K_META][lane] = meta;
    }
    w3[0] = kh;
    w3[1] = kf;
    w3[2] = kin ? ((uint64_t)tag_family(meta_tag(meta)) << 56) | meta_order(meta) : ~0ull;
  }
  wave_bitonic<3>(w3, idx);
  wave_sync();
  const uint64_t kh = w3[0], kf = w3[1];
  const uint32_t fam = (uint32_t)(w3[2] >> 56);
  uint64_t meta = 0, ct = 0, ut = 0, dt = 0, aux = 0;
  if (kin) {
    meta = L.col[K_META][idx];
    ct = L.col[K_CT][idx];
    ut = L.col[K_UT][idx];
    dt = L.col[K_DT][idx];
    aux = L.col[K_AUX][idx];
  }
  const uint64_t pkh = shfl_up64(kh, 1), pkf = shfl_up64(kf, 1);
  const uint32_t pfam = __shfl_up(fam, 1, 64);
  const bool khead = kin && (lane == 0 || pkh != kh || pkf != kf || pfam != fam);
  const bool nxt_head = __shfl_down((int)khead, 1, 64) != 0;
  const bool ktail = kin && (lane == (int)K - 1 || nxt_head);
  const int hl = seg_head_lane(khead);
  const int tl = seg_tail_lane(ktail);
  const uint32_t tag = meta_tag(meta), pos = meta_pos(meta);
  // duplicate rows (same key twice at one pos): never written by db.rs:122-136
  const uint64_t pmeta = shfl_up64(meta, 1);  // shuffles stay in wave-uniform control flow
  if (kin && !khead && meta_pos(pmeta) == pos) ++st_dup;
  const uint32_t T = __shfl(tag, hl, 64);
  const uint32_t hp = __shfl(pos, hl, 64);
  const bool data = fam == 0;
  const bool valid = kin && data && tag == T;
  // Bytes: (ct, winner) with strictly-greater replacement; ut/dt maxima; validity mask
  uint64_t bct = valid ? ct : 0;
  uint32_t bwin = lane;
  seg_argmax<false>(bct, bwin, hl);
  const uint64_t mut = seg_max_u64(valid ? ut : 0, hl), mdt = seg_max_u64(valid ? dt : 0, hl);
  uint64_t vm = seg_or_u64(valid ? (1ull << pos) : 0, hl);
  const uint32_t nvalid = seg_sum_u32(valid ? 1u : 0u, hl);
  // deletes GC (db.rs:82-95): removed iff a popped garbage entry carries the final t
  const uint64_t t_last = shfl64(ct, tl);
  const uint64_t last_bad = (A.flags & F_GC_DELETES) ? *A.last_bad : 0;
  const bool gc_hit = kin && fam == 2 && (A.flags & F_GC_DELETES) && meta_order(meta) + 1 > last_bad && ct == t_last;
  const bool gc_any = seg_or_u64(gc_hit ? 1 : 0, hl) != 0;
  const bool emit = ktail && !(fam == 2 && gc_any);
  if (ktail && fam == 2 && gc_any) ++st_gcd;
  if (ktail && data) {
    const uint32_t seglen = lane - hl + 1;
    st_conf += seglen - nvalid;
    if (T == TAG_DICT) st_dict += nvalid - 1;
  }
  const uint32_t orank = lane_rank(emit);
  const uint32_t kout = __popcll(__ballot(emit));
  const uint64_t hmeta = shfl64(meta, hl);
  const uint64_t hct = shfl64(ct, hl), hut = shfl64(ut, hl), hdt = shfl64(dt, hl), haux = shfl64(aux, hl);
  const uint64_t wmeta = shfl64(meta, (int)bwin);
  if (emit) {
    uint64_t oct, out_, odt, owin, ometa;
    if (!data) {  // expires / deletes: plain overwrite, the last (pos, src) wins
      oct = ct;
      out_ = odt = 0;
      ometa = meta;
      owin = meta_order(meta);
    } else if (T == TAG_BYTES) {
      oct = bct;
      out_ = mut;
      odt = mdt;
      ometa = hmeta;
      owin = meta_order(wmeta);
    } else {  // Counter / Set / Dict keep the head's times (object.rs:68,78-79)
      oct = hct;
      out_ = hut;
      odt = hdt;
      ometa = hmeta;
      owin = 0;
    }
    if (data && T == TAG_COUNTER && nvalid >= 2) vm |= kVmaskMerged;
    const uint32_t o = kb + orank;
    A.ko[O_KH][o] = kh;
    A.ko[O_KF][o] = kf;
    A.ko[O_CT][o] = oct;
    A.ko[O_UT][o] = out_;
    A.ko[O_DT][o] = odt;
    A.ko[O_META][o] = ometa;
    A.ko[O_WIN][o] = owin;
    L.okh[orank] = kh;
    L.okf[orank] = kf;
    L.ovm[orank] = vm;
    L.otp[orank] = (data ? T : meta_tag(meta)) | (hp << 8);
    L.osum[orank] = (data && T == TAG_COUNTER && nvalid < 2) ? haux : 0;  // load-time total
    L.ocnt[orank] = 0;
    L.ocb[orank] = kNone;
  }
  wave_sync();

  // ------------------------------------------------------------ children
  uint32_t couts[2];
#pragma unroll
  for (int famc = 0; famc < 2; ++famc) {
    const bool nodes = famc == 0;
    const uint32_t n = nodes ? N : M, base = nodes ? A.nbase[b] : A.mbase[b];
    const uint64_t* const* C = nodes ? A.nd : A.mb;
    uint64_t* const* O = nodes ? A.no : A.mo;
    const bool in = lane < (int)n;
    uint64_t cpkh = 0, cpkf = 0, c1 = 0, c2 = 0, ct2 = 0, cm = 0;
    uint32_t key = 255;
    if (in) {
      cpkh = C[C_PKH][base + lane];
      cpkf = C[C_PKF][base + lane];
      c1 = C[C_ID1][base + lane];
      c2 = C[C_ID2][base + lane];
      ct2 = C[C_T][base + lane];
      cm = C[C_META][base + lane];
      L.col[0][lane] = c2;
      L.col[1][lane] = ct2;
      L.col[2][lane] = cm;
      uint32_t lo = 0, hi = kout;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.okh[mid] < cpkh || (L.okh[mid] == cpkh && L.okf[mid] < cpkf)) lo = mid + 1;
        else hi = mid;
      }
      if (lo < kout && L.okh[lo] == cpkh && L.okf[lo] == cpkf && (L.otp[lo] & 0xFF) <= TAG_SET) {
        const uint32_t KT = L.otp[lo] & 0xFF, khp = L.otp[lo] >> 8, p = meta_pos(cm);
        const bool type_ok = nodes ? KT == TAG_COUNTER : (KT == TAG_SET || KT == TAG_DICT);
        const bool elem_ok = (L.ovm[lo] >> p) & 1;
        const bool cand = nodes || meta_tag(cm) == KIND_ADD || p == khp;  // remote dels ignored
        if (type_ok && elem_ok && cand) key = lo;
      } else {
        ++st_orph;
      }
    }
    wave_sync();
    uint32_t cidx = lane;
    uint32_t cur_key;
    uint64_t id1, id2;
    if (nodes) {
      uint64_t w[3] = {in ? (uint64_t)key : ~0ull, in ? c1 : ~0ull, in ? meta_order(cm) : ~0ull};
      wave_bitonic<3>(w, cidx);
      cur_key = (uint32_t)w[0];
      id1 = w[1];
      id2 = 0;
    } else {
      uint64_t w[4] = {in ? (uint64_t)key : ~0ull, in ? c1 : ~0ull, in ? c2 : ~0ull, in ? meta_order(cm) : ~0ull};
      wave_bitonic<4>(w, cidx);
      cur_key = (uint32_t)w[0];
      id1 = w[1];
      id2 = w[2];
    }
    const bool live = lane < (int)n && cur_key < 255u;
    uint64_t v = 0, t = 0, m = 0;
    if (lane < (int)n) {
      v = L.col[0][cidx];
      t = L.col[1][cidx];
      m = L.col[2][cidx];
    }
    const uint32_t pk = __shfl_up(cur_key, 1, 64);
    const uint64_t p1 = shfl_up64(id1, 1), p2 = shfl_up64(id2, 1);
    const bool chead = live && (lane == 0 || pk != cur_key || p1 != id1 || p2 != id2);
    const bool cnext = __shfl_down((int)chead, 1, 64) != 0;
    const bool clast_live = __shfl_down((int)live, 1, 64) != 0;
    const bool ctail = live && (lane == 63 || cnext || !clast_live);
    const int chl = seg_head_lane(chead);
    uint64_t outv, outt, outm;
    bool cemit;
    if (nodes) {  // Counter::merge per (key, node): head (v0, t0), later elements as functions
      const uint64_t t0 = shfl64(t, chl), v0 = shfl64(v, chl);
      uint32_t kind = 0;
      uint64_t c = 0;
      if (live && !chead) {
        if (t > t0) { kind = 1; c = v; }
        else if (t == t0) { kind = 2; c = v; }
      }
      seg_counter(kind, c, chl);
      outv = kind == 1 ? c : (kind == 2 ? imax64(v0, c) : v0);
      outt = t0;
      outm = meta_pack(0, meta_pos(shfl64(m, chl)), meta_src(shfl64(m, chl)));
      cemit = ctail;
    } else {  // LWWHash::set chain: the later candidate wins ties
      uint64_t tv = t;
      uint32_t wl = lane;
      seg_argmax<true>(tv, wl, chl);
      outv = tv;
      outt = tv;
      outm = shfl64(m, (int)wl);
      cemit = ctail;
      if (cemit && (A.flags & F_GC_MEMBERS) && meta_tag(outm) == KIND_DEL && tv < A.gc_wm) {
        cemit = false;
        ++st_gcm;
      }
    }
    // every lane must take part in the shuffles above; emission below
    const uint32_t crank = lane_rank(cemit);
    couts[famc] = __popcll(__ballot(cemit));
    if (cemit) {
      const uint32_t o = base + crank;
      O[C_PKH][o] = L.okh[cur_key];
      O[C_PKF][o] = L.okf[cur_key];
      O[C_ID1][o] = id1;
      if (nodes) {
        O[C_ID2][o] = outv;
        O[C_T][o] = outt;
        if (L.ovm[cur_key] & kVmaskMerged) atomicAdd((unsigned long long*)&L.osum[cur_key], (unsigned long long)outv);
      } else {
        O[C_ID2][o] = id2;
        O[C_T][o] = outt;
      }
      O[C_META][o] = outm;
      atomicMin(&L.ocb[cur_key], crank);
      atomicAdd(&L.ocnt[cur_key], 1u);
    }
    wave_sync();
  }

  // ------------------------------------------------------------ per-key finish
  if (lane < (int)kout) {
    const uint32_t o = kb + lane;
    if ((L.otp[lane] & 0xFF) == TAG_COUNTER) A.ko[O_WIN][o] = L.osum[lane];
    A.ko[O_CREF][o] = cref_pack(L.ocnt[lane] ? L.ocb[lane] : 0, L.ocnt[lane]);
  }
  if (lane == 0) {
    A.kout[b] = kout;
    A.nout[b] = couts[0];
    A.mout[b] = couts[1];
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
