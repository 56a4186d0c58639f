// Fused per-bucket merge kernel for gfx950.
//
// One workgroup owns one bucket (all key rows whose kh falls in it, plus every counter
// node and set/dict member row whose parent key does) and runs the reference's fold for
// every key of the bucket at once:
//   1. key rows: LDS counting sort on the next 11 bits of kh, per-run insertion sort on
//      (kh, kf, family, pos, src); segment = one key of one family;
//   2. segment folds: DB::merge_entry/Object::merge (db.rs:31-43, object.rs:63-83) for
//      data rows, last-pos-wins for expires/deletes (db.rs:68-76), DB::gc's LIFO rule for
//      deletes (db.rs:82-95);
//   3. counter nodes and set/dict members: each row finds its key in the bucket's sorted
//      key table (LDS binary search), is kept only if its element has the key's head
//      type (object.rs:80), members of non-head positions keep only adds
//      (lwwhash.rs:319-323 via SetIter); rows are sorted by (key, id, pos, src) and
//      folded per (key, node) with Counter::merge's rule (type_counter.rs:59-87) or per
//      (key, member) with LWWHash::set's rule (lwwhash.rs:87-107);
//   4. counter sums (cal_sum, type_counter.rs:89-91) and child ranges per key.
// Scratch arrays live in LDS (fast path) or in a global scratch slab (buckets over the
// LDS capacity: same code, Scratch points elsewhere).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cdb {

constexpr int kBktThreads = 512;
constexpr int kCapK = 1024;    // key rows per bucket (LDS path)
constexpr int kCapC = 1024;    // node rows / member rows per bucket (LDS path)
constexpr int kDigBits = 11;   // key sub-digit bits for the counting sort
constexpr int kDig = 1 << kDigBits;
constexpr int kRunMax = 32;    // longest run sorted by one lane (else bitonic)
constexpr uint32_t kNone = 0xFFFFFFFFu;

enum Stat {
  ST_TYPE_CONFLICTS = 0, ST_DICT_MERGES, ST_DELETES_GCED, ST_MEMBERS_GCED, ST_DUP_ROWS,
  ST_ORPHANS, ST_HOT, ST_WIDE, ST_HOT_SLOW, ST_HOT_MERGED, ST_PIPE, ST_PIPE_UNITS, ST_COUNT
};
// Statistics are counted into kStatShards shards of kStatStride u64 (one 128-B line each):
// millions of waves adding to ONE word serialise at its memory-side atomic unit.
constexpr int kStatShards = 512, kStatStride = 16;
__device__ __forceinline__ unsigned long long* stat_shard(unsigned long long* stats) {
  return stats + (size_t)(blockIdx.x & (kStatShards - 1)) * kStatStride;
}
enum : uint32_t { F_DICT_STRICT = 1, F_GC_DELETES = 2, F_GC_MEMBERS = 4 };

struct BucketArgs {
  // Partitioned rows, AoS: key row r is kr[r * kKeyStride + K_*], node / member row r is
  // nr / mr[r * kChildStride + C_*].
  const uint64_t *kr, *nr, *mr;
  // Row permutations: the final partition level is index-only, so bucket b's i-th key row
  // is row kp[kbase[b] + i] (rows of one bucket lie in one small, cache-resident segment).
  const uint32_t *kp, *np, *mp;
  const uint32_t *kbase, *kcnt, *nbase, *ncnt, *mbase, *mcnt;
  uint64_t nbuckets;          // bucket(h) = floor((h << key_shift) * nbuckets / 2^64)
  // Sparse-by-bucket outputs, AoS: key output row o is kos[o * kKeyOutCols + O_*] (one 64-B
  // line), node / member output row o is nos / mos[o * kChildStride + C_*] (48 B). Whole rows
  // are written and later read by the compaction with 16-B accesses.
  uint64_t *kos, *nos, *mos;
  uint32_t *kout, *nout, *mout;
  uint32_t flags;
  uint32_t force_tier;
  int key_shift;
  // bucket b's smallest hash is >= b * bw (bw = floor((2^64 - 1) / nbuckets)) and its hashes span
  // less than 2^(44 + rel_shift): the wave kernels order a bucket's keys by the 44 leading bits of
  // (h << key_shift) - b * bw (exact key-hash order when rel_shift == 0, i.e. nbuckets > ~2^21)
  uint64_t bw;
  int rel_shift;
  uint64_t gc_wm;
  const uint64_t* last_bad;   // (pos,src)+1 of the newest garbage entry with t > wm; 0 = none
  unsigned long long* stats;
  uint32_t* hot_list;
  uint32_t* hot_count;
  const uint32_t* hot_in;     // hot kernel: bucket ids to process
  uint64_t* hot_scratch;      // hot kernel: global scratch slab
  const uint64_t* hot_scratch_off;  // per hot bucket, u64 offset into the slab
};

__device__ __forceinline__ uint64_t kget(const BucketArgs& A, int c, uint32_t r) {
  return A.kr[(uint64_t)r * kKeyStride + c];
}
__device__ __forceinline__ uint64_t cget(const uint64_t* C, int c, uint32_t r) {
  return C[(uint64_t)r * kChildStride + c];
}

// Scratch: every array the bucket algorithm needs, wherever it lives.
struct Scratch {
  // key phase
  uint64_t *kh, *kf, *meta;  // capacity ck
  uint32_t *idx, *rk, *flag, *rank;  // capacity pk (pow2 >= ck) for idx
  uint32_t* cnt;             // capacity max(kDig, cc + 1) + 1
  // per output key (sorted): capacity ck
  uint64_t *okh, *okf, *ovm, *osum;
  uint32_t *otp, *ocb, *occ;
  // child phase: capacity cc (idx: pow2 >= cc)
  uint64_t *c1, *c2, *cm, *rt, *rm;
  uint32_t *ck, *cidx, *crk, *cflag, *crank;
  unsigned long long* st;    // ST_COUNT counters
  uint32_t* misc;            // [0] need-bitonic flag, [1] total
};

__device__ __forceinline__ uint32_t pow2_ceil(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Exclusive scan in place over a[0..L) by the whole workgroup; returns the total.
__device__ uint32_t wg_scan(uint32_t* a, uint32_t L, uint32_t* tmp /* >= 16 */) {
  const int nt = blockDim.x, t = threadIdx.x;
  const uint32_t per = (L + nt - 1) / nt;
  const uint32_t b0 = t * per, b1 = min(L, b0 + per);
  uint32_t s = 0;
  for (uint32_t i = b0; i < b1; ++i) s += a[i];
  const int lane = t & 63, w = t >> 6;
  uint32_t incl = s;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  __syncthreads();
  if (lane == 63) tmp[w] = incl;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int i = 0; i < nt / 64; ++i) {
    if (i < w) off += tmp[i];
    tot += tmp[i];
  }
  uint32_t run = off + incl - s;
  for (uint32_t i = b0; i < b1; ++i) {
    const uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
  __syncthreads();
  return tot;
}

struct KeyLess {
  const Scratch& S;
  int shift;  // order by (kh << shift, kh, ...): monotone with the counting-sort digit
  __device__ bool operator()(uint32_t a, uint32_t b) const {
    if (a == kNone) return false;
    if (b == kNone) return true;
    const uint64_t sa = S.kh[a] << shift, sb = S.kh[b] << shift;
    if (sa != sb) return sa < sb;
    if (S.kh[a] != S.kh[b]) return S.kh[a] < S.kh[b];
    if (S.kf[a] != S.kf[b]) return S.kf[a] < S.kf[b];
    const uint32_t fa = tag_family(meta_tag(S.meta[a])), fb = tag_family(meta_tag(S.meta[b]));
    if (fa != fb) return fa < fb;
    return meta_order(S.meta[a]) < meta_order(S.meta[b]);
  }
};
struct ChildLess {
  const Scratch& S;
  __device__ bool operator()(uint32_t a, uint32_t b) const {
    if (a == kNone) return false;
    if (b == kNone) return true;
    if (S.ck[a] != S.ck[b]) return S.ck[a] < S.ck[b];
    if (S.c1[a] != S.c1[b]) return child_order(S.c1[a]) < child_order(S.c1[b]);
    if (S.c2[a] != S.c2[b]) return S.c2[a] < S.c2[b];
    return meta_order(S.cm[a]) < meta_order(S.cm[b]);
  }
};

// Bitonic sort of idx[0..n) (padded to a power of two with kNone) by `less`.
template <class Less>
__device__ void wg_bitonic(uint32_t* idx, uint32_t n, Less less) {
  const uint32_t P = pow2_ceil(n);
  for (uint32_t i = n + threadIdx.x; i < P; i += blockDim.x) idx[i] = kNone;
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint32_t a = idx[i], b = idx[l];
          const bool up = (i & k) == 0;
          if (up ? less(b, a) : less(a, b)) { idx[i] = b; idx[l] = a; }
        }
      }
      __syncthreads();
    }
  }
}

// Counting sort of n items by digit d(i) < D, then order each equal-digit run by `less`.
template <class Digit, class Less>
__device__ void wg_sort(uint32_t* idx, uint32_t* rk, uint32_t* cnt, uint32_t n, uint32_t D, Digit dig,
                        Less less, uint32_t* misc, uint32_t* tmp) {
  for (uint32_t i = threadIdx.x; i < D; i += blockDim.x) cnt[i] = 0;
  if (threadIdx.x == 0) misc[0] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) rk[i] = atomicAdd(&cnt[dig(i)], 1u);
  __syncthreads();
  wg_scan(cnt, D, tmp);
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) idx[cnt[dig(i)] + rk[i]] = i;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
    const uint32_t d = dig(idx[j]);
    if (j > 0 && dig(idx[j - 1]) == d) continue;  // not a run start
    uint32_t e = j + 1;
    while (e < n && dig(idx[e]) == d) ++e;
    if (e - j > kRunMax) { misc[0] = 1; continue; }
    for (uint32_t a = j + 1; a < e; ++a) {  // insertion sort of the run
      const uint32_t x = idx[a];
      uint32_t b = a;
      while (b > j && less(x, idx[b - 1])) { idx[b] = idx[b - 1]; --b; }
      idx[b] = x;
    }
  }
  __syncthreads();
  if (misc[0]) wg_bitonic(idx, n, less);
}

__device__ __forceinline__ uint64_t imax64(uint64_t a, uint64_t b) { return (int64_t)a > (int64_t)b ? a : b; }

// Key phase of one bucket by one workgroup: sorts the key rows, folds every (key, family)
// segment, writes the key output rows (win of counters and cref are completed by the caller)
// and leaves the sorted output keys in S.okh / okf / ovm / osum / otp / ocb / occ. Returns kout.
__device__ uint32_t bucket_keys(const BucketArgs& A, uint32_t b, const Scratch& S) {
  const uint32_t K = A.kcnt[b], kb = A.kbase[b];
  uint32_t* tmp = S.misc + 4;  // 16 words for wg_scan
  for (int i = threadIdx.x; i < ST_COUNT; i += blockDim.x) S.st[i] = 0;

  // ------------------------------------------------------------ key phase
  for (uint32_t i = threadIdx.x; i < K; i += blockDim.x) {
    S.kh[i] = kget(A, K_KH, A.kp[kb + i]);
    S.kf[i] = kget(A, K_KF, A.kp[kb + i]);
    S.meta[i] = kget(A, K_META, A.kp[kb + i]);
  }
  __syncthreads();
  const int ks = A.key_shift;
  const uint64_t nbk = A.nbuckets;
  // position inside the bucket: the fractional part of (h << shift) * nb / 2^64
  auto kdig = [&](uint32_t i) { return (uint32_t)(((S.kh[i] << ks) * nbk) >> (64 - kDigBits)); };
  wg_sort(S.idx, S.rk, S.cnt, K, kDig, kdig, KeyLess{S, ks}, S.misc, tmp);

  // segment starts (flag) and emit decisions (rank, scanned below)
  const uint64_t last_bad = (A.flags & F_GC_DELETES) ? *A.last_bad : 0;
  for (uint32_t j = threadIdx.x; j < K; j += blockDim.x) {
    const uint32_t x = S.idx[j];
    bool start = true;
    if (j > 0) {
      const uint32_t p = S.idx[j - 1];
      start = !(S.kh[p] == S.kh[x] && S.kf[p] == S.kf[x] &&
                tag_family(meta_tag(S.meta[p])) == tag_family(meta_tag(S.meta[x])));
      if (!start && meta_pos(S.meta[p]) == meta_pos(S.meta[x])) atomicAdd(&S.st[ST_DUP_ROWS], 1ull);
    }
    S.flag[j] = start;
    uint32_t emit = start;
    if (start && meta_tag(S.meta[x]) == TAG_DELETE && (A.flags & F_GC_DELETES)) {
      uint32_t e = j + 1;
      while (e < K && S.kh[S.idx[e]] == S.kh[x] && S.kf[S.idx[e]] == S.kf[x] &&
             meta_tag(S.meta[S.idx[e]]) == TAG_DELETE)
        ++e;
      const uint64_t tfin = kget(A, K_CT, A.kp[kb + S.idx[e - 1]]);
      for (uint32_t q = j; q < e; ++q) {  // DB::gc (db.rs:82-95)
        const uint32_t r = S.idx[q];
        if (meta_order(S.meta[r]) + 1 > last_bad && kget(A, K_CT, A.kp[kb + r]) == tfin) { emit = 0; break; }
      }
      if (!emit) atomicAdd(&S.st[ST_DELETES_GCED], 1ull);
    }
    S.rank[j] = emit;
  }
  __syncthreads();
  const uint32_t kout = wg_scan(S.rank, K, tmp);

  for (uint32_t j = threadIdx.x; j < K; j += blockDim.x) {
    if (!S.flag[j]) continue;
    const uint32_t h = S.idx[j];
    uint32_t e = j + 1;
    while (e < K && !S.flag[e]) ++e;
    const bool emitted = (j + 1 < K ? S.rank[j + 1] : kout) != S.rank[j];
    if (!emitted) continue;
    const uint32_t o = S.rank[j];
    const uint64_t hm = S.meta[h];
    const uint32_t T = meta_tag(hm), hp = meta_pos(hm);
    uint64_t ct = kget(A, K_CT, A.kp[kb + h]), ut = kget(A, K_UT, A.kp[kb + h]), dt = kget(A, K_DT, A.kp[kb + h]);
    uint64_t win = 0, vm = 1ull << hp, outmeta = hm, osum = 0;
    if (T == TAG_EXPIRE || T == TAG_DELETE) {  // plain overwrite: the last (pos, src) wins
      const uint32_t l = S.idx[e - 1];
      ct = kget(A, K_CT, A.kp[kb + l]);
      outmeta = S.meta[l];
      win = meta_order(outmeta);
      ut = dt = 0;
    } else {
      uint32_t nvalid = 1, conflicts = 0, dicts = 0;
      win = meta_order(hm);
      for (uint32_t q = j + 1; q < e; ++q) {  // Object::merge in pos order
        const uint32_t r = S.idx[q];
        const uint64_t m = S.meta[r];
        if (meta_tag(m) != T) { ++conflicts; continue; }  // object.rs:80 Err(())
        ++nvalid;
        vm |= 1ull << meta_pos(m);
        if (T == TAG_BYTES) {  // object.rs:69-77
          const uint64_t c2 = kget(A, K_CT, A.kp[kb + r]);
          if (ct < c2) win = meta_order(m);
          ct = max(ct, c2);
          dt = max(dt, kget(A, K_DT, A.kp[kb + r]));
          ut = max(ut, kget(A, K_UT, A.kp[kb + r]));
        } else if (T == TAG_DICT) {
          ++dicts;
        }
      }
      if (conflicts) atomicAdd(&S.st[ST_TYPE_CONFLICTS], (unsigned long long)conflicts);
      if (dicts) atomicAdd(&S.st[ST_DICT_MERGES], (unsigned long long)dicts);
      if (T == TAG_COUNTER) {
        if (nvalid >= 2) vm |= kVmaskMerged;       // cal_sum after Counter::merge
        else osum = kget(A, K_AUX, A.kp[kb + h]);           // load-time total (type_counter.rs:114-124)
        win = 0;
      } else if (T != TAG_BYTES) {
        win = 0;
      }
    }
    const uint64_t gkh = S.kh[h], gkf = S.kf[h];
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_KH] = gkh;
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_KF] = gkf;
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_CT] = ct;
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_UT] = ut;
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_DT] = dt;
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_META] = meta_pack(meta_tag(outmeta), meta_pos(outmeta), meta_src(outmeta));
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_WIN] = win;
    S.okh[o] = gkh;
    S.okf[o] = gkf;
    S.ovm[o] = vm;
    S.osum[o] = osum;
    S.otp[o] = T | (hp << 8);
    S.ocb[o] = kNone;
    S.occ[o] = 0;
  }
  __syncthreads();
  return kout;
}

__device__ void process_bucket(const BucketArgs& A, uint32_t b, const Scratch& S) {
  const uint32_t kb = A.kbase[b];
  const uint32_t N = A.ncnt[b], nb = A.nbase[b];
  const uint32_t M = A.mcnt[b], mb = A.mbase[b];
  uint32_t* tmp = S.misc + 4;  // 16 words for wg_scan
  const uint32_t kout = bucket_keys(A, b, S);
  const int ks = A.key_shift;

  // ------------------------------------------------------------ child phases
  uint32_t outs[2] = {0, 0};
  for (int fam = 0; fam < 2; ++fam) {
    const bool nodes = fam == 0;
    const uint32_t n = nodes ? N : M, base = nodes ? nb : mb;
    const uint64_t* C = nodes ? A.nr : A.mr;
    const uint32_t* P = nodes ? A.np : A.mp;  // bucket order -> row
    uint64_t* const O = nodes ? A.nos : A.mos;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint64_t pkh = cget(C, C_PKH, P[base + i]), pkf = cget(C, C_PKF, P[base + i]);
      const uint64_t m = cget(C, C_META, P[base + i]);
      // lower_bound over the sorted output keys on (kh, kf); the data row sorts first
      uint32_t lo = 0, hi = kout;
      const uint64_t spkh = pkh << ks;
      while (lo < hi) {  // output keys are in (kh << shift, kh, kf) order
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t sm = S.okh[mid] << ks;
        const bool less = sm < spkh || (sm == spkh && (S.okh[mid] < pkh || (S.okh[mid] == pkh && S.okf[mid] < pkf)));
        if (less) lo = mid + 1;
        else hi = mid;
      }
      uint32_t key = kNone;
      if (lo < kout && S.okh[lo] == pkh && S.okf[lo] == pkf && (S.otp[lo] & 0xFF) <= TAG_SET) {
        const uint32_t T = S.otp[lo] & 0xFF, hp = S.otp[lo] >> 8, p = meta_pos(m);
        const bool type_ok = nodes ? T == TAG_COUNTER : (T == TAG_SET || T == TAG_DICT);
        const bool elem_ok = (S.ovm[lo] >> p) & 1;           // element has the head type
        const bool cand = nodes || meta_tag(m) == KIND_ADD || p == hp;  // remote dels ignored
        if (type_ok && elem_ok && cand) key = lo;
      } else {
        atomicAdd(&S.st[ST_ORPHANS], 1ull);
      }
      S.ck[i] = key == kNone ? kout : key;  // invalid rows sort last (digit kout)
      S.c1[i] = cget(C, C_ID1, P[base + i]);
      S.c2[i] = nodes ? 0 : cget(C, C_ID2, P[base + i]);
      S.cm[i] = m;
    }
    __syncthreads();
    auto cdig = [&](uint32_t i) { return S.ck[i]; };
    wg_sort(S.cidx, S.crk, S.cnt, n, kout + 1, cdig, ChildLess{S}, S.misc, tmp);

    // pass A: fold each (key, id) segment, decide emission
    for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
      const uint32_t x = S.cidx[j];
      uint32_t start = 0;
      if (S.ck[x] != kout) {
        start = 1;
        if (j > 0) {
          const uint32_t p = S.cidx[j - 1];
          start = !(S.ck[p] == S.ck[x] && S.c1[p] == S.c1[x] && S.c2[p] == S.c2[x]);
        }
      }
      S.cflag[j] = start;
      uint32_t emit = 0;
      if (start) {
        uint32_t e = j + 1;
        while (e < n) {
          const uint32_t y = S.cidx[e];
          if (!(S.ck[y] == S.ck[x] && S.c1[y] == S.c1[x] && S.c2[y] == S.c2[x])) break;
          ++e;
        }
        if (nodes) {  // Counter::merge per node (type_counter.rs:60-84): t of the head kept
          const uint64_t t0 = cget(C, C_T, P[base + x]);
          uint64_t v = cget(C, C_ID2, P[base + x]);
          for (uint32_t q = j + 1; q < e; ++q) {
            const uint32_t r = S.cidx[q];
            const uint64_t tt = cget(C, C_T, P[base + r]), vv = cget(C, C_ID2, P[base + r]);
            if (tt > t0) v = vv;
            else if (tt == t0) v = imax64(v, vv);
          }
          S.rt[j] = v;
          S.rm[j] = meta_pack(0, meta_pos(S.cm[x]), meta_src(S.cm[x]));
          emit = 1;
        } else {  // LWWHash::set chain (lwwhash.rs:87-107): ties go to the later candidate
          uint32_t w = x;
          uint64_t tw = cget(C, C_T, P[base + x]);
          for (uint32_t q = j + 1; q < e; ++q) {
            const uint32_t r = S.cidx[q];
            const uint64_t tr = cget(C, C_T, P[base + r]);
            if (!(tw > tr)) { w = r; tw = tr; }
          }
          S.rt[j] = tw;
          S.rm[j] = S.cm[w];
          emit = 1;
          if ((A.flags & F_GC_MEMBERS) && meta_tag(S.cm[w]) == KIND_DEL && tw < A.gc_wm) {
            emit = 0;
            atomicAdd(&S.st[ST_MEMBERS_GCED], 1ull);
          }
        }
      }
      S.crank[j] = emit;
    }
    __syncthreads();
    const uint32_t cout = wg_scan(S.crank, n, tmp);
    outs[fam] = cout;
    // pass B: write outputs, per-key child ranges and counter sums
    for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
      if (!S.cflag[j]) continue;
      const bool emitted = (j + 1 < n ? S.crank[j + 1] : cout) != S.crank[j];
      if (!emitted) continue;
      const uint32_t x = S.cidx[j], o = S.crank[j], key = S.ck[x];
      O[(uint64_t)(base + o) * kChildStride + C_PKH] = S.okh[key];
      O[(uint64_t)(base + o) * kChildStride + C_PKF] = S.okf[key];
      O[(uint64_t)(base + o) * kChildStride + C_ID1] = S.c1[x];
      if (nodes) {
        O[(uint64_t)(base + o) * kChildStride + C_ID2] = S.rt[j];
        O[(uint64_t)(base + o) * kChildStride + C_T] = cget(C, C_T, P[base + x]);
        if (S.ovm[key] & kVmaskMerged) atomicAdd((unsigned long long*)&S.osum[key], (unsigned long long)S.rt[j]);
      } else {
        O[(uint64_t)(base + o) * kChildStride + C_ID2] = S.c2[x];
        O[(uint64_t)(base + o) * kChildStride + C_T] = S.rt[j];
      }
      O[(uint64_t)(base + o) * kChildStride + C_META] = S.rm[j];
      atomicMin(&S.ocb[key], o);
      atomicAdd(&S.occ[key], 1u);
    }
    __syncthreads();
  }

  // ------------------------------------------------------------ per-key finish
  for (uint32_t o = threadIdx.x; o < kout; o += blockDim.x) {
    const uint32_t T = S.otp[o] & 0xFF;
    if (T == TAG_COUNTER) A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_WIN] = S.osum[o];
    A.kos[(uint64_t)(kb + o) * kKeyOutCols + O_CREF] = cref_pack(S.occ[o] ? S.ocb[o] : 0, S.occ[o]);
  }
  if (threadIdx.x == 0) {
    A.kout[b] = kout;
    A.nout[b] = outs[0];
    A.mout[b] = outs[1];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ST_COUNT; i += blockDim.x)
    if (S.st[i]) atomicAdd(&stat_shard(A.stats)[i], S.st[i]);
}

// LDS carve for the fast path.
struct LdsPool {
  uint64_t kh[kCapK], kf[kCapK], meta[kCapK];
  uint64_t okh[kCapK], okf[kCapK], ovm[kCapK], osum[kCapK];
  uint64_t c1[kCapC], c2[kCapC], cm[kCapC], rt[kCapC], rm[kCapC];
  uint32_t idx[kCapK], rk[kCapK], flag[kCapK], rank[kCapK];
  uint32_t otp[kCapK], ocb[kCapK], occ[kCapK];
  uint32_t ck[kCapC], cidx[kCapC], crk[kCapC], cflag[kCapC], crank[kCapC];
  uint32_t cnt[(kDig > kCapK + 1 ? kDig : kCapK + 1) + 1];
  unsigned long long st[ST_COUNT];
  uint32_t misc[32];
};

// Mid tier: buckets too large for one wave (bucket_wave.hip.h) but within the LDS pool.
// Persistent over the device-side list written by the wave kernel (no host round trip).
__global__ void __launch_bounds__(kBktThreads) bucket_mid_kernel(BucketArgs A, const uint32_t* __restrict__ list,
                                                                 const uint32_t* __restrict__ count) {
  __shared__ LdsPool L;
  Scratch S;
  S.kh = L.kh; S.kf = L.kf; S.meta = L.meta;
  S.idx = L.idx; S.rk = L.rk; S.flag = L.flag; S.rank = L.rank; S.cnt = L.cnt;
  S.okh = L.okh; S.okf = L.okf; S.ovm = L.ovm; S.osum = L.osum;
  S.otp = L.otp; S.ocb = L.ocb; S.occ = L.occ;
  S.c1 = L.c1; S.c2 = L.c2; S.cm = L.cm; S.rt = L.rt; S.rm = L.rm;
  S.ck = L.ck; S.cidx = L.cidx; S.crk = L.crk; S.cflag = L.cflag; S.crank = L.crank;
  S.st = L.st; S.misc = L.misc;
  const uint32_t total = *count;
  for (uint32_t i = blockIdx.x; i < total; i += gridDim.x) {
    const uint32_t b = list[i];
    if (A.kcnt[b] > kCapK || A.ncnt[b] > kCapC || A.mcnt[b] > kCapC || A.force_tier == 2 || A.force_tier == 4) {
      if (threadIdx.x == 0) {
        const uint32_t s = atomicAdd(A.hot_count, 1u);
        A.hot_list[s] = b;
        A.kout[b] = A.nout[b] = A.mout[b] = 0;
      }
      continue;
    }
    __syncthreads();
    process_bucket(A, b, S);
    __syncthreads();
  }
}

// Over-capacity buckets: the same algorithm with scratch in a global slab. Slab layout per
// hot bucket (u64 units), sized by hot_scratch_words().
__host__ __device__ inline uint64_t hot_scratch_words(uint64_t K, uint64_t C) {
  const uint64_t PK = K < 2 ? 2 : K, PC = C < 2 ? 2 : C;
  uint64_t pk = 1, pc = 1;
  while (pk < PK) pk <<= 1;
  while (pc < PC) pc <<= 1;
  const uint64_t dig = (kDig > K + 1 ? kDig : K + 1) + 1;
  // u64 arrays: 3K + 4K + 5C ; u32 arrays (in u64 units, rounded): 4*pk(idx..)+3K + 5*pc + dig
  return 7 * K + 5 * C + (4 * pk + 3 * K + 5 * pc + dig + 1) / 2 + 1 + ST_COUNT + 32;
}

__global__ void __launch_bounds__(kBktThreads) bucket_hot_kernel(BucketArgs A) {
  const uint32_t b = A.hot_in[blockIdx.x];
  const uint64_t K = A.kcnt[b];
  const uint64_t C = max(A.ncnt[b], A.mcnt[b]);
  uint64_t* w = A.hot_scratch + A.hot_scratch_off[blockIdx.x];
  uint64_t pk = 1, pc = 1;
  while (pk < (K < 2 ? 2 : K)) pk <<= 1;
  while (pc < (C < 2 ? 2 : C)) pc <<= 1;
  const uint64_t dig = (kDig > K + 1 ? kDig : K + 1) + 1;
  Scratch S;
  S.kh = w; w += K; S.kf = w; w += K; S.meta = w; w += K;
  S.okh = w; w += K; S.okf = w; w += K; S.ovm = w; w += K; S.osum = w; w += K;
  S.c1 = w; w += C; S.c2 = w; w += C; S.cm = w; w += C; S.rt = w; w += C; S.rm = w; w += C;
  S.st = reinterpret_cast<unsigned long long*>(w); w += ST_COUNT;
  uint32_t* u = reinterpret_cast<uint32_t*>(w);
  S.idx = u; u += pk; S.rk = u; u += pk; S.flag = u; u += pk; S.rank = u; u += pk;
  S.otp = u; u += K; S.ocb = u; u += K; S.occ = u; u += K;
  S.cidx = u; u += pc; S.ck = u; u += pc; S.crk = u; u += pc; S.cflag = u; u += pc; S.crank = u; u += pc;
  S.cnt = u; u += dig;
  S.misc = u;
  __syncthreads();
  process_bucket(A, b, S);
}

}  // namespace cdb
