// The fold-order selection of the chip-wide child path (hot.hip.h, hot_fold_kernel), reduced to its
// loop structure, in three forms -- test infrastructure for the round-2 "compiler hazard" (DESIGN.md
// §4a, VERDICT r02 What's weak 6). A run of rows must be visited in (id, pos|src, j) order whatever
// order the sort left them in; each step selects the successor of the last visited row.
//   divergent_if     : the first chip-wide fold as DESIGN.md describes it (a reconstruction: that code
//                      was replaced before it was committed): every loop runs to the lane's own row
//                      count, and the smallest candidate goes into a loop-carried struct by an `if`;
//   divergent_select : the same loops with the struct updated by selects;
//   uniform          : the shipped form: every loop runs the wave's largest row count, with per-lane
//                      predicates (hot.hip.h, the selection path).
// Each returns an order-sensitive digest of the visited rows, so a wrong successor anywhere shows.
// Plain C++ (no HIP types): the same source is compiled for gfx950 (select_loop.hip) and for the host
// under UBSan / MSan (select_loop_host.cpp).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SL_HD __host__ __device__ __forceinline__
#else
#define SL_HD inline
#endif

struct SlRow {
  uint64_t id1, id2, t, meta;
  uint32_t j;
};

SL_HD bool sl_before(const SlRow& a, const SlRow& b) {
  if (a.id1 != b.id1) return a.id1 < b.id1;
  if (a.id2 != b.id2) return a.id2 < b.id2;
  const uint64_t oa = a.meta & 0x00FFFFFFFFFFFFFFull, ob = b.meta & 0x00FFFFFFFFFFFFFFull;
  if (oa != ob) return oa < ob;
  return a.j < b.j;
}

SL_HD uint64_t sl_mix(uint64_t h, const SlRow& r) { return (h ^ (r.j + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2))) * 0x100000001B3ull; }

// the pre-fix shape: per-lane trip counts, an `if` into an uninitialised loop-carried struct
SL_HD uint64_t sl_divergent_if(const SlRow* rows, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  SlRow last;
  bool started = false;
  for (uint32_t step = 0; step < n; ++step) {
    SlRow c;
    bool have = false;
    for (uint32_t k = 0; k < n; ++k) {
      const SlRow x = rows[k];
      const bool after = !started || sl_before(last, x);
      if (after && (!have || sl_before(x, c))) {
        c = x;
        have = true;
      }
    }
    if (!have) break;
    h = sl_mix(h, c);
    last = c;
    started = true;
  }
  return h;
}

// the same with selects (no branch around the update)
SL_HD uint64_t sl_divergent_select(const SlRow* rows, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  SlRow last{0, 0, 0, 0, 0};
  for (uint32_t step = 0; step < n; ++step) {
    SlRow c = last;
    bool have = false;
    for (uint32_t k = 0; k < n; ++k) {
      const SlRow x = rows[k];
      const bool after = step == 0 || sl_before(last, x);
      const bool take = after && (!have || sl_before(x, c));
      c.id1 = take ? x.id1 : c.id1;
      c.id2 = take ? x.id2 : c.id2;
      c.t = take ? x.t : c.t;
      c.meta = take ? x.meta : c.meta;
      c.j = take ? x.j : c.j;
      have = have || take;
    }
    if (!have) break;
    h = sl_mix(h, c);
    last = c;
  }
  return h;
}

// the shipped shape: trip counts kmax (the wave's largest n), per-lane predicates
SL_HD uint64_t sl_uniform(const SlRow* rows, uint32_t n, uint32_t kmax) {
  uint64_t h = 1469598103934665603ull;
  SlRow last{0, 0, 0, 0, 0};
  for (uint32_t step = 0; step < kmax + 1 && kmax; ++step) {
    SlRow c = last;
    bool have = false;
    for (uint32_t k = 0; k < kmax; ++k) {
      if (k < n && step < n) {
        const SlRow x = rows[k];
        const bool after = step == 0 || sl_before(last, x);
        const bool take = after && (!have || sl_before(x, c));
        c.id1 = take ? x.id1 : c.id1;
        c.id2 = take ? x.id2 : c.id2;
        c.t = take ? x.t : c.t;
        c.meta = take ? x.meta : c.meta;
        c.j = take ? x.j : c.j;
        have = have || take;
      }
    }
    if (have) {
      h = sl_mix(h, c);
      last = c;
    }
  }
  return h;
}

// Deterministic test runs: run i has 1 + (i * 7 + i / 13) % 12 rows of few distinct ids (ties on id,
// distinct (pos, src)), in a scrambled order.
SL_HD uint32_t sl_len(uint32_t i) { return 1 + (i * 7u + i / 13u) % 12u; }
SL_HD uint64_t sl_rng(uint64_t x) {
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
SL_HD SlRow sl_row(uint32_t i, uint32_t k) {
  const uint64_t r = sl_rng(((uint64_t)i << 8) | k);
  SlRow x;
  x.id1 = 1000 + (r & 3);             // 4 ids: runs of several rows per id
  x.id2 = (r >> 2) & 1;
  x.t = r >> 40;
  x.meta = ((uint64_t)((r >> 3) & 7) << 48) | (sl_rng(r) & 0xFFFF) ;  // pos 0..7, src
  x.j = (uint32_t)k;
  return x;
}
