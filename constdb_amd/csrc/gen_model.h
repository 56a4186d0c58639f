// Deterministic synthetic replica model, evaluated identically on
// the host (snapshot bytes for the decode path and the oracle) and on gfx950 (rows
// written straight into HBM for the benches). Everything is a pure function of
// (seed, key index i, replica r, slot): no state, no ordering dependence.
#pragma once
#include <stdint.h>

#include "common.h"

namespace cdb {

// Hot-key skew (config C5): expected children per present (key, replica) as a function of the
// key's popularity rank k = i + 1, tabulated on the host (model_of) at ranks 1..16 and then every
// quarter octave, in 2^16 fixed point; looked up with integer interpolation so that the host
// writer and the device generator draw identical rows.
constexpr int kHotTab = 128;

struct GenModel {
  uint64_t seed, universe;
  uint32_t n_replicas, key_permille;
  uint32_t mix[4];  // bytes, counter, set, dict weights
  uint32_t conflict_ppm, tie_permille, max_nodes, mean_members, member_universe, del_permille,
      side_permille, value_min, value_max, shard, n_shards;
  uint32_t flags;   // CDB_GEN_* (cdb_merge.h)
  uint32_t hot_n;   // hot-mode table entries (0 = hot mode off)
  uint32_t hot_rank[kHotTab];  // strictly increasing ranks
  uint64_t hot_lam[kHotTab];   // expected children x 2^16 at hot_rank[j]
};

constexpr uint32_t kGenNodePerReplica = 1u;  // CDB_GEN_NODE_PER_REPLICA
constexpr uint32_t kGenOpsZipfMembers = 2u;  // CDB_GEN_OPS_ZIPF_MEMBERS
constexpr uint32_t kGenOpsTagsOnly = 4u;     // CDB_GEN_OPS_TAGS_ONLY
constexpr uint64_t kHotSrcStride = 1ull << 22;  // hot-mode child src = i * stride + slot

constexpr uint64_t kT0Ms = 1700000000000ull;  // uuid = ms << 22 | seq (server.rs:159-173)
constexpr uint32_t kAllReplicas = 0xFFFFu;

CDB_HD uint64_t grnd(const GenModel& g, uint64_t i, uint32_t r, uint32_t slot) {
  return mix64(g.seed ^ mix64(i * 0x9E3779B97F4A7C15ull + 0x1234567ull) ^
               mix64(((uint64_t)r << 32) ^ slot ^ 0xA5A5A5A5ull));
}

// Key bytes of key index i: "key:<decimal i>". Returns the length (<= 24).
CDB_HD int key_bytes(uint64_t i, uint8_t* out) {
  uint8_t tmp[20];
  int n = 0;
  do { tmp[n++] = (uint8_t)('0' + i % 10); i /= 10; } while (i);
  out[0] = 'k'; out[1] = 'e'; out[2] = 'y'; out[3] = ':';
  for (int k = 0; k < n; ++k) out[4 + k] = tmp[n - 1 - k];
  return 4 + n;
}
// Member bytes of member index j: "m<decimal j>".
CDB_HD int member_bytes(uint64_t j, uint8_t* out) {
  uint8_t tmp[20];
  int n = 0;
  do { tmp[n++] = (uint8_t)('0' + j % 10); j /= 10; } while (j);
  out[0] = 'm';
  for (int k = 0; k < n; ++k) out[1 + k] = tmp[n - 1 - k];
  return 1 + n;
}

CDB_HD Hash128 gen_key_hash(uint64_t i) {
  uint8_t b[24];
  const int n = key_bytes(i, b);
  return hash_bytes(b, (uint64_t)n, kDomainKey);
}
CDB_HD Hash128 gen_member_hash(uint64_t j) {
  uint8_t b[24];
  const int n = member_bytes(j, b);
  return hash_bytes(b, (uint64_t)n, kDomainMember);
}

CDB_HD bool gen_in_shard(const GenModel& g, uint64_t kh) {
  if (g.n_shards <= 1) return true;
  int bits = 0;
  while ((1u << bits) < g.n_shards) ++bits;
  return (kh >> (64 - bits)) == g.shard;
}

CDB_HD bool gen_present(const GenModel& g, uint64_t i, uint32_t r) {
  return grnd(g, i, r, 0) % 1000 < g.key_permille;
}

CDB_HD uint8_t gen_pick_type(const GenModel& g, uint64_t u) {
  const uint32_t tot = g.mix[0] + g.mix[1] + g.mix[2] + g.mix[3];
  uint32_t x = (uint32_t)(u % (tot ? tot : 1));
  if (x < g.mix[0]) return TAG_BYTES;
  x -= g.mix[0];
  if (x < g.mix[1]) return TAG_COUNTER;
  x -= g.mix[1];
  if (x < g.mix[2]) return TAG_SET;
  return TAG_DICT;
}

CDB_HD uint8_t gen_type(const GenModel& g, uint64_t i, uint32_t r) {
  if (grnd(g, i, r, 2) % 1000000 < g.conflict_ppm) return gen_pick_type(g, grnd(g, i, r, 3));
  return gen_pick_type(g, grnd(g, i, kAllReplicas, 1));
}

// uuid of time slot `slot`: a forced tie puts every replica on the same per-key uuid.
CDB_HD uint64_t gen_time(const GenModel& g, uint64_t i, uint32_t r, uint32_t slot) {
  const uint64_t base_ms = kT0Ms + grnd(g, i, kAllReplicas, 4) % (1u << 20);
  const uint64_t u = grnd(g, i, r, 100 + slot);
  if (u % 1000 < g.tie_permille) return ((base_ms + slot % 7) << 22) | (slot & 7);
  return ((base_ms + (u >> 12) % 100000) << 22) | ((u >> 40) % 4096);
}

struct GenKey {  // the data entry of key i in replica r
  uint8_t tag;
  uint64_t ct, ut, dt;
  uint32_t value_len;    // Bytes
  uint32_t n_nodes;      // Counter
  uint32_t node_start;
  uint32_t n_members;    // Set / Dict
  uint32_t member_start;
  uint32_t child_universe;  // node ids / member indices are drawn modulo this
};

// Hot mode: expected children (x 2^16) of key i in a replica that holds it.
CDB_HD uint64_t gen_hot_lam(const GenModel& g, uint64_t i) {
  const uint64_t k = i + 1;
  uint32_t lo = 0, hi = g.hot_n;  // largest j with hot_rank[j] <= k (hot_rank[0] = 1)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (g.hot_rank[mid] <= k) lo = mid;
    else hi = mid;
  }
  if (lo + 1 >= g.hot_n) return g.hot_lam[lo];
  const uint64_t r0 = g.hot_rank[lo], r1 = g.hot_rank[lo + 1];
  const uint64_t l0 = g.hot_lam[lo], l1 = g.hot_lam[lo + 1];  // l0 >= l1
  const uint64_t f = ((k - r0) << 16) / (r1 - r0);
  return l0 - (((l0 - l1) * f) >> 16);
}

// Hot mode: child count of (i, r) = floor(lam) or floor(lam) + 1 (by the fraction), and the
// universe the children are drawn from (2 ceil(lam): a child is in about half of the replicas
// holding the key, so (key, child) segments run up to R rows).
CDB_HD uint32_t gen_hot_count(const GenModel& g, uint64_t i, uint32_t r, uint32_t* universe) {
  const uint64_t lam = gen_hot_lam(g, i);
  const uint64_t whole = lam >> 16;
  *universe = (uint32_t)(2 * ((lam + 0xFFFF) >> 16));
  if (*universe == 0) *universe = 1;
  return (uint32_t)whole + ((lam & 0xFFFF) > (grnd(g, i, r, 13) & 0xFFFF) ? 1u : 0u);
}

CDB_HD GenKey gen_key(const GenModel& g, uint64_t i, uint32_t r) {
  GenKey k;
  k.tag = gen_type(g, i, r);
  k.ct = gen_time(g, i, r, 0);
  k.ut = gen_time(g, i, r, 1);
  k.dt = grnd(g, i, r, 5) % 8 == 0 ? gen_time(g, i, r, 2) : 0;
  const uint32_t span = g.value_max >= g.value_min ? g.value_max - g.value_min + 1 : 1;
  k.value_len = g.value_min + (uint32_t)(grnd(g, i, r, 6) % span);
  if (g.hot_n) {  // C5: one popularity-driven child count for counters and sets / dicts alike
    uint32_t cu = 1;
    const uint32_t c = gen_hot_count(g, i, r, &cu);
    k.child_universe = cu;
    k.n_nodes = k.n_members = c;
    k.node_start = (uint32_t)(grnd(g, i, r, 8) % cu);
    k.member_start = (uint32_t)(grnd(g, i, r, 10) % cu);
    return k;
  }
  uint64_t u = grnd(g, i, r, 7);
  uint32_t c = 1;
  const uint32_t mn = g.max_nodes ? g.max_nodes : 1;
  while (c < mn && ((u >> (c - 1)) & 1)) ++c;  // geometric(1/2): mean ~2
  k.n_nodes = (g.flags & kGenNodePerReplica) ? 1 : c;
  k.node_start = (uint32_t)(grnd(g, i, kAllReplicas, 8) % mn);
  const uint32_t mu = g.member_universe ? g.member_universe : 1;
  uint32_t m = (uint32_t)(grnd(g, i, r, 9) % (2 * g.mean_members + 1));
  k.n_members = m > mu ? mu : m;
  k.member_start = (uint32_t)(grnd(g, i, r, 10) % mu);
  k.child_universe = 0;
  return k;
}

// Counter node id of child j. MEET shape (CDB_GEN_NODE_PER_REPLICA): the one node is the
// replica's own node id r + 1 (bin/test.rs:85-106 snapshots counters written by each node).
CDB_HD uint64_t gen_node_id(const GenModel& g, const GenKey& k, uint32_t j, uint32_t r) {
  if (g.flags & kGenNodePerReplica) return r + 1;
  if (k.child_universe) return 1 + (k.node_start + j) % k.child_universe;
  const uint32_t mn = g.max_nodes ? g.max_nodes : 1;
  return 1 + (k.node_start + j) % mn;
}
CDB_HD uint64_t gen_node_v(const GenModel& g, uint64_t i, uint32_t r, uint32_t j) {
  return grnd(g, i, r, 200 + j) % (1u << 20);  // non-negative: R1 cannot encode negatives
}
CDB_HD uint64_t gen_node_t(const GenModel& g, uint64_t i, uint32_t r, uint32_t j) {
  return gen_time(g, i, r, 8 + j);
}
CDB_HD uint64_t gen_member_index(const GenModel& g, const GenKey& k, uint32_t j) {
  const uint32_t mu = k.child_universe ? k.child_universe : (g.member_universe ? g.member_universe : 1);
  return (k.member_start + j) % mu;
}
// src coordinates of the device generator's child rows (unique per key and replica)
CDB_HD uint64_t gen_node_src(const GenModel& g, uint64_t i, uint32_t j) {
  return g.hot_n ? i * kHotSrcStride + j : i * (g.max_nodes ? g.max_nodes : 1) + j;
}
CDB_HD uint64_t gen_member_src(const GenModel& g, uint64_t i, uint64_t mi) {
  return g.hot_n ? i * kHotSrcStride + mi : i * (g.member_universe ? g.member_universe : 1) + mi;
}
CDB_HD bool gen_member_is_del(const GenModel& g, uint64_t i, uint32_t r, uint32_t j) {
  return grnd(g, i, r, 300 + j) % 1000 < g.del_permille;
}
CDB_HD uint64_t gen_member_t(const GenModel& g, uint64_t i, uint32_t r, uint32_t j) {
  return gen_time(g, i, r, 16 + j);
}
CDB_HD uint32_t gen_dict_value_len(const GenModel& g, uint64_t i, uint32_t r, uint32_t j) {
  return 4 + (uint32_t)(grnd(g, i, r, 400 + j) % 9);
}
CDB_HD bool gen_has_expire(const GenModel& g, uint64_t i, uint32_t r) {
  return grnd(g, i, r, 11) % 1000 < g.side_permille;
}
CDB_HD bool gen_has_delete(const GenModel& g, uint64_t i, uint32_t r) {
  return grnd(g, i, r, 12) % 1000 < g.side_permille;
}
// Payload byte b of a generated byte string identified by (i, r, stream).
CDB_HD uint8_t gen_byte(const GenModel& g, uint64_t i, uint32_t r, uint32_t stream, uint32_t b) {
  return (uint8_t)(grnd(g, i, r, 1000 + stream * 64 + b / 8) >> (8 * (b % 8)));
}

}  // namespace cdb
