// Deterministic synthetic replica model, evaluated identically on
// the host (snapshot bytes for the decode path and the oracle) and on gfx950 (rows
// written straight into HBM for the benches). Everything is a pure function of
// (seed, key index i, replica r, slot): no state, no ordering dependence.
#pragma once
#include <stdint.h>

#include "common.h"

namespace cdb {

struct GenModel {
  uint64_t seed, universe;
  uint32_t n_replicas, key_permille;
  uint32_t mix[4];  // bytes, counter, set, dict weights
  uint32_t conflict_ppm, tie_permille, max_nodes, mean_members, member_universe, del_permille,
      side_permille, value_min, value_max, shard, n_shards;
};

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
};

CDB_HD GenKey gen_key(const GenModel& g, uint64_t i, uint32_t r) {
  GenKey k;
  k.tag = gen_type(g, i, r);
  k.ct = gen_time(g, i, r, 0);
  k.ut = gen_time(g, i, r, 1);
  k.dt = grnd(g, i, r, 5) % 8 == 0 ? gen_time(g, i, r, 2) : 0;
  const uint32_t span = g.value_max >= g.value_min ? g.value_max - g.value_min + 1 : 1;
  k.value_len = g.value_min + (uint32_t)(grnd(g, i, r, 6) % span);
  uint64_t u = grnd(g, i, r, 7);
  uint32_t c = 1;
  const uint32_t mn = g.max_nodes ? g.max_nodes : 1;
  while (c < mn && ((u >> (c - 1)) & 1)) ++c;  // geometric(1/2): mean ~2
  k.n_nodes = c;
  k.node_start = (uint32_t)(grnd(g, i, kAllReplicas, 8) % mn);
  const uint32_t mu = g.member_universe ? g.member_universe : 1;
  uint32_t m = (uint32_t)(grnd(g, i, r, 9) % (2 * g.mean_members + 1));
  k.n_members = m > mu ? mu : m;
  k.member_start = (uint32_t)(grnd(g, i, r, 10) % mu);
  return k;
}

CDB_HD uint64_t gen_node_id(const GenModel& g, const GenKey& k, uint32_t j) {
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
  const uint32_t mu = g.member_universe ? g.member_universe : 1;
  return (k.member_start + j) % mu;
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
