// Host side of the synthetic generator: writes replica snapshots in the reference's wire
// format (server.rs:183-215, db.rs:122-136, object.rs:85-108, type_counter.rs:101-109,
// crdt/lwwhash.rs:189-205/325-339; Bytes values length-prefixed as the loader expects,
// object.rs:114-117).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cdb_merge.h"
#include "gen_model.h"

namespace cdb {

struct SnapWriter {  // SnapshotWriter (snapshot.rs:9-69) without the CRC (done at the end)
  std::vector<uint8_t> b;
  void bytes(const void* p, size_t n) {
    const uint8_t* q = (const uint8_t*)p;
    b.insert(b.end(), q, q + n);
  }
  void byte(uint8_t x) { b.push_back(x); }
  void integer(int64_t i) {  // write_integer (snapshot.rs:25-37)
    if (i < (1 << 6)) {
      byte((uint8_t)i);
    } else if (i < (1 << 14)) {
      const uint16_t v = (uint16_t)((uint16_t)i | (1 << 14));
      byte(v >> 8);
      byte(v & 0xFF);
    } else if (i < (1 << 30)) {
      const uint32_t v = (uint32_t)i | (1u << 31);
      for (int s = 24; s >= 0; s -= 8) byte((v >> s) & 0xFF);
    } else {
      byte(3 << 6);
      for (int s = 56; s >= 0; s -= 8) byte(((uint64_t)i >> s) & 0xFF);
    }
  }
  void str(const void* p, size_t n) {
    integer((int64_t)n);
    bytes(p, n);
  }
};

uint64_t crc64_jones(const uint8_t* p, size_t n) {
  struct Table {  // function-local static: initialised once, thread-safe (C++11)
    uint64_t t[256];
    Table() {
      for (int i = 0; i < 256; ++i) {
        uint64_t c = (uint64_t)i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x95AC9329AC4BC9B5ull : c >> 1;
        t[i] = c;
      }
    }
  };
  static const Table tab;
  uint64_t crc = 0;
  for (size_t i = 0; i < n; ++i) crc = tab.t[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
  return crc;
}

GenModel model_of(const cdb_gen_config& c) {
  GenModel g;
  g.seed = c.seed;
  g.universe = c.universe;
  g.n_replicas = c.n_replicas;
  g.key_permille = c.key_permille;
  g.mix[0] = c.mix_bytes;
  g.mix[1] = c.mix_counter;
  g.mix[2] = c.mix_set;
  g.mix[3] = c.mix_dict;
  g.conflict_ppm = c.conflict_ppm;
  g.tie_permille = c.tie_permille;
  g.max_nodes = c.max_nodes;
  g.mean_members = c.mean_members;
  g.member_universe = c.member_universe;
  g.del_permille = c.del_permille;
  g.side_permille = c.side_permille;
  g.value_min = c.value_min;
  g.value_max = c.value_max;
  g.shard = c.shard;
  g.n_shards = c.n_shards;
  g.flags = c.flags;
  g.hot_n = 0;
  for (int j = 0; j < kHotTab; ++j) g.hot_rank[j] = 0, g.hot_lam[j] = 0;
  if (c.hot_zipf_milli && c.hot_events && c.universe) {
    // popularity rank k = i + 1 draws lam(k) = E k^-s / (H R p f) children per present
    // (key, replica): E = hot_events over all replicas, H = sum_k k^-s (exact up to 4096, the
    // integral beyond), p = presence probability, f = share of child-bearing types
    const double s = c.hot_zipf_milli / 1000.0;
    const double U = (double)c.universe;
    double H = 0;
    const uint64_t head = std::min<uint64_t>(c.universe, 4096);
    for (uint64_t k = 1; k <= head; ++k) H += std::pow((double)k, -s);
    if (c.universe > head) {
      H += std::fabs(s - 1.0) < 1e-9 ? std::log((U + 0.5) / (head + 0.5))
                                     : (std::pow(U + 0.5, 1 - s) - std::pow(head + 0.5, 1 - s)) / (1 - s);
    }
    const double tot = (double)c.mix_bytes + c.mix_counter + c.mix_set + c.mix_dict;
    const double f = tot > 0 ? (c.mix_counter + c.mix_set + c.mix_dict) / tot : 0;
    const double p = c.key_permille / 1000.0;
    const double R = c.n_replicas ? (double)c.n_replicas : 1.0;
    const double scale = (f > 0 && p > 0) ? (double)c.hot_events / (H * R * p * f) : 0.0;
    uint64_t prev = 0;
    for (int j = 0; j < kHotTab; ++j) {
      uint64_t k = j < 16 ? (uint64_t)j + 1 : (uint64_t)std::llround(16.0 * std::pow(2.0, (j - 15) / 4.0));
      if (k <= prev) k = prev + 1;
      if (k > 0xFFFFFFFFull) break;
      g.hot_rank[j] = (uint32_t)k;
      g.hot_lam[j] = (uint64_t)std::llround(scale * std::pow((double)k, -s) * 65536.0);
      g.hot_n = (uint32_t)j + 1;
      prev = k;
      if (k >= c.universe) break;
    }
  }
  return g;
}

}  // namespace cdb

using namespace cdb;

extern "C" {

void cdb_gen_default(cdb_gen_config* c) {
  std::memset(c, 0, sizeof *c);
  c->seed = 1;
  c->universe = 1000;
  c->n_replicas = 2;
  c->key_permille = 500;
  c->mix_bytes = 60;       // C4 type mix
  c->mix_counter = 30;
  c->mix_set = 5;
  c->mix_dict = 5;
  c->conflict_ppm = 1000;  // 0.1 % cross-replica type conflicts
  c->tie_permille = 20;    // ~2 % forced time ties
  c->max_nodes = 8;
  c->mean_members = 4;
  c->member_universe = 16;
  c->del_permille = 200;
  c->side_permille = 20;
  c->value_min = 8;
  c->value_max = 32;
  c->shard = 0;
  c->n_shards = 1;
  c->replica_lo = 0;
  c->replica_hi = 2;
}

cdb_status cdb_gen_snapshot(const cdb_gen_config* cfg, uint32_t r, uint8_t** out, size_t* len) {
  if (!cfg || !out || !len) return CDB_BAD_ARGUMENT;
  const GenModel g = model_of(*cfg);
  SnapWriter data, exp, del;
  uint64_t nd = 0, ne = 0, ndel = 0;
  uint8_t kb[24], mbuf[24];
  for (uint64_t i = 0; i < g.universe; ++i) {
    const Hash128 h = gen_key_hash(i);
    if (!gen_in_shard(g, h.h)) continue;
    const int kl = key_bytes(i, kb);
    if (gen_present(g, i, r)) {
      const GenKey k = gen_key(g, i, r);
      ++nd;
      data.str(kb, kl);
      data.integer((int64_t)k.ct);
      data.integer((int64_t)k.ut);
      data.integer((int64_t)k.dt);
      data.byte(k.tag);
      if (k.tag == TAG_BYTES) {
        data.integer(k.value_len);
        for (uint32_t b = 0; b < k.value_len; ++b) data.byte(gen_byte(g, i, r, 0, b));
      } else if (k.tag == TAG_COUNTER) {
        data.integer(k.n_nodes);
        for (uint32_t j = 0; j < k.n_nodes; ++j) {
          data.integer((int64_t)gen_node_id(g, k, j, r));
          data.integer((int64_t)gen_node_v(g, i, r, j));
          data.integer((int64_t)gen_node_t(g, i, r, j));
        }
      } else {
        uint32_t nadd = 0;
        for (uint32_t j = 0; j < k.n_members; ++j) nadd += !gen_member_is_del(g, i, r, j);
        for (int pass = 0; pass < 2; ++pass) {  // add map, then del map
          data.integer(pass == 0 ? nadd : k.n_members - nadd);
          for (uint32_t j = 0; j < k.n_members; ++j) {
            if (gen_member_is_del(g, i, r, j) != (pass == 1)) continue;
            const int ml = member_bytes(gen_member_index(g, k, j), mbuf);
            data.str(mbuf, ml);
            data.integer((int64_t)gen_member_t(g, i, r, j));
            if (pass == 0 && k.tag == TAG_DICT) {
              const uint32_t vl = gen_dict_value_len(g, i, r, j);
              data.integer(vl);
              for (uint32_t b = 0; b < vl; ++b) data.byte(gen_byte(g, i, r, 1 + j, b));
            }
          }
        }
      }
    }
    if (gen_has_expire(g, i, r)) {
      ++ne;
      exp.str(kb, kl);
      exp.integer((int64_t)gen_time(g, i, r, 3));
    }
    if (gen_has_delete(g, i, r)) {
      ++ndel;
      del.str(kb, kl);
      del.integer((int64_t)gen_time(g, i, r, 4));
    }
  }
  SnapWriter w;
  w.bytes("CONSTDB", 7);
  const uint8_t ver[4] = {0, 1, 1, 1};
  w.bytes(ver, 4);
  const std::string alias = "n" + std::to_string(r + 1), addr = "127.0.0.1:" + std::to_string(9001 + r);
  w.integer(r + 1);
  w.str(alias.data(), alias.size());
  w.str(addr.data(), addr.size());
  w.integer((int64_t)((kT0Ms + 2000000) << 22));
  w.byte(5);
  w.integer((int64_t)nd);
  w.bytes(data.b.data(), data.b.size());
  w.byte(6);
  w.integer((int64_t)ne);
  w.bytes(exp.b.data(), exp.b.size());
  w.byte(7);
  w.integer((int64_t)ndel);
  w.bytes(del.b.data(), del.b.size());
  w.byte(8);
  const uint64_t crc = crc64_jones(w.b.data(), w.b.size());
  for (int i = 0; i < 8; ++i) w.byte((crc >> (8 * i)) & 0xFF);
  *out = (uint8_t*)std::malloc(w.b.size());
  if (!*out) return CDB_OUT_OF_MEMORY;
  std::memcpy(*out, w.b.data(), w.b.size());
  *len = w.b.size();
  return CDB_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- op streams
namespace {
// An index in [0, n) from the random word u: uniform (s <= 0) or power-law skewed, rank ~
// x^(1/(1-s)) for x uniform in (0, 1] (s < 1); `spread` scatters the hot ranks over [0, n).
uint64_t skewed(uint64_t u, double s, uint64_t n, bool spread) {
  if (s <= 0) return u % n;
  const double x = ((u >> 11) + 1) * (1.0 / 9007199254740992.0);
  const double r = std::pow(x, 1.0 / (1.0 - std::min(s, 0.99))) * (double)n;
  const uint64_t i = std::min<uint64_t>((uint64_t)r, n - 1);
  return spread ? (i * 0x9E3779B97F4A7C15ull) % n : i;
}

struct RespWriter {  // WriteBuf::write_msg (conn/buf_write.rs:127-150)
  std::vector<uint8_t> b;
  void lit(const char* s) { b.insert(b.end(), s, s + std::strlen(s)); }
  void num(int64_t v) {
    char t[24];
    const int n = std::snprintf(t, sizeof t, "%lld", (long long)v);
    b.insert(b.end(), t, t + n);
  }
  void arr(int n) { lit("*"), num(n), lit("\r\n"); }
  void integer(int64_t v) { lit(":"), num(v), lit("\r\n"); }
  void bulk(const void* p, size_t n) {
    lit("$"), num((int64_t)n), lit("\r\n");
    const uint8_t* q = (const uint8_t*)p;
    b.insert(b.end(), q, q + n);
    lit("\r\n");
  }
  void bulk(const char* s) { bulk(s, std::strlen(s)); }
};
}  // namespace

extern "C" cdb_status cdb_gen_ops(const cdb_gen_config* cfg, uint64_t n_ops, uint64_t uuid_he_sent,
                                  uint32_t zipf_milli, uint8_t** out, size_t* len) {
  if (!cfg || !out || !len) return CDB_BAD_ARGUMENT;
  const GenModel g = model_of(*cfg);
  RespWriter w;
  w.b.reserve(n_ops * 48);
  uint64_t last = uuid_he_sent;
  const double s = zipf_milli / 1000.0;
  uint8_t kb[24], mb[24];
  const uint32_t mu = g.member_universe ? g.member_universe : 1;
  // the per-op draws use a replica slot of their own: 0xFFFE, or one salted by cfg->stream (the
  // key types stay gen_type's, a function of the seed alone)
  const uint32_t os = cfg->stream ? 0x10000u + cfg->stream : 0xFFFEu;
  for (uint64_t q = 0; q < n_ops; ++q) {
    const uint64_t u0 = grnd(g, q, os, 1), u1 = grnd(g, q, os, 2), u2 = grnd(g, q, os, 3);
    // key index: uniform, or a power-law skew (rank ~ x^(1/(1-s)) for x uniform in (0,1])
    const bool zmem = (g.flags & kGenOpsZipfMembers) != 0, tags_only = (g.flags & kGenOpsTagsOnly) != 0;
    const uint64_t i = zmem ? u0 % g.universe : skewed(u0, zmem ? 0 : s, g.universe, true);
    const Hash128 h = gen_key_hash(i);
    if (!gen_in_shard(g, h.h)) continue;
    const uint8_t tag = (!tags_only && u1 % 1000 < 2) ? gen_pick_type(g, u2) : gen_type(g, i, kAllReplicas);
    // ~2^20 ms past the state's times, with 5 % of the ops older than the state
    const uint64_t ms = (u1 >> 20) % 1000 < 50 ? kT0Ms + (u2 >> 24) % (1u << 20) : kT0Ms + (1u << 20) + q / 64;
    const uint64_t uuid = (ms << 22) | (q & 0x3FFFFF);
    const int kl = key_bytes(i, kb);
    const uint32_t pick = (uint32_t)(u2 % 100);
    const uint32_t nm = 1 + (uint32_t)((u2 >> 8) % 3);
    const uint64_t node = 1 + (u0 >> 40) % (g.max_nodes ? g.max_nodes : 1);
    const char* name;
    int nargs = 1;  // key
    if (tag == TAG_BYTES) {
      name = pick < 95 ? "set" : "delbytes";
      nargs += pick < 95;
    } else if (tag == TAG_COUNTER) {
      name = pick < 60 ? "incr" : pick < 97 ? "decr" : "delcnt";
      if (pick >= 97) nargs += 2;
    } else if (tag == TAG_SET) {
      name = pick < 70 ? "sadd" : (pick < 99 || tags_only) ? "srem" : "delset";
      if (pick < 99 || tags_only) nargs += nm;
    } else {
      name = pick < 70 ? "hset" : (pick < 99 || tags_only) ? "hdel" : "deldict";
      if (pick < 99 || tags_only) nargs += pick < 70 ? 2 * nm : nm;
    }
    w.arr(5 + nargs);
    w.bulk("replicate");
    w.integer((int64_t)node);
    w.integer((int64_t)last);
    w.integer((int64_t)uuid);
    w.bulk(name);
    w.bulk(kb, kl);
    last = uuid;
    if (!std::strcmp(name, "set")) {
      const uint32_t vl = g.value_min + (uint32_t)(u0 % (g.value_max >= g.value_min ? g.value_max - g.value_min + 1 : 1));
      uint8_t v[64];
      for (uint32_t b = 0; b < vl && b < 64; ++b) v[b] = (uint8_t)('a' + (grnd(g, q, os, 10 + b / 8) >> (8 * (b % 8))) % 26);
      w.bulk(v, std::min<uint32_t>(vl, 64));
    } else if (!std::strcmp(name, "delcnt")) {
      w.integer((int64_t)node);
      w.integer(-(int64_t)(u1 % 100));
    } else if (nargs > 1) {
      for (uint32_t j = 0; j < nm; ++j) {
        const uint64_t mj = zmem ? skewed(grnd(g, q, os, 20 + j), s, mu, false) : (u0 >> 16) % mu + j;
        const int ml = member_bytes(mj, mb);
        w.bulk(mb, ml);
        if (!std::strcmp(name, "hset")) w.bulk("v", 1);
      }
    }
  }
  *out = (uint8_t*)std::malloc(std::max<size_t>(w.b.size(), 1));
  if (!*out) return CDB_OUT_OF_MEMORY;
  std::memcpy(*out, w.b.data(), w.b.size());
  *len = w.b.size();
  return CDB_OK;
}
