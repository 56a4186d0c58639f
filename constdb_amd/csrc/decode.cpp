// Snapshot decoder: ConstDB wire format -> columnar Batch.
//
// Follows the reference loader (snapshot.rs:120-295) and the object loaders
// (object.rs:110-129, type_counter.rs:111-126, crdt/lwwhash.rs:207-226,341-358) but reads
// from one in-memory buffer in a single pass (the reference issues one awaited
// read_exact per varint flag byte and CRCs byte-slices as it goes) and emits SoA rows.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/cdb_merge.h"
#include "batch.h"

namespace cdb {
namespace {

// CRC-64/Jones (crc64 2.0.0, Cargo.lock:197-200): reflected poly 0x95AC9329AC4BC9B5,
// init 0, no xorout. Slice-by-8 table for the decoder's one CRC pass over the stream.
struct Crc64 {
  uint64_t t[8][256];
  Crc64() {
    for (int i = 0; i < 256; ++i) {
      uint64_t c = (uint64_t)i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x95AC9329AC4BC9B5ull : c >> 1;
      t[0][i] = c;
    }
    for (int i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = t[0][t[s - 1][i] & 0xFF] ^ (t[s - 1][i] >> 8);
  }
  uint64_t update(uint64_t crc, const uint8_t* p, size_t n) const {
    while (n >= 8) {
      uint64_t w;
      std::memcpy(&w, p, 8);
      crc ^= w;
      crc = t[7][crc & 0xFF] ^ t[6][(crc >> 8) & 0xFF] ^ t[5][(crc >> 16) & 0xFF] ^
            t[4][(crc >> 24) & 0xFF] ^ t[3][(crc >> 32) & 0xFF] ^ t[2][(crc >> 40) & 0xFF] ^
            t[1][(crc >> 48) & 0xFF] ^ t[0][crc >> 56];
      p += 8;
      n -= 8;
    }
    while (n--) crc = t[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    return crc;
  }
};
const Crc64& crc_tables() {
  static const Crc64 c;
  return c;
}

struct Cursor {
  const uint8_t* p;
  size_t n, off = 0;
  int err = CDB_OK;

  bool need(size_t k) {
    if (k > n - off) { err = CDB_IO_ERROR; return false; }  // read_exact -> UnexpectedEof
    return true;
  }
  bool u8(uint8_t* b) {
    if (!need(1)) return false;
    *b = p[off++];
    return true;
  }
  // read_integer (snapshot.rs:243-264): 2-bit tag in the flag byte's top bits.
  bool integer(int64_t* out) {
    uint8_t f;
    if (!u8(&f)) return false;
    switch (f >> 6) {
      case 0: *out = f & 0x3F; return true;
      case 1:
        if (!need(1)) return false;
        *out = ((int64_t)(f & 0x3F) << 8) | p[off];
        off += 1;
        return true;
      case 2:
        if (!need(3)) return false;
        *out = ((int64_t)(f & 0x3F) << 24) | ((int64_t)p[off] << 16) | ((int64_t)p[off + 1] << 8) | p[off + 2];
        off += 3;
        return true;
      default: {
        if (!need(8)) return false;
        uint64_t v = 0;
        for (int i = 0; i < 8; ++i) v = (v << 8) | p[off + i];
        off += 8;
        *out = (int64_t)v;
        return true;
      }
    }
  }
  bool u64(uint64_t* out) {  // `as u64` of the i64
    int64_t v;
    if (!integer(&v)) return false;
    *out = (uint64_t)v;
    return true;
  }
  bool length(uint64_t* out) {  // `as usize`: a negative length can never be read
    int64_t v;
    if (!integer(&v)) return false;
    if (v < 0) { err = CDB_IO_ERROR; return false; }
    *out = (uint64_t)v;
    return true;
  }
  bool span(ByteRef* r) {  // length-prefixed bytes
    uint64_t l;
    if (!length(&l) || !need(l)) return false;
    r->off = off;
    r->len = l;
    off += l;
    return true;
  }
};

bool valid_utf8(const uint8_t* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    size_t k;
    uint32_t cp;
    if (c < 0x80) { i += 1; continue; }
    if ((c >> 5) == 6) { k = 1; cp = c & 0x1F; }
    else if ((c >> 4) == 14) { k = 2; cp = c & 0x0F; }
    else if ((c >> 3) == 30) { k = 3; cp = c & 0x07; }
    else return false;
    if (i + k >= n) return false;
    for (size_t j = 1; j <= k; ++j) {
      if ((s[i + j] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (s[i + j] & 0x3F);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000) || cp > 0x10FFFF ||
        (cp >= 0xD800 && cp <= 0xDFFF))
      return false;
    i += k + 1;
  }
  return true;
}

struct Decoder {
  Cursor c;
  Batch* b;
  const uint8_t* base;
  EntryIndex* idx = nullptr;  // index mode (GPU decode): validate and record, no rows
  DeferredCrc* dcrc = nullptr;  // index mode: leave the checksum to the GPU
  uint32_t threads = 1;         // index mode: threads for a large DATAS section (parallel_datas)
  bool speculative = false;     // parallel_datas' walks: counts the rest of the stream cannot hold
                                // fail at once (the sequential pass reports those streams)
  uint64_t spec_max = ~0ull;    // ... and, in the sync search, counts past this many bytes
  DeferredDatas* defer = nullptr;  // index mode: a large first DATAS section is left to the device

  bool parallel_datas(uint64_t cnt);

  bool str(std::string* s) {
    ByteRef r;
    if (!c.span(&r)) return false;
    if (!valid_utf8(base + r.off, r.len)) {  // snapshot.rs:143-149 unwraps -> panic
      c.err = CDB_INVALID_SNAPSHOT;
      return false;
    }
    s->assign((const char*)base + r.off, r.len);
    return true;
  }

  // Counter::load_snapshot (type_counter.rs:111-126): data.insert per node (the last of a
  // duplicated node id wins) while `total` sums every value read (wrapping i64).
  bool counter(uint64_t kh, uint64_t kf, uint64_t* total) {
    uint64_t cnt;
    if (!c.length(&cnt)) return false;
    if (speculative && cnt > std::min<uint64_t>(c.n - c.off, spec_max) / 3) return false;  // 3 varints of >= 1 byte
    if (idx) {  // index mode: skip the triples, the GPU parses them
      for (uint64_t i = 0; i < cnt; ++i) {
        uint64_t x;
        int64_t v;
        if (!c.u64(&x) || !c.integer(&v) || !c.u64(&x)) return false;
      }
      return true;
    }
    struct N { uint64_t node, v, t; };
    std::vector<N> ns;
    ns.reserve(cnt < (1u << 20) ? cnt : (1u << 20));
    uint64_t sum = 0;
    for (uint64_t i = 0; i < cnt; ++i) {
      N x;
      int64_t v;
      if (!c.u64(&x.node) || !c.integer(&v) || !c.u64(&x.t)) return false;
      x.v = (uint64_t)v;
      sum += x.v;
      ns.push_back(x);
    }
    // A node id repeated inside one counter (never written by type_counter.rs:101-109):
    // HashMap::insert keeps the last (node, v, t); `total` still counted every value.
    std::vector<uint8_t> keep(ns.size(), 1);
    if (ns.size() > 1) {
      std::vector<uint32_t> ord(ns.size());
      for (uint32_t i = 0; i < ord.size(); ++i) ord[i] = i;
      std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b2) {
        return ns[a].node != ns[b2].node ? ns[a].node < ns[b2].node : a < b2;
      });
      for (size_t j = 0; j + 1 < ord.size(); ++j)
        if (ns[ord[j]].node == ns[ord[j + 1]].node) keep[ord[j]] = 0;
    }
    for (size_t i = 0; i < ns.size(); ++i) {
      if (!keep[i]) continue;
      const uint64_t src = b->n_pkh.size();
      b->n_pkh.push_back(kh);
      b->n_pkf.push_back(kf);
      b->n_node.push_back(ns[i].node);
      b->n_v.push_back(ns[i].v);
      b->n_t.push_back(ns[i].t);
      b->n_meta.push_back(meta_pack(0, 0, src));
    }
    *total = sum;
    return true;
  }

  // Set/Dict::load_snapshot (lwwhash.rs:207-226, 341-358): every add through set(), then
  // every del through rem(). Emits the resulting single tag per member.
  bool lwwhash(uint64_t kh, uint64_t kf, bool is_dict) {
    struct Op { Hash128 id; ByteRef m, v; uint64_t t; bool add; };
    std::vector<Op> ops;
    uint64_t na;
    if (!c.length(&na)) return false;
    if (speculative && na > std::min<uint64_t>(c.n - c.off, spec_max) / 2) return false;  // a span and a varint
    if (idx) {  // index mode: skip the tags, the GPU parses them
      ByteRef r;
      uint64_t t, nd;
      for (uint64_t i = 0; i < na; ++i)
        if (!c.span(&r) || !c.u64(&t) || (is_dict && !c.span(&r))) return false;
      if (!c.length(&nd)) return false;
      if (speculative && nd > std::min<uint64_t>(c.n - c.off, spec_max) / 2) return false;
      for (uint64_t i = 0; i < nd; ++i)
        if (!c.span(&r) || !c.u64(&t)) return false;
      return true;
    }
    ops.reserve(na);
    for (uint64_t i = 0; i < na; ++i) {
      Op o;
      if (!c.span(&o.m) || !c.u64(&o.t)) return false;
      o.v = {0, 0};
      if (is_dict && !c.span(&o.v)) return false;
      o.add = true;
      o.id = hash_bytes(base + o.m.off, o.m.len, kDomainMember);
      ops.push_back(o);
    }
    uint64_t nd;
    if (!c.length(&nd)) return false;
    for (uint64_t i = 0; i < nd; ++i) {
      Op o;
      if (!c.span(&o.m) || !c.u64(&o.t)) return false;
      o.v = {0, 0};
      o.add = false;
      o.id = hash_bytes(base + o.m.off, o.m.len, kDomainMember);
      ops.push_back(o);
    }
    // Duplicate members within one object (never written by lwwhash.rs:189-205/325-339,
    // whose add/del maps hold a member at most once in total): replay set/rem exactly.
    std::vector<uint32_t> order(ops.size());
    for (uint32_t i = 0; i < ops.size(); ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
      if (ops[x].id.h != ops[y].id.h) return ops[x].id.h < ops[y].id.h;
      if (ops[x].id.f != ops[y].id.f) return ops[x].id.f < ops[y].id.f;
      return x < y;
    });
    std::vector<uint8_t> keep(ops.size(), 1);
    for (size_t s = 0; s < order.size();) {
      size_t e = s + 1;
      while (e < order.size() && ops[order[e]].id.h == ops[order[s]].id.h && ops[order[e]].id.f == ops[order[s]].id.f) ++e;
      if (e - s > 1) {
        // state machine of lwwhash.rs:87-128 over the ops of this member in stream order
        int st = -1;  // index of the op holding the current tag, -1 = none
        for (size_t j = s; j < e; ++j) {
          const Op& o = ops[order[j]];
          if (st >= 0 && ops[st].t > o.t) continue;  // tag newer than o -> rejected
          st = (int)order[j];
        }
        for (size_t j = s; j < e; ++j) keep[order[j]] = (int)order[j] == st;
      }
      s = e;
    }
    for (size_t i = 0; i < ops.size(); ++i) {
      if (!keep[i]) continue;
      const Op& o = ops[i];
      const uint64_t src = b->m_pkh.size();
      b->m_pkh.push_back(kh);
      b->m_pkf.push_back(kf);
      b->m_h.push_back(o.id.h);
      b->m_f.push_back(o.id.f);
      b->m_t.push_back(o.t);
      b->m_meta.push_back(meta_pack(o.add ? KIND_ADD : KIND_DEL, 0, src));
      b->m_ref.push_back(o.m);
      b->m_vref.push_back(o.v);
    }
    return true;
  }

  bool data_entry() {  // read_entry (snapshot.rs:280-287) + Object::load_snapshot
    if (idx) {
      idx->offset.push_back(c.off);
      idx->kind.push_back(0);
    }
    ByteRef k;
    if (!c.span(&k)) return false;
    if (speculative && k.len > spec_max) return false;
    uint64_t ct, ut, dt;
    if (!c.u64(&ct) || !c.u64(&ut) || !c.u64(&dt)) return false;
    uint8_t tag;
    if (!c.u8(&tag)) return false;
    const Hash128 h = idx ? Hash128{0, 0} : hash_bytes(base + k.off, k.len, kDomainKey);
    uint64_t aux = 0;
    ByteRef v{0, 0};
    switch (tag) {
      case TAG_COUNTER:
        if (!counter(h.h, h.f, &aux)) return false;
        break;
      case TAG_BYTES:
        if (!c.span(&v)) return false;
        break;
      case TAG_SET:
      case TAG_DICT:
        if (!lwwhash(h.h, h.f, tag == TAG_DICT)) return false;
        break;
      default:
        c.err = CDB_INVALID_TYPE;  // object.rs:121
        return false;
    }
    if (!idx) push_key(h, ct, ut, dt, aux, tag, k, v);
    return true;
  }

  void push_key(const Hash128& h, uint64_t ct, uint64_t ut, uint64_t dt, uint64_t aux, uint8_t tag,
                ByteRef k, ByteRef v) {
    const uint64_t src = b->kh.size();
    b->kh.push_back(h.h);
    b->kf.push_back(h.f);
    b->ct.push_back(ct);
    b->ut.push_back(ut);
    b->dt.push_back(dt);
    b->aux.push_back(aux);
    b->meta.push_back(meta_pack(tag, 0, src));
    b->key_ref.push_back(k);
    b->val_ref.push_back(v);
  }

  bool side_entry(uint8_t tag) {  // read_key_int (snapshot.rs:289-295)
    if (idx) {
      idx->offset.push_back(c.off);
      idx->kind.push_back(tag == TAG_EXPIRE ? 1 : 2);
    }
    ByteRef k;
    uint64_t t;
    if (!c.span(&k) || !c.u64(&t)) return false;
    if (idx) return true;
    const Hash128 h = hash_bytes(base + k.off, k.len, kDomainKey);
    push_key(h, t, 0, 0, 0, tag, k, ByteRef{0, 0});
    return true;
  }

  int run(uint32_t flags, size_t* err_off) {
    auto fail = [&]() {
      *err_off = c.off;
      return c.err == CDB_OK ? CDB_INVALID_SNAPSHOT : c.err;
    };
    // Begin + Version (snapshot.rs:123-139); the magic is not checked by the reference.
    if (!c.need(11)) return fail();
    char vbuf[32];
    snprintf(vbuf, sizeof vbuf, "%u.%u.%u.%u", base[7], base[8], base[9], base[10]);
    b->version = vbuf;
    c.off = 11;
    // Node (snapshot.rs:140-153)
    if (!c.u64(&b->node_id) || !str(&b->alias) || !str(&b->addr) || !c.u64(&b->uuid_he_sent)) return fail();
    return loop(flags, err_off);
  }

  // The sections, from c.off on (run; and after a deferred DATAS section, from its end).
  int loop(uint32_t flags, size_t* err_off) {
    auto fail = [&]() {
      *err_off = c.off;
      return c.err == CDB_OK ? CDB_INVALID_SNAPSHOT : c.err;
    };
    for (;;) {
      uint8_t flag;
      if (!c.u8(&flag)) return fail();  // convert_stat (snapshot.rs:222-241)
      if (flag == 3) {                  // SNAPSHOT_FLAG_REPLICA_ADD
        ReplicaAdd r;
        if (!c.u64(&r.add_time) || !c.u64(&r.node_id) || !str(&r.alias) || !str(&r.addr) || !c.u64(&r.uuid))
          return fail();
        r.seq = (uint32_t)(b->replica_add.size() + b->replica_del.size());
        b->replica_add.push_back(std::move(r));
      } else if (flag == 4) {  // SNAPSHOT_FLAG_REPLICA_REM
        ReplicaDel r;
        if (!str(&r.addr) || !c.u64(&r.t)) return fail();
        r.seq = (uint32_t)(b->replica_add.size() + b->replica_del.size());
        b->replica_del.push_back(std::move(r));
      } else if (flag == 5 || flag == 6 || flag == 7) {  // DATAS / EXPIRES / DELETES
        uint64_t cnt;
        if (!c.length(&cnt)) return fail();
        if (flag == 5 && idx && defer && idx->offset.empty() && cnt >= kDeviceIndexMinEntries) {
          *defer = DeferredDatas{true, (uint64_t)c.off, cnt};  // the device finds the entries
          b->n_data += cnt;
          return kIndexDeferred;
        }
        if (flag == 5 && idx && parallel_datas(cnt)) {  // indexed side by side (c.off at its end)
          b->n_data += cnt;
          continue;
        }
        for (uint64_t i = 0; i < cnt; ++i) {
          bool ok = flag == 5 ? data_entry() : side_entry(flag == 6 ? TAG_EXPIRE : TAG_DELETE);
          if (!ok) return fail();
        }
        if (flag == 5) b->n_data += cnt;
        else if (flag == 6) b->n_expires += cnt;
        else b->n_deletes += cnt;
      } else if (flag == 8) {  // SNAPSHOT_FLAG_CHECKSUM
        const bool defer = dcrc && idx && (!idx->offset.empty() || (this->defer && this->defer->pending));
        if (defer) {  // same prefix, value and error offset as below, checked by the caller
          int64_t got;
          if (flags & CDB_DECODE_REFERENCE_CHECKSUM) {
            if (!c.integer(&got)) return fail();
            *dcrc = DeferredCrc{true, (uint64_t)c.off, (uint64_t)got, c.off};
            return CDB_OK;
          }
          if (!c.need(8)) return fail();
          uint64_t w = 0;
          for (int i = 7; i >= 0; --i) w = (w << 8) | base[c.off + i];
          *dcrc = DeferredCrc{true, (uint64_t)c.off, w, c.off + 8};
          c.off += 8;
          return CDB_OK;
        }
        const uint64_t crc = crc_tables().update(0, base, c.off);
        if (flags & CDB_DECODE_REFERENCE_CHECKSUM) {
          // snapshot.rs:207-213: read the checksum as a varint, CRC those bytes too
          const size_t at = c.off;
          int64_t got;
          if (!c.integer(&got)) return fail();
          const uint64_t crc2 = crc_tables().update(crc, base + at, c.off - at);
          if ((uint64_t)got != crc2) { *err_off = c.off; return CDB_INVALID_SNAPSHOT_CHECKSUM; }
          return CDB_OK;
        }
        if (!c.need(8)) return fail();
        uint64_t got = 0;
        for (int i = 7; i >= 0; --i) got = (got << 8) | base[c.off + i];
        c.off += 8;
        if (got != crc) { *err_off = c.off; return CDB_INVALID_SNAPSHOT_CHECKSUM; }
        return CDB_OK;
      } else {
        c.err = CDB_INVALID_SNAPSHOT;
        c.off -= 1;
        return fail();
      }
    }
  }
};

// The DATAS section of a large snapshot, indexed by several threads. The format has no sync
// marks (an entry starts where its predecessor ends), so each thread speculates:
//   * thread t's range starts at a byte offset B_t; it looks for the first offset o >= B_t from
//     which kSyncEntries consecutive entries parse (data entries have a tag byte that must be
//     0, 3, 4 or 5, and every span must fit: a wrong offset almost never survives 16 of them),
//     then records the entries from o until one starts at or past B_{t+1};
//   * stitching, in order: the true chain enters range t at `cur` (range 0: the section start).
//     Parsing is deterministic from an offset, so if cur is one of thread t's recorded offsets,
//     thread t's entries from there on ARE the true chain; otherwise range t is parsed again from
//     cur on this thread. The section ends after `cnt` entries (later ranges parsed the next
//     sections' bytes as data entries: discarded).
// Any error on the true chain, or a thread that gave up, hands the whole section back to the
// sequential loop (false), so statuses and offsets stay the loader's.
constexpr uint32_t kSyncEntries = 16;
constexpr uint64_t kParallelMinEntries = 1u << 17;
constexpr uint64_t kSyncSearch = 1u << 20;  // bytes a thread searches for its first entry
constexpr uint64_t kSyncEntryMax = 1u << 16; // largest entry a sync chain may hold

bool Decoder::parallel_datas(uint64_t cnt) {
  const uint64_t S = c.off, end = c.n;
  if (threads < 2 || cnt < kParallelMinEntries || end - S < (uint64_t)threads * 4096) return false;
  const uint32_t T = threads;
  std::vector<uint64_t> B(T + 1);
  for (uint32_t t = 0; t <= T; ++t) B[t] = S + (end - S) * t / T;
  struct Part {
    std::vector<uint64_t> off;
    uint64_t stop = 0;     // offset of the first entry at or past the range end (or of the failure)
    bool ok = false;       // reached the range end without a parse error
  };
  std::vector<Part> parts(T);
  auto walk = [&](uint64_t from, uint64_t lim, Part& P) {  // entries from `from` up to lim
    Decoder d{Cursor{base, end}, b, base};
    EntryIndex scratch;
    d.idx = &scratch;
    d.speculative = true;
    d.c.off = from;
    P.off.clear();
    P.off.reserve((lim - from) / 40 + 16);
    while (d.c.off < lim) {
      const uint64_t at = d.c.off;
      scratch.offset.clear();
      scratch.kind.clear();
      if (!d.data_entry()) {
        P.stop = at;
        P.ok = false;
        return;
      }
      P.off.push_back(at);
    }
    P.stop = d.c.off;
    P.ok = true;
  };
  auto work = [&](uint32_t t) {
    Part& P = parts[t];
    uint64_t o = B[t];
    if (t > 0) {  // speculative sync point
      Decoder d{Cursor{base, end}, b, base};
      EntryIndex scratch;
      d.idx = &scratch;
      d.speculative = true;
      d.spec_max = kSyncEntryMax;
      const uint64_t last = std::min(end, B[t] + kSyncSearch);
      for (; o < last; ++o) {
        d.c.off = o;
        d.c.err = CDB_OK;
        uint32_t k = 0;
        for (; k < kSyncEntries && d.c.off < end; ++k) {
          scratch.offset.clear();
          scratch.kind.clear();
          const uint64_t at = d.c.off;
          // (a wrong offset can read a huge "length" that still fits the stream and land on true
          // entries after it: sync points only come from chains of small entries)
          if (!d.data_entry() || d.c.off - at > kSyncEntryMax) break;
        }
        if (k == kSyncEntries) break;
      }
      if (o >= last) {
        P.ok = false;
        P.stop = B[t];
        return;
      }
    }
    walk(o, B[t + 1], P);
  };
  const auto tp0 = std::chrono::steady_clock::now();
  {
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
  }
  const auto tp1 = std::chrono::steady_clock::now();
  if (std::getenv("CDB_SELFTEST_VERBOSE"))
    for (uint32_t t = 0; t < T; ++t)
      fprintf(stderr, "part %u: B %llu ok %d n %zu first %llu stop %llu\n", t, (unsigned long long)B[t], (int)parts[t].ok,
              parts[t].off.size(), (unsigned long long)(parts[t].off.empty() ? 0 : parts[t].off[0]),
              (unsigned long long)parts[t].stop);
  // stitch
  const size_t base_n = idx->offset.size();
  idx->offset.reserve(base_n + cnt);
  idx->kind.reserve(base_n + cnt);
  auto rollback = [&]() {
    idx->offset.resize(base_n);
    idx->kind.resize(base_n);
    return false;
  };
  uint64_t cur = S, got = 0;
  uint32_t rewalks = 0;
  Decoder d{Cursor{base, end}, b, base};  // entries the threads' chains do not hold
  EntryIndex scratch;
  d.idx = &scratch;
  d.speculative = true;
  for (uint32_t t = 0; t < T && got < cnt; ++t) {
    Part& P = parts[t];
    // a speculative chain either is the true one or joins it within a few entries (parsing
    // from a shared offset is deterministic): entries from cur are parsed here until they reach
    // an offset thread t recorded, then thread t's entries are taken from there
    auto join = std::lower_bound(P.off.begin(), P.off.end(), cur);
    bool walked = false;
    while (got < cnt && cur < B[t + 1] && !(join != P.off.end() && *join == cur)) {
      scratch.offset.clear();
      scratch.kind.clear();
      d.c.off = cur;
      if (!d.data_entry()) return rollback();  // an error on the true chain: the sequential loop reports it
      idx->offset.push_back(cur);
      idx->kind.push_back(0);
      ++got;
      cur = d.c.off;
      walked = true;
      while (join != P.off.end() && *join < cur) ++join;
    }
    rewalks += walked;
    if (got >= cnt || join == P.off.end() || *join != cur) continue;  // (cur left range t)
    const uint64_t take = std::min<uint64_t>((uint64_t)(P.off.end() - join), cnt - got);
    idx->offset.insert(idx->offset.end(), join, join + take);
    idx->kind.resize(idx->kind.size() + take, 0);
    got += take;
    if (got < cnt) {
      if (!P.ok) return rollback();  // thread t's chain (the true one) failed there
      cur = P.stop;
    }
  }
  if (got < cnt) return rollback();  // (the stream ended first: the sequential loop reports where)
  if (std::getenv("CDB_SELFTEST_TIMING"))
    fprintf(stderr, "parallel_datas: %u threads %.1f ms, stitch %.1f ms (%u ranges parsed again), %llu entries\n", T,
            std::chrono::duration<double, std::milli>(tp1 - tp0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp1).count(), rewalks,
            (unsigned long long)cnt);
  // the section ends after its last entry: parse that entry again for its end offset
  Decoder e{Cursor{base, end}, b, base};
  EntryIndex last;
  e.idx = &last;
  e.c.off = idx->offset.back();
  if (!e.data_entry()) return rollback();
  c.off = e.c.off;
  return true;
}

}  // namespace

struct IndexCursor {
  Decoder d;
  uint32_t flags;
};

int index_resume(IndexCursor* ic, uint64_t datas_end, size_t* err_off) {
  ic->d.c.off = datas_end;
  ic->d.c.err = CDB_OK;
  *err_off = 0;
  return ic->d.loop(ic->flags, err_off);
}
void index_cursor_free(IndexCursor* ic) { delete ic; }

bool index_data_entry_end(const Batch& b, uint64_t off, uint64_t* end) {
  Decoder d{Cursor{b.raw.data(), b.raw.size()}, const_cast<Batch*>(&b), b.raw.data()};
  EntryIndex scratch;
  d.idx = &scratch;
  d.c.off = off;
  if (!d.data_entry()) return false;
  *end = d.c.off;
  return true;
}

int decode_snapshot(const uint8_t* buf, size_t len, uint32_t flags, Batch* out, size_t* err_off) {
  adopt_raw(out, buf, len);
  Decoder d{Cursor{out->raw.data(), out->raw.size()}, out, out->raw.data()};
  *err_off = 0;
  return d.run(flags, err_off);
}

int index_snapshot(const uint8_t* buf, size_t len, uint32_t flags, Batch* out, EntryIndex* idx, size_t* err_off,
                   DeferredCrc* crc, uint32_t threads, DeferredDatas* defer, IndexCursor** cursor) {
  if (buf) adopt_raw(out, buf, len);
  Decoder d{Cursor{out->raw.data(), out->raw.size()}, out, out->raw.data()};
  d.idx = idx;
  d.dcrc = crc;
  d.threads = threads;
  d.defer = defer && cursor ? defer : nullptr;
  if (!d.defer) {
    idx->offset.reserve(len / 48 + 16);  // generator-shaped streams run ~58 bytes per entry
    idx->kind.reserve(len / 48 + 16);
  }
  *err_off = 0;
  const int rc = d.run(flags, err_off);
  if (rc == kIndexDeferred) *cursor = new IndexCursor{d, flags};
  return rc;
}

// The entries the GPU found too large for its per-entry dedup: decoded here, exactly as
// decode_snapshot would, into `side` (rows in entry order, src fields relative to `side`).
bool decode_entry_children(const Batch& b, uint64_t off, uint64_t kh, uint64_t kf, Batch* side, uint64_t* total) {
  Decoder d{Cursor{b.raw.data(), b.raw.size()}, side, b.raw.data()};
  d.c.off = off;
  ByteRef k;
  uint64_t ct, ut, dt;
  uint8_t tag;
  if (!d.c.span(&k) || !d.c.u64(&ct) || !d.c.u64(&ut) || !d.c.u64(&dt) || !d.c.u8(&tag)) return false;
  *total = 0;
  if (tag == TAG_COUNTER) return d.counter(kh, kf, total);
  if (tag == TAG_SET || tag == TAG_DICT) return d.lwwhash(kh, kf, tag == TAG_DICT);
  return true;
}

}  // namespace cdb
