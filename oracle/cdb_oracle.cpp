// ConstDB merge ORACLE (C++ restatement) — TEST INFRASTRUCTURE ONLY.
//
// Same restatement as oracle/constdb_oracle.py, in C++ for medium sizes and for the CPU
// baseline (bench.py cpu_baseline, kind "port"). It is never linked into the product
// (constdb_amd/libcdbmerge.so); tests/ and bench.py load it with ctypes as the checker.
//
// The fold mirrors the reference's single-threaded main-task merge:
//   replica/pull.rs:116-159 (Data -> DB::merge_entry, Deletes -> DB::delete,
//   Expires -> DB::expire_at) -> db.rs:31-43 -> object.rs:63-83 ->
//   type_counter.rs:59-91 / crdt/lwwhash.rs:87-128,176-181,319-323.
// Decoding mirrors snapshot.rs:120-295, object.rs:110-129, type_counter.rs:111-126,
// crdt/lwwhash.rs:207-226,341-358. Parity pinning: see the header of constdb_oracle.py.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

// ---------------------------------------------------------------- CRC-64/Jones
struct CrcTable {
  uint64_t t[256];
  CrcTable() {
    for (int i = 0; i < 256; ++i) {
      uint64_t c = (uint64_t)i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x95AC9329AC4BC9B5ULL : c >> 1;
      t[i] = c;
    }
  }
};
const CrcTable kCrc;
inline uint64_t crc_update(uint64_t crc, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i) crc = kCrc.t[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
  return crc;
}

enum Status : int {  // mirrors cdb_status values of include/cdb_merge.h
  OK = 0, INVALID_SNAPSHOT = 1, INVALID_CHECKSUM = 2, INVALID_TYPE = 3, IO_ERROR = 4,
  DICT_PANIC = 5, BAD_ARG = 6
};

enum : uint8_t { ENC_COUNTER = 0, ENC_BYTES = 3, ENC_DICT = 4, ENC_SET = 5 };

// ---------------------------------------------------------------- CRDT types
struct LWWHash {  // crdt/lwwhash.rs:11-16
  int32_t size = 0;
  std::unordered_map<std::string, std::pair<uint64_t, std::string>> add;
  std::unordered_map<std::string, uint64_t> del;

  bool set(const std::string& k, const std::string& v, uint64_t t) {  // lwwhash.rs:87-107
    auto d = del.find(k);
    if (d != del.end() && d->second > t) return false;
    auto a = add.find(k);
    if (a != add.end()) {
      if (a->second.first > t) return false;
      a->second.second = v;
      a->second.first = t;
    } else {
      if (d != del.end()) del.erase(d);
      add.emplace(k, std::make_pair(t, v));
    }
    size += 1;
    return true;
  }
  bool rem(const std::string& k, uint64_t t) {  // lwwhash.rs:109-128
    auto a = add.find(k);
    if (a != add.end() && a->second.first > t) return false;
    auto d = del.find(k);
    if (d != del.end()) {
      if (d->second > t) return false;
      d->second = t;
    } else {
      del.emplace(k, t);
      if (a != add.end()) add.erase(a);
    }
    size -= 1;
    return true;
  }
  // Set::merge / Dict::merge loop (lwwhash.rs:176-179, 319-323) over SetIter/DictIter
  // (lwwhash.rs:229-248, 361-380): only adds not shadowed by a strictly later del.
  void merge_from(const LWWHash& o) {
    for (const auto& kv : o.add) {
      auto d = o.del.find(kv.first);
      if (d != o.del.end() && d->second > kv.second.first) continue;
      set(kv.first, kv.second.second, kv.second.first);
    }
  }
};

struct Counter {  // type_counter.rs:18-22
  int64_t sum = 0;
  std::unordered_map<uint64_t, std::pair<int64_t, uint64_t>> data;
  void merge(const Counter& o) {  // type_counter.rs:59-87
    for (auto& kv : data) {
      auto it = o.data.find(kv.first);
      if (it != o.data.end()) {
        int64_t vv = it->second.first; uint64_t tt = it->second.second;
        if (tt > kv.second.second) kv.second.first = vv;
        else if (tt == kv.second.second) kv.second.first = std::max(kv.second.first, vv);
      }
    }
    for (const auto& kv : o.data) {
      auto it = data.find(kv.first);
      if (it != data.end()) {
        int64_t vv = kv.second.first; uint64_t tt = kv.second.second;
        if (tt > it->second.second) it->second.first = vv;
        else if (tt == it->second.second) it->second.first = std::max(it->second.first, vv);
      } else {
        data.emplace(kv.first, kv.second);
      }
    }
    uint64_t s = 0;  // cal_sum, wrapping i64 (release build)
    for (const auto& kv : data) s += (uint64_t)kv.second.first;
    sum = (int64_t)s;
  }
};

struct Object {  // object.rs:11-17
  uint64_t ct = 0, ut = 0, dt = 0;
  uint8_t tag = 0;
  std::string bytes;
  std::unique_ptr<Counter> counter;
  std::unique_ptr<LWWHash> hash;
};

// ---------------------------------------------------------------- loader
struct Reader {
  const uint8_t* p; size_t n; size_t off = 0; uint64_t crc = 0; int err = OK;
  bool need(size_t k) {
    if (k > n - off) { err = IO_ERROR; return false; }
    return true;
  }
  const uint8_t* bytes(size_t k) {  // snapshot.rs:266-274
    if (!need(k)) return nullptr;
    const uint8_t* q = p + off;
    crc = crc_update(crc, q, k);
    off += k;
    return q;
  }
  bool byte(uint8_t* b) { const uint8_t* q = bytes(1); if (!q) return false; *b = *q; return true; }
  bool integer(int64_t* out) {  // snapshot.rs:243-264
    uint8_t f;
    if (!byte(&f)) return false;
    switch ((f >> 6) & 3) {
      case 0: *out = f & 0x3F; return true;
      case 1: { uint8_t b; if (!byte(&b)) return false; *out = ((int64_t)(f & 0x3F) << 8) | b; return true; }
      case 2: { const uint8_t* q = bytes(3); if (!q) return false;
                *out = ((int64_t)(f & 0x3F) << 24) | ((int64_t)q[0] << 16) | ((int64_t)q[1] << 8) | q[2]; return true; }
      default: { const uint8_t* q = bytes(8); if (!q) return false; uint64_t v = 0;
                 for (int i = 0; i < 8; ++i) { v = (v << 8) | q[i]; } *out = (int64_t)v; return true; }
    }
  }
  bool len(size_t* out) {
    int64_t v; if (!integer(&v)) return false;
    if (v < 0) { err = IO_ERROR; return false; }
    *out = (size_t)v; return true;
  }
  bool str(std::string* s) {
    size_t l; if (!len(&l)) return false;
    const uint8_t* q = bytes(l); if (!q) return false;
    s->assign((const char*)q, l); return true;
  }
};

struct Entry {  // SnapshotEntry data-carrying variants (snapshot.rs:303-312)
  enum Kind : uint8_t { DATA, EXPIRES, DELETES } kind;
  std::string key;
  uint64_t t = 0;
  std::unique_ptr<Object> obj;
};

bool load_object(Reader& r, Object* o) {  // object.rs:110-129
  int64_t ct, mt, dt;
  if (!r.integer(&ct) || !r.integer(&mt) || !r.integer(&dt)) return false;
  o->ct = (uint64_t)ct; o->ut = (uint64_t)mt; o->dt = (uint64_t)dt;
  uint8_t tag; if (!r.byte(&tag)) return false;
  o->tag = tag;
  if (tag == ENC_COUNTER) {  // type_counter.rs:111-126
    size_t cnt; if (!r.len(&cnt)) return false;
    o->counter.reset(new Counter());
    uint64_t total = 0;
    for (size_t i = 0; i < cnt; ++i) {
      int64_t nid, v, t;
      if (!r.integer(&nid) || !r.integer(&v) || !r.integer(&t)) return false;
      o->counter->data[(uint64_t)nid] = {v, (uint64_t)t};
      total += (uint64_t)v;
    }
    o->counter->sum = (int64_t)total;
  } else if (tag == ENC_BYTES) {  // object.rs:114-118
    if (!r.str(&o->bytes)) return false;
  } else if (tag == ENC_SET || tag == ENC_DICT) {  // lwwhash.rs:207-226 / 341-358
    o->hash.reset(new LWWHash());
    size_t na; if (!r.len(&na)) return false;
    std::string k, v;
    for (size_t i = 0; i < na; ++i) {
      int64_t t;
      if (!r.str(&k) || !r.integer(&t)) return false;
      v.clear();
      if (tag == ENC_DICT && !r.str(&v)) return false;
      o->hash->set(k, v, (uint64_t)t);
    }
    size_t nd; if (!r.len(&nd)) return false;
    for (size_t i = 0; i < nd; ++i) {
      int64_t t;
      if (!r.str(&k) || !r.integer(&t)) return false;
      o->hash->rem(k, (uint64_t)t);
    }
  } else {
    r.err = INVALID_TYPE;  // object.rs:121
    return false;
  }
  return true;
}

// Decodes one snapshot (writer layout; checksum_mode 1 = the reference loader's quirk,
// snapshot.rs:207-213) into the ordered list of Data/Expires/Deletes entries.
int decode(const uint8_t* buf, size_t n, int checksum_mode, std::vector<Entry>* out,
           size_t* err_off) {
  Reader r{buf, n};
  auto fail = [&](int e) { *err_off = r.off; return e == OK ? INVALID_SNAPSHOT : e; };
  if (!r.bytes(7) || !r.bytes(4)) return fail(r.err);  // magic (unchecked) + version
  int64_t iv; std::string s;
  if (!r.integer(&iv) || !r.str(&s) || !r.str(&s) || !r.integer(&iv)) return fail(r.err);
  for (;;) {
    uint8_t flag; if (!r.byte(&flag)) return fail(r.err);  // convert_stat, snapshot.rs:222-241
    if (flag == 3) {  // ReplicaAdd
      int64_t a, b, c;
      if (!r.integer(&a) || !r.integer(&b) || !r.str(&s) || !r.str(&s) || !r.integer(&c)) return fail(r.err);
    } else if (flag == 4) {  // ReplicaDel
      int64_t a;
      if (!r.str(&s) || !r.integer(&a)) return fail(r.err);
    } else if (flag == 5 || flag == 6 || flag == 7) {
      size_t cnt; if (!r.len(&cnt)) return fail(r.err);
      for (size_t i = 0; i < cnt; ++i) {
        Entry e;
        e.kind = flag == 5 ? Entry::DATA : (flag == 6 ? Entry::EXPIRES : Entry::DELETES);
        if (!r.str(&e.key)) return fail(r.err);
        if (flag == 5) {
          e.obj.reset(new Object());
          if (!load_object(r, e.obj.get())) return fail(r.err);
        } else {
          int64_t t; if (!r.integer(&t)) return fail(r.err);
          e.t = (uint64_t)t;
        }
        out->push_back(std::move(e));
      }
    } else if (flag == 8) {
      if (checksum_mode == 1) {
        int64_t got; if (!r.integer(&got)) return fail(r.err);
        if ((uint64_t)got != r.crc) return fail(INVALID_CHECKSUM);
      } else {
        uint64_t expect = r.crc;
        const uint8_t* q = r.bytes(8); if (!q) return fail(r.err);
        uint64_t got = 0;
        for (int i = 7; i >= 0; --i) got = (got << 8) | q[i];
        if (got != expect) return fail(INVALID_CHECKSUM);
      }
      return OK;
    } else {
      return fail(INVALID_SNAPSHOT);  // snapshot.rs:236-238
    }
  }
}

// ---------------------------------------------------------------- DB
struct DB {  // db.rs:10-15
  std::unordered_map<std::string, std::unique_ptr<Object>> data;
  std::unordered_map<std::string, uint64_t> expires, deletes;
  std::vector<std::pair<std::string, uint64_t>> garbages;  // key-only (field path is dead)
  uint64_t type_conflicts = 0, dict_merges = 0;

  int merge_entry(std::string&& key, std::unique_ptr<Object>&& v, bool dict_panic) {  // db.rs:31-43
    auto it = data.find(key);
    if (it == data.end()) { data.emplace(std::move(key), std::move(v)); return OK; }
    Object& o = *it->second;
    if (o.tag != v->tag) { type_conflicts++; return OK; }  // object.rs:80 -> error! log
    switch (o.tag) {  // object.rs:67-81
      case ENC_COUNTER: o.counter->merge(*v->counter); break;
      case ENC_BYTES:
        if (o.ct < v->ct) o.bytes = std::move(v->bytes);
        o.ct = std::max(o.ct, v->ct); o.dt = std::max(o.dt, v->dt); o.ut = std::max(o.ut, v->ut);
        break;
      case ENC_DICT:
        dict_merges++;
        o.hash->merge_from(*v->hash);
        if (dict_panic) return DICT_PANIC;  // lwwhash.rs:180 unimplemented!()
        break;
      default: o.hash->merge_from(*v->hash); break;
    }
    return OK;
  }
  void gc(uint64_t tombstone) {  // db.rs:82-119 (LIFO; stops at the first t > tombstone)
    while (!garbages.empty()) {
      auto g = std::move(garbages.back());
      garbages.pop_back();
      if (g.second > tombstone) break;
      auto d = deletes.find(g.first);
      if (d != deletes.end() && d->second == g.second) deletes.erase(d);
    }
  }
  uint64_t gc_member_tombstones(uint64_t wm) {  // BUILD EXTENSION (see constdb_oracle.py)
    uint64_t n = 0;
    for (auto& kv : data) {
      Object& o = *kv.second;
      if (o.tag != ENC_SET && o.tag != ENC_DICT) continue;
      for (auto it = o.hash->del.begin(); it != o.hash->del.end();) {
        if (!o.hash->add.count(it->first) && it->second < wm) { it = o.hash->del.erase(it); ++n; }
        else ++it;
      }
    }
    return n;
  }
};

std::string hex(const std::string& s) {
  static const char* d = "0123456789abcdef";
  std::string o; o.resize(s.size() * 2);
  for (size_t i = 0; i < s.size(); ++i) { o[2*i] = d[(uint8_t)s[i] >> 4]; o[2*i+1] = d[(uint8_t)s[i] & 15]; }
  return o;
}

// Canonical dump — identical text format to constdb_oracle.canonical_dump().
std::string canonical_dump(const DB& db) {
  std::string out;
  std::vector<const std::string*> keys;
  for (const auto& kv : db.data) keys.push_back(&kv.first);
  std::sort(keys.begin(), keys.end(), [](const std::string* a, const std::string* b) { return *a < *b; });
  char buf[128];
  for (const std::string* k : keys) {
    const Object& o = *db.data.at(*k);
    snprintf(buf, sizeof buf, " %u %llu %llu %llu\n", o.tag, (unsigned long long)o.ct,
             (unsigned long long)o.ut, (unsigned long long)o.dt);
    out += "K " + hex(*k) + buf;
    if (o.tag == ENC_BYTES) {
      out += " V " + hex(o.bytes) + "\n";
    } else if (o.tag == ENC_COUNTER) {
      snprintf(buf, sizeof buf, " S %lld\n", (long long)o.counter->sum);
      out += buf;
      std::vector<uint64_t> nodes;
      for (const auto& kv : o.counter->data) nodes.push_back(kv.first);
      std::sort(nodes.begin(), nodes.end());
      for (uint64_t nd : nodes) {
        const auto& vt = o.counter->data.at(nd);
        snprintf(buf, sizeof buf, " N %llu %lld %llu\n", (unsigned long long)nd,
                 (long long)vt.first, (unsigned long long)vt.second);
        out += buf;
      }
    } else {
      std::vector<const std::string*> ms;
      for (const auto& kv : o.hash->add) ms.push_back(&kv.first);
      for (const auto& kv : o.hash->del) if (!o.hash->add.count(kv.first)) ms.push_back(&kv.first);
      std::sort(ms.begin(), ms.end(), [](const std::string* a, const std::string* b) { return *a < *b; });
      for (const std::string* m : ms) {
        auto a = o.hash->add.find(*m);
        if (a != o.hash->add.end()) {
          snprintf(buf, sizeof buf, " %llu", (unsigned long long)a->second.first);
          out += " A " + hex(*m) + buf;
          if (o.tag == ENC_DICT) out += " " + hex(a->second.second);
          out += "\n";
        }
        auto d = o.hash->del.find(*m);
        if (d != o.hash->del.end()) {
          snprintf(buf, sizeof buf, " %llu\n", (unsigned long long)d->second);
          out += " D " + hex(*m) + buf;
        }
      }
    }
  }
  auto side = [&](const std::unordered_map<std::string, uint64_t>& m, const char* tag) {
    std::vector<const std::string*> ks;
    for (const auto& kv : m) ks.push_back(&kv.first);
    std::sort(ks.begin(), ks.end(), [](const std::string* a, const std::string* b) { return *a < *b; });
    for (const std::string* k : ks) {
      snprintf(buf, sizeof buf, " %llu\n", (unsigned long long)m.at(*k));
      out += std::string(tag) + " " + hex(*k) + buf;
    }
  };
  side(db.expires, "X");
  side(db.deletes, "R");
  return out;
}

// Applies the decoded entries of snapshots in pos order (replica/pull.rs:120-158).
int fold(std::vector<std::vector<Entry>>& snaps, DB& db, bool dict_panic) {
  for (auto& entries : snaps) {
    for (auto& e : entries) {
      if (e.kind == Entry::DATA) {
        int st = db.merge_entry(std::move(e.key), std::move(e.obj), dict_panic);
        if (st != OK) return st;
      } else if (e.kind == Entry::DELETES) {  // db.rs:73-76
        db.deletes[e.key] = e.t;
        db.garbages.emplace_back(e.key, e.t);
      } else {  // db.rs:68-71
        db.expires[e.key] = e.t;
      }
    }
  }
  return OK;
}

}  // namespace

extern "C" {

struct cdbo_stats {
  uint64_t type_conflicts, dict_merges, member_tombstones_gced;
  size_t err_offset;
  int32_t err_snapshot;
};

// flags: bit0 dict_panic, bit1 reference checksum quirk, bit2 run DB::gc(gc_wm),
//        bit3 run the member-tombstone GC extension at gc_wm.
int cdbo_fold(const uint8_t* const* bufs, const size_t* lens, int n, int flags, uint64_t gc_wm,
              char** dump, size_t* dump_len, cdbo_stats* st) {
  std::vector<std::vector<Entry>> snaps(n);
  std::memset(st, 0, sizeof *st);
  for (int i = 0; i < n; ++i) {
    int rc = decode(bufs[i], lens[i], (flags >> 1) & 1, &snaps[i], &st->err_offset);
    if (rc != OK) { st->err_snapshot = i; return rc; }
  }
  DB db;
  int rc = fold(snaps, db, flags & 1);
  st->type_conflicts = db.type_conflicts;
  st->dict_merges = db.dict_merges;
  if (rc != OK) return rc;
  if (flags & 4) db.gc(gc_wm);
  if (flags & 8) st->member_tombstones_gced = db.gc_member_tombstones(gc_wm);
  std::string d = canonical_dump(db);
  *dump = (char*)std::malloc(d.size() + 1);
  std::memcpy(*dump, d.data(), d.size());
  (*dump)[d.size()] = 0;
  *dump_len = d.size();
  return OK;
}

void cdbo_free(void* p) { std::free(p); }

static Entry clone_entry(const Entry& e) {  // deep copy (Entry owns its object through unique_ptrs)
  Entry c;
  c.kind = e.kind;
  c.key = e.key;
  c.t = e.t;
  if (e.obj) {
    c.obj.reset(new Object());
    Object& o = *c.obj;
    o.ct = e.obj->ct; o.ut = e.obj->ut; o.dt = e.obj->dt; o.tag = e.obj->tag; o.bytes = e.obj->bytes;
    if (e.obj->counter) o.counter.reset(new Counter(*e.obj->counter));
    if (e.obj->hash) o.hash.reset(new LWWHash(*e.obj->hash));
  }
  return c;
}

// CPU baseline: decodes once (untimed), then times ONLY the sequential fold into a fresh DB
// (the reference's merge loop minus its per-entry DEBUG formatting), best of `reps`; every rep
// folds its own untimed copy of the decoded entries. Returns the best fold time in ns;
// *entries = entries (Data/Expires/Deletes) folded per run.
int64_t cdbo_time_fold(const uint8_t* const* bufs, const size_t* lens, int n, int reps,
                       uint64_t* entries) {
  std::vector<std::vector<Entry>> base(n);
  size_t eo;
  uint64_t cnt = 0;
  for (int i = 0; i < n; ++i) {
    if (decode(bufs[i], lens[i], 0, &base[i], &eo) != OK) return -1;
    cnt += base[i].size();  // Data + Expires + Deletes entries
  }
  *entries = cnt;
  int64_t best = -1;
  for (int r = 0; r < reps; ++r) {
    std::vector<std::vector<Entry>> snaps(n);
    for (int i = 0; i < n; ++i) {
      snaps[i].reserve(base[i].size());
      for (const Entry& e : base[i]) snaps[i].push_back(clone_entry(e));
    }
    DB db;
    db.data.reserve(1024);
    auto t0 = std::chrono::steady_clock::now();
    fold(snaps, db, false);
    auto t1 = std::chrono::steady_clock::now();
    int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    if (best < 0 || ns < best) best = ns;
  }
  return best;
}

}  // extern "C"
