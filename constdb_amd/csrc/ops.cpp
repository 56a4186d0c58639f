// Host decode of a partial-replication stream: the RESP messages a Puller
// receives after the snapshot (replica/pull.rs:160-235) become columnar op rows for the
// device apply (ops_apply.hip). This pass does what the reference does per message before a
// handler touches the DB: RESP framing (conn/buf_read.rs:114-210), the uuid gate
// (pull.rs:199-209), the command lookup (cmd.rs:39-41) and each handler's argument parsing
// (cmd.rs:348-397 NextArg; the handlers in cmd.rs, type_counter.rs, type_set.rs,
// type_hash.rs). Everything that reads or writes the DB happens on the device.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "batch.h"
#include "ops.h"

namespace cdb {
namespace {

struct Item {       // one RESP value (top-level argument of a message)
  char kind;        // '+', '-', ':', '$', 'n' (nil), '*'
  uint64_t off, len;  // payload bytes inside the stream (strings; the digits for ':')
  int64_t ival;     // ':' value
};

// bytes2i64 (lib/utils.rs:3-28), release-build wrapping arithmetic.
bool bytes2i64(const uint8_t* p, uint64_t n, int64_t* out) {
  if (n == 0) return false;
  uint64_t r = 0;
  bool invalid = true, neg = false;
  for (uint64_t i = 0; i < n; ++i) {
    if (i == 0 && p[i] == '-') {
      neg = true;
      continue;
    }
    if (p[i] >= '0' && p[i] <= '9') {
      invalid = false;
      r = r * 10 + (uint64_t)(p[i] - '0');
    } else {
      break;
    }
  }
  if (invalid) return false;
  *out = (int64_t)(neg ? 0 - r : r);
  return true;
}

struct Reader {
  const uint8_t* b;
  uint64_t n;
  // index of the '\n' of the first "\r\n" at or after `cur` (buf_read.rs:202-210)
  bool until_crlf(uint64_t cur, uint64_t* at) const {
    for (uint64_t i = cur; i + 1 < n; ++i)
      if (b[i] == '\r' && b[i + 1] == '\n') {
        *at = i + 1;
        return true;
      }
    return false;
  }
  // parse_msg_inner (buf_read.rs:114-171). Returns 0 ok, 1 malformed, 2 truncated.
  // The items of a top-level array (depth 0) go to `items`.
  int parse(uint64_t cur, uint64_t* size, int depth, std::vector<Item>* items, Item* self) {
    if (cur >= n) return 2;
    const uint8_t t = b[cur];
    uint64_t s;
    Item it{};
    switch (t) {
      case '+':
      case '-':
        if (!until_crlf(cur + 1, &s)) return 2;
        it = Item{(char)t, cur + 1, s - 1 - (cur + 1), 0};
        *size = s - cur + 1;
        break;
      case ':':
        if (!until_crlf(cur + 1, &s)) return 2;
        if (!bytes2i64(b + cur + 1, s - 1 - (cur + 1), &it.ival)) return 1;
        it.kind = ':';
        it.off = cur + 1;
        it.len = s - 1 - (cur + 1);
        *size = s - cur + 1;
        break;
      case '$': {  // read_bulk_string (buf_read.rs:173-200)
        uint64_t he;
        if (!until_crlf(cur + 1, &he)) return 2;
        int64_t cnt;
        if (!bytes2i64(b + cur + 1, he - 1 - (cur + 1), &cnt)) return 1;
        if (cnt == -1) {
          it.kind = 'n';
          *size = 5;
          break;
        }
        if (cnt < 0) return 1;
        uint64_t se;
        if (!until_crlf(he, &se)) return 2;
        if (se - he != (uint64_t)cnt + 2) return 1;  // a payload holding "\r\n" fails here too
        it = Item{'$', he + 1, (uint64_t)cnt, 0};
        *size = se - cur + 1;
        break;
      }
      case '*': {
        uint64_t le;
        if (!until_crlf(cur + 1, &le)) return 2;
        int64_t cnt;
        if (!bytes2i64(b + cur + 1, le - 1 - (cur + 1), &cnt)) return 1;
        if (cnt < 0) return 1;  // Vec::with_capacity(negative as usize) aborts the reference
        uint64_t sub = le + 1;
        for (int64_t i = 0; i < cnt; ++i) {
          uint64_t sz;
          Item child;
          const int rc = parse(sub, &sz, depth + 1, items, &child);
          if (rc) return rc;
          if (depth == 0 && items) items->push_back(child);
          sub += sz;
        }
        it.kind = '*';
        *size = sub - cur;
        break;
      }
      default:
        return 1;
    }
    if (self) *self = it;
    return 0;
  }
};

// NextArg (cmd.rs:348-397) over the items of one message; every call consumes one item.
struct Args {
  const std::vector<Item>& it;
  size_t i;
  std::vector<uint8_t>* arena;  // decimal forms of ':' arguments that differ from the literal
  const uint8_t* raw;
  bool next_bytes(ByteRef* out) {
    if (i >= it.size()) return false;  // WrongArity
    const Item& x = it[i++];
    if (x.kind == ':') {  // get_int_bytes (resp.rs:20-26): the decimal form of the value
      const std::string d = std::to_string(x.ival);
      if (d.size() == x.len && std::memcmp(d.data(), raw + x.off, x.len) == 0) {
        *out = ByteRef{x.off, x.len};
      } else {
        *out = ByteRef{(uint64_t)arena->size() | (1ull << 63), d.size()};
        arena->insert(arena->end(), d.begin(), d.end());
      }
      return true;
    }
    if (x.kind == '+' || x.kind == '-' || x.kind == '$') {
      *out = ByteRef{x.off, x.len};
      return true;
    }
    return false;  // nil / array: "should be non-array type"
  }
  bool next_i64(int64_t* v) {
    if (i >= it.size()) return false;
    const Item& x = it[i++];
    if (x.kind == ':') {
      *v = x.ival;
      return true;
    }
    if (x.kind == '+' || x.kind == '$') return bytes2i64(raw + x.off, x.len, v);
    return false;
  }
  bool next_u64(uint64_t* v) {
    int64_t s;
    if (!next_i64(&s) || s < 0) return false;
    *v = (uint64_t)s;
    return true;
  }
};

bool name_is(const uint8_t* raw, const ByteRef& r, const char* lower) {
  const size_t n = std::strlen(lower);
  if (r.len != n || (r.off >> 63)) return false;
  for (size_t i = 0; i < n; ++i) {
    uint8_t c = raw[r.off + i];
    if (c >= 'A' && c <= 'Z') c = (uint8_t)(c - 'A' + 'a');
    if (c != (uint8_t)lower[i]) return false;
  }
  return true;
}

}  // namespace

int decode_ops(const uint8_t* buf, size_t len, uint64_t uuid_he_sent, Batch* out, cdb_ops_info* info,
               size_t* err_off) {
  Batch& b = *out;
  adopt_raw(&b, buf, len);
  cdb_ops_info& st = *info;
  std::memset(&st, 0, sizeof st);
  st.uuid_he_sent = uuid_he_sent;
  std::vector<uint8_t> arena;
  Reader rd{buf, len};
  std::vector<Item> items;
  std::vector<ByteRef> mem, val;
  struct NodeArg { uint64_t node; int64_t v; };
  std::vector<NodeArg> nodes;
  uint64_t cur = 0;
  bool truncated = false;
  while (cur < len) {
    items.clear();
    uint64_t size = 0;
    Item top;
    const int rc = rd.parse(cur, &size, 0, &items, &top);
    if (rc == 1) {
      *err_off = cur;
      return CDB_INVALID_REQUEST_MSG;
    }
    if (rc == 2) {  // NeedMoreMsg: the ops of the complete messages are kept
      truncated = true;
      break;
    }
    const uint64_t msg_at = cur;
    cur += size;
    ++st.n_messages;
    if (top.kind != '*') {  // "should be array" (pull.rs:187-190)
      ++st.lost;
      continue;
    }
    Args a{items, 0, &arena, buf};
    ByteRef name;
    if (!a.next_bytes(&name)) {
      ++st.lost;
      continue;
    }
    if (name_is(buf, name, "replack")) {  // pull.rs:226-228
      uint64_t acked;
      if (a.next_u64(&acked)) {
        st.uuid_he_acked = acked;
        ++st.replacks;
      } else {
        ++st.lost;
      }
      continue;
    }
    if (!name_is(buf, name, "replicate")) {
      ++st.lost;
      continue;
    }
    uint64_t nodeid, last_uuid, cur_uuid;
    if (!a.next_u64(&nodeid) || !a.next_u64(&last_uuid)) {
      ++st.lost;
      continue;
    }
    if (st.uuid_he_sent < last_uuid) {  // ReplicateCommandsLost (pull.rs:201-204)
      ++st.lost;
      continue;
    }
    if (st.uuid_he_sent > last_uuid) {  // duplicated commands (pull.rs:205-206)
      ++st.duplicates;
      continue;
    }
    ByteRef cmd;
    if (!a.next_u64(&cur_uuid) || !a.next_bytes(&cmd)) {
      ++st.lost;
      continue;
    }
    static const struct { const char* name; uint32_t code; } kCmds[] = {
        {"set", OP_SET}, {"delbytes", OP_DELBYTES}, {"incr", OP_INCR}, {"decr", OP_DECR},
        {"delcnt", OP_DELCNT}, {"sadd", OP_SADD}, {"srem", OP_SREM}, {"delset", OP_DELSET},
        {"hset", OP_HSET}, {"hdel", OP_HDEL}, {"deldict", OP_DELDICT}};
    static const char* kUnsupported[] = {"spop", "del", "node", "replicas", "sync", "meet", "client",
                                         "repllog", "info", "get", "desc", "smembers", "hget", "hgetall"};
    uint32_t code = 0;
    bool unsup = false;
    if (!(cmd.off >> 63)) {  // a command name given as an integer matches nothing
      for (const auto& c : kCmds)
        if (name_is(buf, cmd, c.name)) code = c.code;
      for (const char* u : kUnsupported)
        if (name_is(buf, cmd, u)) unsup = true;
    }
    st.uuid_he_sent = cur_uuid;  // advanced for every command that reaches Cmd::new (pull.rs:214-223)
    if (!code) {
      ++(unsup ? st.unsupported : st.unknown);
      continue;
    }
    ++st.applied;
    // ---- the handler's argument parsing, up to the point where it first touches the DB
    Args r{items, a.i, &arena, buf};
    ByteRef key, value{0, 0};
    mem.clear();
    val.clear();
    nodes.clear();
    bool err = false;       // the handler returns Err (counted; uuid already advanced)
    bool touches = true;    // false: the error came before the DB was touched
    if (!r.next_bytes(&key)) {
      err = true;
      touches = false;
    } else if (code == OP_SET) {  // cmd.rs:188-210
      if (!r.next_bytes(&value)) err = true, touches = false;
    } else if (code == OP_INCR || code == OP_DECR) {  // type_counter.rs:169-204
      nodes.push_back(NodeArg{nodeid, code == OP_INCR ? 1 : -1});
    } else if (code == OP_DELCNT) {  // type_counter.rs:142-167: pairs up to the first bad node id;
      uint64_t nd;                   // a bad value after a good node id errors AFTER the pairs ran
      while (r.next_u64(&nd)) {
        int64_t v;
        if (!r.next_i64(&v)) {
          err = true;
          break;
        }
        nodes.push_back(NodeArg{nd, v});
      }
    } else if (code == OP_SADD || code == OP_SREM || code == OP_HDEL) {  // members up to the first non-bytes
      ByteRef m;
      while (r.next_bytes(&m)) mem.push_back(m);
    } else if (code == OP_HSET) {  // type_hash.rs:11-20: an odd count errors before the DB is touched
      ByteRef f, v;
      while (r.next_bytes(&f)) {
        if (!r.next_bytes(&v)) {
          err = true;
          touches = false;
          break;
        }
        mem.push_back(f);
        val.push_back(v);
      }
    }
    if (err) ++st.cmd_errors;
    if (!touches) continue;
    // ---- one op row (+ its children); byte refs into raw (the arena is appended below)
    const uint64_t row = b.kh.size();
    b.kh.push_back(0);  // hashed after the arena is appended (refs may point into it)
    b.kf.push_back(0);
    b.ct.push_back(cur_uuid);
    b.ut.push_back(nodeid);
    b.dt.push_back(0);
    b.aux.push_back(msg_at);
    b.meta.push_back(meta_pack(code, 0, row));
    b.key_ref.push_back(key);
    b.val_ref.push_back(value);
    for (const NodeArg& na : nodes) {
      b.n_pkh.push_back(0);
      b.n_pkf.push_back(0);
      b.n_node.push_back(na.node);
      b.n_v.push_back((uint64_t)na.v);
      b.n_t.push_back(row);
      b.n_meta.push_back(meta_pack(0, 0, b.n_meta.size()));
    }
    for (size_t i = 0; i < mem.size(); ++i) {
      b.m_pkh.push_back(0);
      b.m_pkf.push_back(0);
      b.m_h.push_back(0);
      b.m_f.push_back(0);
      b.m_t.push_back(row);
      b.m_meta.push_back(meta_pack(KIND_ADD, 0, b.m_meta.size()));
      b.m_ref.push_back(mem[i]);
      b.m_vref.push_back(code == OP_HSET ? val[i] : ByteRef{0, 0});
    }
  }
  // decimal arena after the stream bytes; refs tagged with bit 63 point into it
  const uint64_t base = b.raw.size();
  b.raw.insert(b.raw.end(), arena.begin(), arena.end());
  auto fix = [&](ByteRef& r) {
    if (r.off >> 63) r.off = base + (r.off & ~(1ull << 63));
  };
  for (auto& r : b.key_ref) fix(r);
  for (auto& r : b.val_ref) fix(r);
  for (auto& r : b.m_ref) fix(r);
  for (auto& r : b.m_vref) fix(r);
  const uint8_t* raw = b.raw.data();
  for (uint64_t i = 0; i < b.kh.size(); ++i) {
    const Hash128 h = hash_bytes(raw + b.key_ref[i].off, b.key_ref[i].len, kDomainKey);
    b.kh[i] = h.h;
    b.kf[i] = h.f;
  }
  for (uint64_t j = 0; j < b.n_pkh.size(); ++j) {
    b.n_pkh[j] = b.kh[b.n_t[j]];
    b.n_pkf[j] = b.kf[b.n_t[j]];
  }
  for (uint64_t j = 0; j < b.m_pkh.size(); ++j) {
    b.m_pkh[j] = b.kh[b.m_t[j]];
    b.m_pkf[j] = b.kf[b.m_t[j]];
    const Hash128 h = hash_bytes(raw + b.m_ref[j].off, b.m_ref[j].len, kDomainMember);
    b.m_h[j] = h.h;
    b.m_f[j] = h.f;
  }
  b.n_data = b.kh.size();
  st.n_ops = b.kh.size();
  st.n_node_args = b.n_pkh.size();
  st.n_member_args = b.m_pkh.size();
  *err_off = truncated ? cur : 0;
  return truncated ? CDB_NEED_MORE_MSG : CDB_OK;
}

}  // namespace cdb
