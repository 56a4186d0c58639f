// GPU decode of a partial-replication stream: the same cdb_ops as decode_ops
// (ops.cpp) -- op rows, children, byte references and counters, field for field -- with the
// per-message work on the GPU. RESP framing (conn/buf_read.rs:114-210) is a sequential format:
// a message's start is known once its predecessor is parsed. It does resynchronise, though: a
// message starts on a line (after "\r\n") with '*', so
//   1. resp_cand_*    every '*' at a line start is a candidate message start (in stream order);
//   2. resp_frame     one thread per candidate parses a whole RESP value there (nested arrays
//                     followed iteratively): status and size;
//   3. host           walks the chain from byte 0 through the candidates' sizes (candidates
//                     inside bulk payloads are never reached), stopping where the host decoder
//                     would: malformed (InvalidRequestMsg) or truncated (NeedMoreMsg);
//   4. resp_classify  one thread per message: pull.rs:184-235 up to the uuid gate and the
//                     handler's argument parsing (cmd.rs:348-397), as a compact record;
//   5. host           the uuid gate (pull.rs:199-209), sequential over the records (it carries
//                     uuid_he_sent from message to message);
//   6. resp_emit      one thread per applied op: the op row, its node / member rows, key and
//                     member hashes, byte references.
// Rare shapes fall back to decode_ops for the whole stream: an argument given as a RESP
// integer whose decimal form differs from its digits (get_int_bytes needs the decimal arena),
// nesting deeper than the device parser follows, and top-level values that are not arrays are
// parsed on the host inside the chain walk.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "batch.h"
#include "engine.h"
#include "ops.h"
#include "partition.hip.h"

namespace cdb {
namespace {

constexpr int kRespThreads = 256;
constexpr uint32_t kCandBytes = 16;                         // bytes per thread (candidate search)
constexpr uint32_t kCandTile = kRespThreads * kCandBytes;   // bytes per workgroup
constexpr int kMaxDepth = 16;
enum : uint8_t { R_OK = 0, R_BAD = 1, R_SHORT = 2, R_HOST = 3 };

// ------------------------------------------------------------------ RESP on the device
// (the same functions as ops.cpp's Reader / bytes2i64 / NextArg / name_is)
__device__ bool d_until_crlf(const uint8_t* b, uint64_t n, uint64_t cur, uint64_t* at) {
  for (uint64_t i = cur; i + 1 < n; ++i)
    if (b[i] == '\r' && b[i + 1] == '\n') {
      *at = i + 1;
      return true;
    }
  return false;
}

__device__ bool d_bytes2i64(const uint8_t* p, uint64_t n, int64_t* out) {  // lib/utils.rs:3-28
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

struct DItem {
  uint8_t kind;  // '+', '-', ':', '$', 'n' (nil), '*'
  uint64_t off, len;
  int64_t ival;
};

// A value at cur that is not an array (parse_msg_inner's scalar cases).
__device__ uint8_t d_scalar(const uint8_t* b, uint64_t n, uint64_t cur, uint64_t* size, DItem* it) {
  uint64_t s;
  const uint8_t t = b[cur];
  it->ival = 0;
  switch (t) {
    case '+':
    case '-':
      if (!d_until_crlf(b, n, cur + 1, &s)) return R_SHORT;
      it->kind = t;
      it->off = cur + 1;
      it->len = s - 1 - (cur + 1);
      *size = s - cur + 1;
      return R_OK;
    case ':':
      if (!d_until_crlf(b, n, cur + 1, &s)) return R_SHORT;
      if (!d_bytes2i64(b + cur + 1, s - 1 - (cur + 1), &it->ival)) return R_BAD;
      it->kind = ':';
      it->off = cur + 1;
      it->len = s - 1 - (cur + 1);
      *size = s - cur + 1;
      return R_OK;
    case '$': {
      uint64_t he;
      if (!d_until_crlf(b, n, cur + 1, &he)) return R_SHORT;
      int64_t cnt;
      if (!d_bytes2i64(b + cur + 1, he - 1 - (cur + 1), &cnt)) return R_BAD;
      if (cnt == -1) {
        it->kind = 'n';
        it->off = it->len = 0;
        *size = 5;
        return R_OK;
      }
      if (cnt < 0) return R_BAD;
      uint64_t se;
      if (!d_until_crlf(b, n, he, &se)) return R_SHORT;
      if (se - he != (uint64_t)cnt + 2) return R_BAD;
      it->kind = '$';
      it->off = he + 1;
      it->len = (uint64_t)cnt;
      *size = se - cur + 1;
      return R_OK;
    }
    default:
      return R_BAD;
  }
}

// The whole value at cur, arrays followed with an explicit stack (same order of checks as the
// recursive host parser, so the same first error wins).
__device__ uint8_t d_value(const uint8_t* b, uint64_t n, uint64_t cur, uint64_t* size) {
  int64_t rem[kMaxDepth];
  int d = 0;
  uint64_t p = cur;
  for (;;) {
    if (p >= n) return R_SHORT;
    if (b[p] == '*') {
      uint64_t le;
      if (!d_until_crlf(b, n, p + 1, &le)) return R_SHORT;
      int64_t cnt;
      if (!d_bytes2i64(b + p + 1, le - 1 - (p + 1), &cnt)) return R_BAD;
      if (cnt < 0) return R_BAD;
      p = le + 1;
      if (cnt > 0) {
        if (d == kMaxDepth) return R_HOST;
        rem[d++] = cnt;
        continue;
      }
    } else {
      uint64_t sz;
      DItem it;
      const uint8_t r = d_scalar(b, n, p, &sz, &it);
      if (r) return r;
      p += sz;
    }
    while (d > 0) {  // a value ended: close the arrays it completes
      if (--rem[d - 1] > 0) break;
      --d;
    }
    if (d == 0) {
      *size = p - cur;
      return R_OK;
    }
  }
}

// The top-level items of a well-formed array message (NextArg's cursor).
struct Args {
  const uint8_t* b;
  uint64_t n, p;
  int64_t left;
  bool arena;  // an integer argument used as bytes whose decimal form differs from its digits
  __device__ bool next(DItem* it) {
    if (left <= 0) return false;
    uint64_t sz = 0;
    if (b[p] == '*') {
      it->kind = '*';
      (void)d_value(b, n, p, &sz);
    } else {
      (void)d_scalar(b, n, p, &sz, it);
    }
    p += sz;
    --left;
    return true;
  }
  __device__ bool next_bytes(uint64_t* off, uint64_t* len) {
    DItem x;
    if (!next(&x)) return false;
    if (x.kind == ':') {  // get_int_bytes (resp.rs:20-26): the decimal form of the value
      char d[24];
      int k = 0;
      uint64_t u = x.ival < 0 ? 0 - (uint64_t)x.ival : (uint64_t)x.ival;
      do {
        d[k++] = (char)('0' + u % 10);
        u /= 10;
      } while (u);
      const int nd = k + (x.ival < 0);
      bool same = (uint64_t)nd == x.len;
      for (int i = 0; same && i < nd; ++i) {
        const char c = (x.ival < 0 && i == 0) ? '-' : d[nd - 1 - i];
        same = b[x.off + i] == (uint8_t)c;
      }
      if (!same) arena = true;  // (the host decoder takes these streams)
      *off = x.off;
      *len = x.len;
      return true;
    }
    if (x.kind == '+' || x.kind == '-' || x.kind == '$') {
      *off = x.off;
      *len = x.len;
      return true;
    }
    return false;
  }
  __device__ bool next_i64(int64_t* v) {
    DItem x;
    if (!next(&x)) return false;
    if (x.kind == ':') {
      *v = x.ival;
      return true;
    }
    if (x.kind == '+' || x.kind == '$') return d_bytes2i64(b + x.off, x.len, v);
    return false;
  }
  __device__ bool next_u64(uint64_t* v) {
    int64_t s;
    if (!next_i64(&s) || s < 0) return false;
    *v = (uint64_t)s;
    return true;
  }
};

__device__ bool d_name_is(const uint8_t* b, uint64_t off, uint64_t len, const char* lower) {
  uint64_t n = 0;
  while (lower[n]) ++n;
  if (len != n) return false;
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t c = b[off + i];
    if (c >= 'A' && c <= 'Z') c = (uint8_t)(c - 'A' + 'a');
    if (c != (uint8_t)lower[i]) return false;
  }
  return true;
}

// cmd.rs:39-41 (the replayed subset) and the commands counted as unsupported (see ops.cpp)
__device__ uint32_t d_command(const uint8_t* b, uint64_t off, uint64_t len, bool* unsup) {
  const char* names[11] = {"set", "delbytes", "incr", "decr", "delcnt", "sadd", "srem", "delset", "hset", "hdel", "deldict"};
  const uint32_t codes[11] = {OP_SET, OP_DELBYTES, OP_INCR, OP_DECR, OP_DELCNT, OP_SADD, OP_SREM, OP_DELSET,
                              OP_HSET, OP_HDEL, OP_DELDICT};
  const char* uns[14] = {"spop", "del", "node", "replicas", "sync", "meet", "client", "repllog", "info", "get",
                         "desc", "smembers", "hget", "hgetall"};
  uint32_t code = 0;
  for (int i = 0; i < 11; ++i)
    if (d_name_is(b, off, len, names[i])) code = codes[i];
  *unsup = false;
  for (int i = 0; i < 14; ++i)
    if (d_name_is(b, off, len, uns[i])) *unsup = true;
  return code;
}

// ------------------------------------------------------------------ kernels
struct RespArgs {
  const uint8_t* b;
  uint64_t n;
  uint32_t* tile_cnt;   // candidates per tile
  uint32_t* tile_off;   // exclusive scan of tile_cnt
  uint64_t* cand;       // candidate offsets, stream order
  uint64_t n_cand;
  uint32_t* size;       // per candidate: value size (status != R_OK: 0)
  uint8_t* status;      // per candidate
  const uint32_t* chain;  // the messages, as candidate indices, in stream order
  uint64_t n_msg;
  uint8_t* cls;         // per message: class | post << 4
  uint8_t* flags;       // per message: err | touches << 1 | arena << 2
  uint64_t* last;       // per message: last_uuid (replicate) / the acked uuid (replack)
  uint64_t* curu;       // per message: current_uuid
  uint32_t* nn;         // per message: node / member arguments (if it emits)
  uint32_t* nm;
  const uint32_t* emit;   // per message: 1 if its op row is emitted (host gate)
  const uint32_t* orow;   // exclusive scans of emit, nn * emit, nm * emit
  const uint32_t* nrow;
  const uint32_t* mrow;
  uint64_t* k[7];       // op rows: kh kf ct ut dt aux meta
  ulonglong2 *kref, *vref;
  uint64_t* nd[6];
  uint64_t* mb[6];
  ulonglong2 *mref, *mvref;
};

__device__ __forceinline__ bool is_cand(const uint8_t* b, uint64_t p) {
  return b[p] == '*' && (p == 0 || b[p - 1] == '\n');
}

__global__ void __launch_bounds__(kRespThreads) resp_cand_count(RespArgs A) {
  const uint64_t t0 = (uint64_t)blockIdx.x * kCandTile + threadIdx.x * kCandBytes;
  uint32_t c = 0;
  for (uint32_t i = 0; i < kCandBytes; ++i)
    if (t0 + i < A.n) c += is_cand(A.b, t0 + i);
  __shared__ uint32_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  if (c) atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0) A.tile_cnt[blockIdx.x] = s;
}

__global__ void __launch_bounds__(kRespThreads) resp_cand_write(RespArgs A) {
  const uint64_t t0 = (uint64_t)blockIdx.x * kCandTile + threadIdx.x * kCandBytes;
  uint32_t c = 0;
  for (uint32_t i = 0; i < kCandBytes; ++i)
    if (t0 + i < A.n) c += is_cand(A.b, t0 + i);
  __shared__ uint32_t pre[kRespThreads];
  pre[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < kRespThreads; o <<= 1) {  // inclusive scan over the tile's threads
    const uint32_t v = threadIdx.x >= (unsigned)o ? pre[threadIdx.x - o] : 0;
    __syncthreads();
    pre[threadIdx.x] += v;
    __syncthreads();
  }
  uint64_t w = A.tile_off[blockIdx.x] + pre[threadIdx.x] - c;
  for (uint32_t i = 0; i < kCandBytes; ++i)
    if (t0 + i < A.n && is_cand(A.b, t0 + i)) A.cand[w++] = t0 + i;
}

__global__ void __launch_bounds__(kRespThreads) resp_frame(RespArgs A) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n_cand; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t sz = 0;
    const uint8_t r = d_value(A.b, A.n, A.cand[i], &sz);
    A.status[i] = (r == R_OK && sz >= (1ull << 32)) ? R_HOST : r;
    A.size[i] = r == R_OK ? (uint32_t)sz : 0;
  }
}

// classes of a message (the host gate reads them)
enum : uint8_t { C_LOST = 0, C_REPLACK = 1, C_REPLICATE = 2 };
enum : uint8_t { P_LOST = 0, P_UNKNOWN = 1, P_UNSUPPORTED = 2, P_APPLIED = 3 };

struct Semantic {  // one message through pull.rs:184-235 up to the handler's first DB touch
  uint8_t cls, post;
  bool err, touches;
  uint64_t last, cur, nodeid, acked;
  uint32_t code, nn, nm;
  uint64_t koff, klen, voff, vlen;
};

// Parses the message at p (a well-formed array); with EMIT, also writes its rows.
template <bool EMIT>
__device__ void d_message(const RespArgs& A, uint64_t p, Semantic& S, bool* arena, uint64_t msg_row, uint64_t n0,
                          uint64_t m0, uint64_t kh, uint64_t kf) {
  S.cls = C_LOST;
  S.post = P_LOST;
  S.err = false;
  S.touches = false;
  S.last = S.cur = S.nodeid = S.acked = 0;
  S.code = S.nn = S.nm = 0;
  S.koff = S.klen = S.voff = S.vlen = 0;
  Args a;
  a.b = A.b;
  a.n = A.n;
  a.arena = false;
  {
    uint64_t le = 0;
    (void)d_until_crlf(A.b, A.n, p + 1, &le);
    int64_t cnt = 0;
    (void)d_bytes2i64(A.b + p + 1, le - 1 - (p + 1), &cnt);
    a.left = cnt;
    a.p = le + 1;
  }
  uint64_t noff, nlen;
  if (!a.next_bytes(&noff, &nlen)) return;  // lost
  if (d_name_is(A.b, noff, nlen, "replack")) {
    uint64_t acked;
    if (a.next_u64(&acked)) {
      S.cls = C_REPLACK;
      S.acked = acked;
    }
    return;
  }
  if (!d_name_is(A.b, noff, nlen, "replicate")) return;
  if (!a.next_u64(&S.nodeid) || !a.next_u64(&S.last)) return;
  S.cls = C_REPLICATE;
  uint64_t coff, clen;
  if (!a.next_u64(&S.cur) || !a.next_bytes(&coff, &clen)) return;  // lost after the gate
  bool unsup = false;
  // a command name given as an integer matches nothing (its ref is in the arena on the host)
  const uint32_t code = d_command(A.b, coff, clen, &unsup);
  if (!code) {
    S.post = unsup ? P_UNSUPPORTED : P_UNKNOWN;
    return;
  }
  S.post = P_APPLIED;
  S.code = code;
  a.arena = false;  // only the handler's arguments can need the decimal arena
  // ---- the handler's argument parsing (ops.cpp, cmd.rs / type_*.rs)
  bool touches = true;
  if (!a.next_bytes(&S.koff, &S.klen)) {
    S.err = true;
    touches = false;
  } else if (code == OP_SET) {
    if (!a.next_bytes(&S.voff, &S.vlen)) S.err = true, touches = false;
  } else if (code == OP_INCR || code == OP_DECR) {
    if (EMIT) {
      A.nd[0][n0] = kh;
      A.nd[1][n0] = kf;
      A.nd[2][n0] = S.nodeid;
      A.nd[3][n0] = (uint64_t)(int64_t)(code == OP_INCR ? 1 : -1);
      A.nd[4][n0] = msg_row;
      A.nd[5][n0] = meta_pack(0, 0, n0);
    }
    S.nn = 1;
  } else if (code == OP_DELCNT) {
    uint64_t nd_;
    while (a.next_u64(&nd_)) {
      int64_t v;
      if (!a.next_i64(&v)) {
        S.err = true;
        break;
      }
      if (EMIT) {
        const uint64_t r = n0 + S.nn;
        A.nd[0][r] = kh;
        A.nd[1][r] = kf;
        A.nd[2][r] = nd_;
        A.nd[3][r] = (uint64_t)v;
        A.nd[4][r] = msg_row;
        A.nd[5][r] = meta_pack(0, 0, r);
      }
      ++S.nn;
    }
  } else if (code == OP_SADD || code == OP_SREM || code == OP_HDEL || code == OP_HSET) {
    uint64_t mo, ml;
    while (a.next_bytes(&mo, &ml)) {
      uint64_t vo = 0, vl = 0;
      if (code == OP_HSET && !a.next_bytes(&vo, &vl)) {  // an odd count errors before the DB
        S.err = true;
        touches = false;
        break;
      }
      if (EMIT) {
        const uint64_t r = m0 + S.nm;
        const Hash128 mh = hash_bytes(A.b + mo, ml, kDomainMember);
        A.mb[0][r] = kh;
        A.mb[1][r] = kf;
        A.mb[2][r] = mh.h;
        A.mb[3][r] = mh.f;
        A.mb[4][r] = msg_row;
        A.mb[5][r] = meta_pack(KIND_ADD, 0, r);
        A.mref[r] = make_ulonglong2(mo, ml);
        A.mvref[r] = make_ulonglong2(vo, vl);
      }
      ++S.nm;
    }
  }
  S.touches = touches;
  *arena = a.arena;
}

__global__ void __launch_bounds__(kRespThreads) resp_classify(RespArgs A) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n_msg; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t ci = A.chain[i];
    if (ci == 0xFFFFFFFFu) {  // a top-level value that is not an array (parsed on the host): lost
      A.cls[i] = C_LOST;
      A.flags[i] = 0;
      A.last[i] = A.curu[i] = 0;
      A.nn[i] = A.nm[i] = 0;
      continue;
    }
    Semantic S;
    bool arena = false;
    d_message<false>(A, A.cand[ci], S, &arena, 0, 0, 0, 0, 0);
    A.cls[i] = (uint8_t)(S.cls | (S.post << 4));
    A.flags[i] = (uint8_t)((S.err ? 1 : 0) | (S.touches ? 2 : 0) | (arena ? 4 : 0));
    A.last[i] = S.cls == C_REPLACK ? S.acked : S.last;
    A.curu[i] = S.cur;
    A.nn[i] = S.nn;
    A.nm[i] = S.nm;
  }
}

__global__ void __launch_bounds__(kRespThreads) resp_mask(RespArgs A) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n_msg; i += (uint64_t)gridDim.x * blockDim.x)
    if (!A.emit[i]) A.nn[i] = A.nm[i] = 0;
}

__global__ void __launch_bounds__(kRespThreads) resp_emit(RespArgs A) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n_msg; i += (uint64_t)gridDim.x * blockDim.x) {
    if (!A.emit[i]) continue;
    const uint64_t p = A.cand[A.chain[i]];
    const uint64_t r = A.orow[i];
    // the key first (its hash parents the children), then the whole message with rows
    Semantic S;
    bool arena = false;
    d_message<false>(A, p, S, &arena, 0, 0, 0, 0, 0);
    const Hash128 h = hash_bytes(A.b + S.koff, S.klen, kDomainKey);
    d_message<true>(A, p, S, &arena, r, A.nrow[i], A.mrow[i], h.h, h.f);
    A.k[0][r] = h.h;
    A.k[1][r] = h.f;
    A.k[2][r] = S.cur;
    A.k[3][r] = S.nodeid;
    A.k[4][r] = 0;
    A.k[5][r] = p;
    A.k[6][r] = meta_pack(S.code, 0, r);
    A.kref[r] = make_ulonglong2(S.koff, S.klen);
    A.vref[r] = make_ulonglong2(S.voff, S.vlen);
  }
}

template <typename T>
struct DevArr {
  T* p = nullptr;
  ~DevArr() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

// 0: done (*out filled, status in *rc); 1: the stream needs the host decoder; < 0: a HIP call
// failed (-status, ctx->last_error says which): reported to the caller, never a silent fallback.
int decode_ops_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t uuid_he_sent, Batch* out,
                   cdb_ops_info* info, size_t* err_off, int* rc_out, double* host_ms, double* device_ms) {
  using clk = std::chrono::steady_clock;
  double th = 0;
  const auto t_all = clk::now();
  Batch& b = *out;
  cdb_ops_info& st = *info;
  std::memset(&st, 0, sizeof st);
  st.uuid_he_sent = uuid_he_sent;
  *err_off = 0;
  *rc_out = CDB_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return -(int)fail(ctx, CDB_DEVICE_ERROR, "hipSetDevice");
  hipStream_t s = ctx->stream;
  cdb_status cs = CDB_OK;
  auto ck = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && cs == CDB_OK) cs = hip_check(ctx, e, what);
  };
  if (len == 0) {
    adopt_raw(&b, buf, 0);
    return 0;
  }
  // ---- the stream to the device, candidates in stream order
  const uint64_t tiles = (len + kCandTile - 1) / kCandTile;
  DevArr<uint8_t> d_raw;
  DevArr<uint32_t> d_tiles;
  ck(hipMalloc(&d_raw.p, len + 16), "hipMalloc(resp)");
  ck(hipMalloc(&d_tiles.p, (2 * tiles + 2) * sizeof(uint32_t) + (2 * ((tiles + kScanTile - 1) / kScanTile) + 8) * 8),
     "hipMalloc(resp)");
  if (cs != CDB_OK) return -(int)cs;
  RespArgs A;
  std::memset(&A, 0, sizeof A);
  A.b = d_raw.p;
  A.n = len;
  A.tile_cnt = d_tiles.p;
  A.tile_off = d_tiles.p + tiles + 1;
  uint64_t* d_sums = (uint64_t*)(((uintptr_t)(A.tile_off + tiles + 1) + 15) & ~(uintptr_t)15);
  uint64_t* d_tot = d_sums + ((tiles + kScanTile - 1) / kScanTile) + 2;
  ck(hipMemsetAsync(d_raw.p + len, 0, 16, s), "memset(resp)");
  if (cs == CDB_OK) cs = staged_h2d(ctx, d_raw.p, buf, len, s);
  const auto t0 = clk::now();
  adopt_raw(&b, buf, len);  // (the batch's arena; overlaps the upload's tail)
  th += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  if (cs != CDB_OK) return -(int)cs;
  resp_cand_count<<<(uint32_t)tiles, kRespThreads, 0, s>>>(A);
  const uint64_t stiles = (tiles + kScanTile - 1) / kScanTile;
  scan_reduce_kernel<uint32_t><<<(uint32_t)stiles, kScanThreads, 0, s>>>(A.tile_cnt, tiles, d_sums);
  scan_sums_kernel<<<1, kScanThreads, 0, s>>>(d_sums, stiles, d_tot);
  scan_apply_kernel<uint32_t, uint32_t><<<(uint32_t)stiles, kScanThreads, 0, s>>>(A.tile_cnt, tiles, d_sums, A.tile_off,
                                                                               (uint32_t*)nullptr);
  uint64_t nc = 0;
  ck(hipMemcpyAsync(&nc, d_tot, 8, hipMemcpyDeviceToHost, s), "d2h(resp)");
  ck(hipStreamSynchronize(s), "sync(resp)");
  if (cs != CDB_OK) return -(int)cs;
  if (nc >= (1ull << 32) - 1) return 1;
  A.n_cand = nc;
  DevArr<uint8_t> d_cand;  // cand u64 | size u32 | status u8
  ck(hipMalloc(&d_cand.p, nc * 13 + 64), "hipMalloc(resp)");
  if (cs != CDB_OK) return -(int)cs;
  A.cand = (uint64_t*)d_cand.p;
  A.size = (uint32_t*)(A.cand + nc);
  A.status = (uint8_t*)(A.size + nc);
  if (nc) {
    resp_cand_write<<<(uint32_t)tiles, kRespThreads, 0, s>>>(A);
    resp_frame<<<(uint32_t)std::min<uint64_t>((nc + kRespThreads - 1) / kRespThreads, 16384), kRespThreads, 0, s>>>(A);
    ck(hipGetLastError(), "resp kernels");
  }
  std::vector<uint64_t> h_cand(nc);
  std::vector<uint32_t> h_size(nc);
  std::vector<uint8_t> h_status(nc);
  if (cs == CDB_OK && nc) cs = staged_d2h(ctx, h_cand.data(), A.cand, nc * 8, s);
  if (cs == CDB_OK && nc) cs = staged_d2h(ctx, h_size.data(), A.size, nc * 4, s);
  if (cs == CDB_OK && nc) cs = staged_d2h(ctx, h_status.data(), A.status, nc, s);
  if (cs != CDB_OK) return -(int)cs;
  // ---- the chain of messages from byte 0 (host): where the host decoder would stop, we stop
  const auto t1 = clk::now();
  std::vector<uint32_t> chain;
  std::vector<uint64_t> at;  // each message's offset (for the non-array ones; '*' ones: cand)
  chain.reserve(nc);
  uint64_t cur = 0, ci = 0;
  bool truncated = false;
  while (cur < len) {
    if (buf[cur] == '*') {
      while (ci < nc && h_cand[ci] < cur) ++ci;
      if (ci >= nc || h_cand[ci] != cur) return 1;  // (cannot happen: every '*' at a line start is one)
      const uint8_t r = h_status[ci];
      if (r == R_HOST) return 1;
      if (r == R_BAD) {
        *err_off = cur;
        *rc_out = CDB_INVALID_REQUEST_MSG;
        return 0;
      }
      if (r == R_SHORT) {
        truncated = true;
        break;
      }
      chain.push_back((uint32_t)ci);
      cur += h_size[ci];
    } else {
      // a top-level value that is not an array: the host decoder's reader decides (it is lost)
      return 1;
    }
  }
  th += std::chrono::duration<double, std::milli>(clk::now() - t1).count();
  const uint64_t nmsg = chain.size();
  st.n_messages = nmsg;
  // ---- per-message records
  A.n_msg = nmsg;
  DevArr<uint8_t> d_msg;  // chain u32 | cls u8 | flags u8 | last u64 | cur u64 | nn u32 | nm u32 | emit u32 | orow nrow mrow u32
  const size_t msg_bytes = nmsg * (4 + 1 + 1 + 8 + 8 + 4 + 4 + 4 + 12) + 256;
  ck(hipMalloc(&d_msg.p, msg_bytes), "hipMalloc(resp)");
  if (cs != CDB_OK) return -(int)cs;
  {
    uint8_t* w = d_msg.p;
    auto take = [&](size_t bytes) {
      uint8_t* r = w;
      w += (bytes + 15) & ~size_t(15);
      return r;
    };
    A.last = (uint64_t*)take(nmsg * 8);
    A.curu = (uint64_t*)take(nmsg * 8);
    A.chain = (const uint32_t*)take(nmsg * 4);
    A.nn = (uint32_t*)take(nmsg * 4);
    A.nm = (uint32_t*)take(nmsg * 4);
    A.emit = (const uint32_t*)take(nmsg * 4);
    A.orow = (const uint32_t*)take(nmsg * 4);
    A.nrow = (const uint32_t*)take(nmsg * 4);
    A.mrow = (const uint32_t*)take(nmsg * 4);
    A.cls = take(nmsg);
    A.flags = take(nmsg);
  }
  if (nmsg && cs == CDB_OK) cs = staged_h2d(ctx, (void*)A.chain, chain.data(), nmsg * 4, s);
  if (cs != CDB_OK) return -(int)cs;
  const uint32_t mgrid = (uint32_t)std::min<uint64_t>((nmsg + kRespThreads - 1) / kRespThreads, 16384);
  if (nmsg) {
    resp_classify<<<mgrid, kRespThreads, 0, s>>>(A);
    ck(hipGetLastError(), "resp_classify");
  }
  std::vector<uint8_t> h_cls(nmsg), h_flags(nmsg);
  std::vector<uint64_t> h_last(nmsg), h_cur(nmsg);
  if (nmsg) {
    if (cs == CDB_OK) cs = staged_d2h(ctx, h_cls.data(), A.cls, nmsg, s);
    if (cs == CDB_OK) cs = staged_d2h(ctx, h_flags.data(), A.flags, nmsg, s);
    if (cs == CDB_OK) cs = staged_d2h(ctx, h_last.data(), A.last, nmsg * 8, s);
    if (cs == CDB_OK) cs = staged_d2h(ctx, h_cur.data(), A.curu, nmsg * 8, s);
  }
  if (cs != CDB_OK) return -(int)cs;
  // ---- the uuid gate (pull.rs:199-209), message by message
  const auto t2 = clk::now();
  std::vector<uint32_t> emit(nmsg, 0);
  uint64_t n_emit = 0;
  for (uint64_t i = 0; i < nmsg; ++i) {
    const uint8_t c = h_cls[i] & 15, post = h_cls[i] >> 4, f = h_flags[i];
    if (c == C_LOST) {
      ++st.lost;
    } else if (c == C_REPLACK) {  // pull.rs:226-228
      st.uuid_he_acked = h_last[i];
      ++st.replacks;
    } else if (st.uuid_he_sent < h_last[i]) {  // ReplicateCommandsLost (pull.rs:201-204)
      ++st.lost;
    } else if (st.uuid_he_sent > h_last[i]) {  // duplicated commands (pull.rs:205-206)
      ++st.duplicates;
    } else if (post == P_LOST) {
      ++st.lost;
    } else {
      st.uuid_he_sent = h_cur[i];  // advanced for every command that reaches Cmd::new (pull.rs:214-223)
      if (post == P_UNKNOWN) ++st.unknown;
      else if (post == P_UNSUPPORTED) ++st.unsupported;
      else {
        ++st.applied;
        if (f & 1) ++st.cmd_errors;
        if (f & 2) {
          if (f & 4) return 1;  // an argument needs the decimal arena: the host decoder's
          emit[i] = 1;
          ++n_emit;
        }
      }
    }
  }
  th += std::chrono::duration<double, std::milli>(clk::now() - t2).count();
  // ---- op rows: scans of the emitted messages' row counts, then the emit pass
  if (nmsg && cs == CDB_OK) cs = staged_h2d(ctx, (void*)A.emit, emit.data(), nmsg * 4, s);
  if (cs != CDB_OK) return -(int)cs;
  uint64_t tot[3] = {0, 0, 0};
  {
    DevArr<uint64_t> d_s;
    const uint64_t mt = (nmsg + kScanTile - 1) / kScanTile;
    ck(hipMalloc(&d_s.p, (3 * (mt + 1) + 8) * 8), "hipMalloc(resp)");
    if (cs != CDB_OK) return -(int)cs;
    ck(hipMemsetAsync(d_s.p + 3 * (mt + 1), 0, 64, s), "memset(resp)");
    uint64_t* dt = d_s.p + 3 * (mt + 1);
    if (nmsg) {  // nn / nm count only for emitted messages: masked in place
      resp_mask<<<mgrid, kRespThreads, 0, s>>>(A);
      ck(hipGetLastError(), "resp_mask");
    }
    const uint32_t* ins[3] = {A.emit, A.nn, A.nm};
    const uint32_t* outs[3] = {A.orow, A.nrow, A.mrow};
    for (int f = 0; f < 3 && nmsg; ++f) {
      scan_reduce_kernel<uint32_t><<<(uint32_t)std::max<uint64_t>(mt, 1), kScanThreads, 0, s>>>(ins[f], nmsg, d_s.p + f * (mt + 1));
      scan_sums_kernel<<<1, kScanThreads, 0, s>>>(d_s.p + f * (mt + 1), mt, dt + f);
      scan_apply_kernel<uint32_t, uint32_t><<<(uint32_t)std::max<uint64_t>(mt, 1), kScanThreads, 0, s>>>(
          ins[f], nmsg, d_s.p + f * (mt + 1), const_cast<uint32_t*>(outs[f]), (uint32_t*)nullptr);
    }
    ck(hipGetLastError(), "resp scans");
    if (nmsg) ck(hipMemcpyAsync(tot, dt, 24, hipMemcpyDeviceToHost, s), "d2h(resp)");
    ck(hipStreamSynchronize(s), "sync(resp)");
    if (cs != CDB_OK) return -(int)cs;
  }
  const uint64_t no = tot[0], nn = tot[1], nm = tot[2];
  if (no != n_emit) return 1;
  DevArr<uint64_t> d_rows;
  const size_t words = no * 11 + nn * 6 + nm * 10 + 16;
  ck(hipMalloc(&d_rows.p, words * 8), "hipMalloc(resp rows)");
  if (cs != CDB_OK) return -(int)cs;
  {
    uint64_t* w = d_rows.p;
    uint64_t* const w0 = w;
    auto align16 = [&]() { w += (w - w0) & 1; };
    for (int c = 0; c < 7; ++c, w += no) A.k[c] = w;
    align16();
    A.kref = (ulonglong2*)w; w += 2 * no;
    A.vref = (ulonglong2*)w; w += 2 * no;
    for (int c = 0; c < 6; ++c, w += nn) A.nd[c] = w;
    for (int c = 0; c < 6; ++c, w += nm) A.mb[c] = w;
    align16();
    A.mref = (ulonglong2*)w; w += 2 * nm;
    A.mvref = (ulonglong2*)w; w += 2 * nm;
  }
  if (no) {
    resp_emit<<<mgrid, kRespThreads, 0, s>>>(A);
    ck(hipGetLastError(), "resp_emit");
  }
  // ---- rows into the batch
  std::vector<HostSeg> segs;
  auto down = [&](void* host, const void* dev, uint64_t bytes) {
    if (bytes) segs.push_back({host, const_cast<void*>(dev), bytes});
  };
  ColVec* kc[7] = {&b.kh, &b.kf, &b.ct, &b.ut, &b.dt, &b.aux, &b.meta};
  for (int c = 0; c < 7; ++c) {
    kc[c]->resize(no);
    down(kc[c]->data(), A.k[c], no * 8);
  }
  b.key_ref.resize(no);
  b.val_ref.resize(no);
  down(b.key_ref.data(), A.kref, no * 16);
  down(b.val_ref.data(), A.vref, no * 16);
  ColVec* ncv[6] = {&b.n_pkh, &b.n_pkf, &b.n_node, &b.n_v, &b.n_t, &b.n_meta};
  ColVec* mcv[6] = {&b.m_pkh, &b.m_pkf, &b.m_h, &b.m_f, &b.m_t, &b.m_meta};
  for (int c = 0; c < 6; ++c) {
    ncv[c]->resize(nn);
    down(ncv[c]->data(), A.nd[c], nn * 8);
    mcv[c]->resize(nm);
    down(mcv[c]->data(), A.mb[c], nm * 8);
  }
  b.m_ref.resize(nm);
  b.m_vref.resize(nm);
  down(b.m_ref.data(), A.mref, nm * 16);
  down(b.m_vref.data(), A.mvref, nm * 16);
  if (!segs.empty()) cs = staged_copy(ctx, segs.data(), segs.size(), false, s);
  ck(hipStreamSynchronize(s), "sync(resp)");
  if (cs != CDB_OK) return -(int)cs;
  b.n_data = no;
  st.n_ops = no;
  st.n_node_args = nn;
  st.n_member_args = nm;
  if (truncated) {
    *err_off = cur;
    *rc_out = CDB_NEED_MORE_MSG;
  }
  if (host_ms) *host_ms = th;
  if (device_ms) *device_ms = std::chrono::duration<double, std::milli>(clk::now() - t_all).count() - th;
  return 0;
}

}  // namespace cdb
