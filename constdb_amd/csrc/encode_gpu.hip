// GPU snapshot encode: a merge result -> the reference's wire format, with
// the CRC-64/Jones checksum, on the GPU.
//
// Reference writer: Server::dump_all (server.rs:183-215) -> DB::dump (db.rs:122-136) ->
// SnapshotWriter::write_entry (snapshot.rs:48-52) -> Object::save_snapshot (object.rs:85-108),
// Counter::save_snapshot (type_counter.rs:101-109), Dict/Set::save_snapshot
// (crdt/lwwhash.rs:189-205 / 325-339); ReplicaManager::dump_snapshot (replica/replica.rs:100-119);
// write_integer (snapshot.rs:25-37); the running Crc64 (snapshot.rs:39-46,62-64).
//
// The reference writes one entry after another through a buffered writer. Here every entry's
// encoded size is known from its row alone, so the stream is laid out by prefix scans and
// written in parallel:
//   1. parent scans: mark_heads_kernel writes key index + 1 at the first child row of every
//      key; a "last non-zero" scan gives each node / member row its key;
//   2. member scan: per member (add bytes, del bytes, add count) -> exclusive prefixes; a
//      key's add map, del map and add count are differences of prefixes at its child range;
//      node scan: per node bytes -> prefixes;
//   3. key scan: per key row its whole entry size (head + children), split by section
//      (DATAS / EXPIRES / DELETES) -> each row's offset inside its section, section totals;
//   4. host: section headers (flags + counts), node header and replica entries;
//   5. emit kernels: key heads, then nodes and members at their computed offsets;
//   6. CRC: each thread a 1 KB chunk (slice-by-8 tables in LDS), combined per 256-chunk tile
//      and then across tiles by GF(2) multiplication with x^(8·len) mod P. The stream is
//      preceded by zero bytes up to a whole number of tiles: with init 0 and no xorout,
//      leading zeros leave the CRC unchanged, so every combination step has a fixed length.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "batch.h"
#include "engine.h"

namespace cdb {
namespace {

// ------------------------------------------------------------------ write_integer (snapshot.rs:25-37)
// Signed comparisons as in the reference: a negative value takes the 1-byte branch and is
// truncated to its low byte (`[i as u8]`).
CDB_HD uint32_t vi_len(int64_t i) { return i < (1 << 6) ? 1u : i < (1 << 14) ? 2u : i < (1 << 30) ? 4u : 9u; }
CDB_HD uint32_t vi_put(uint8_t* o, int64_t i) {
  if (i < (1 << 6)) {
    o[0] = (uint8_t)i;
    return 1;
  }
  if (i < (1 << 14)) {
    const uint32_t v = ((uint32_t)i & 0xFFFF) | (1u << 14);
    o[0] = (uint8_t)(v >> 8);
    o[1] = (uint8_t)v;
    return 2;
  }
  if (i < (1 << 30)) {
    const uint32_t v = (uint32_t)i | (1u << 31);
    o[0] = (uint8_t)(v >> 24);
    o[1] = (uint8_t)(v >> 16);
    o[2] = (uint8_t)(v >> 8);
    o[3] = (uint8_t)v;
    return 4;
  }
  o[0] = 3 << 6;
  for (int k = 0; k < 8; ++k) o[1 + k] = (uint8_t)((uint64_t)i >> (56 - 8 * k));
  return 9;
}

// ------------------------------------------------------------------ CRC-64/Jones, reflected
constexpr uint64_t kPolyR = 0x95AC9329AC4BC9B5ull;
constexpr uint32_t kCrcChunk = 1024;                 // bytes per thread
constexpr uint32_t kCrcThreads = 256;                // chunks per tile
constexpr uint64_t kCrcTile = (uint64_t)kCrcChunk * kCrcThreads;

// a * b mod P over GF(2), reflected bit order (x^0 is the top bit).
CDB_HD uint64_t gf2_mulmod(uint64_t a, uint64_t b) {
  uint64_t m = 1ull << 63, p = 0;
  while (m) {
    if (a & m) p ^= b;
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kPolyR : b >> 1;
  }
  return p;
}
// x^(8·n) mod P: the operator that appends n zero bytes to a CRC (square and multiply).
uint64_t x8n_mod(uint64_t n) {
  uint64_t r = 1ull << 63, sq = 1ull << 62;  // x^0, x^1
  for (int i = 0; i < 3; ++i) sq = gf2_mulmod(sq, sq);  // x^8
  while (n) {
    if (n & 1) r = gf2_mulmod(r, sq);
    sq = gf2_mulmod(sq, sq);
    n >>= 1;
  }
  return r;
}
void crc_tables(uint64_t* t) {  // slice-by-8 tables, t[k*256 + b]
  for (int i = 0; i < 256; ++i) {
    uint64_t c = (uint64_t)i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPolyR : c >> 1;
    t[i] = c;
  }
  for (int k = 1; k < 8; ++k)
    for (int i = 0; i < 256; ++i) t[k * 256 + i] = (t[(k - 1) * 256 + i] >> 8) ^ t[t[(k - 1) * 256 + i] & 0xFF];
}

struct CrcConsts {
  uint64_t chunk_lvl[8];  // x^(8·kCrcChunk·2^k): the tile tree
  uint64_t tile;          // x^(8·kCrcTile): a tile run, sequentially
  uint64_t run_lvl[8];    // x^(8·kCrcTile·R·2^k): the tree over runs of R tiles
};

// One tile of 256 KB per workgroup; buf is tile-aligned (zero prefix).
__global__ void __launch_bounds__(kCrcThreads) crc_tile_kernel(const uint8_t* buf, const uint64_t* tables, CrcConsts K,
                                                               uint64_t* tile_crc) {
  __shared__ uint64_t T[8 * 256];
  __shared__ uint64_t part[kCrcThreads];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < 8 * 256; i += kCrcThreads) T[i] = tables[i];
  __syncthreads();
  const uint4* p = (const uint4*)(buf + blockIdx.x * kCrcTile + (uint64_t)t * kCrcChunk);
  uint64_t crc = 0;
#pragma unroll 4
  for (uint32_t w = 0; w < kCrcChunk / 16; ++w) {
    const uint4 q = p[w];
    const uint64_t w0 = (uint64_t)q.x | ((uint64_t)q.y << 32), w1 = (uint64_t)q.z | ((uint64_t)q.w << 32);
    uint64_t c = crc ^ w0;
    c = T[7 * 256 + (c & 0xFF)] ^ T[6 * 256 + ((c >> 8) & 0xFF)] ^ T[5 * 256 + ((c >> 16) & 0xFF)] ^
        T[4 * 256 + ((c >> 24) & 0xFF)] ^ T[3 * 256 + ((c >> 32) & 0xFF)] ^ T[2 * 256 + ((c >> 40) & 0xFF)] ^
        T[1 * 256 + ((c >> 48) & 0xFF)] ^ T[(c >> 56)];
    c ^= w1;
    crc = T[7 * 256 + (c & 0xFF)] ^ T[6 * 256 + ((c >> 8) & 0xFF)] ^ T[5 * 256 + ((c >> 16) & 0xFF)] ^
          T[4 * 256 + ((c >> 24) & 0xFF)] ^ T[3 * 256 + ((c >> 32) & 0xFF)] ^ T[2 * 256 + ((c >> 40) & 0xFF)] ^
          T[1 * 256 + ((c >> 48) & 0xFF)] ^ T[(c >> 56)];
  }
  part[t] = crc;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t s = 1u << k;
    if ((t & (2 * s - 1)) == 0) part[t] = gf2_mulmod(part[t], K.chunk_lvl[k]) ^ part[t + s];
    __syncthreads();
  }
  if (t == 0) tile_crc[blockIdx.x] = part[0];
}

// Combines the tile CRCs: thread t folds the virtual tiles [t·R, (t+1)·R) (the first pad_tiles
// are zero), then a tree over the 256 runs. Writes the CRC and its 8 LE bytes at `dst`.
__global__ void __launch_bounds__(kCrcThreads) crc_final_kernel(const uint64_t* tile_crc, uint64_t tiles,
                                                                uint64_t run, uint64_t pad_tiles, CrcConsts K,
                                                                uint64_t* crc_out, uint8_t* dst) {
  __shared__ uint64_t part[kCrcThreads];
  const uint32_t t = threadIdx.x;
  uint64_t crc = 0;
  for (uint64_t u = (uint64_t)t * run; u < (uint64_t)(t + 1) * run; ++u) {
    const uint64_t v = u >= pad_tiles ? tile_crc[u - pad_tiles] : 0;
    crc = gf2_mulmod(crc, K.tile) ^ v;
  }
  part[t] = crc;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t s = 1u << k;
    if ((t & (2 * s - 1)) == 0) part[t] = gf2_mulmod(part[t], K.run_lvl[k]) ^ part[t + s];
    __syncthreads();
  }
  if (t == 0) {
    const uint64_t c = part[0];
    *crc_out = c;
    if (dst)
      for (int k = 0; k < 8; ++k) dst[k] = (uint8_t)(c >> (8 * k));  // to_le_bytes (server.rs:206)
  }
  (void)tiles;
}

// ------------------------------------------------------------------ generic tile scan
constexpr int kST = 256, kSI = 8;
constexpr uint64_t kSTile = (uint64_t)kST * kSI;

template <class Tr>
__device__ typename Tr::V block_exclusive(typename Tr::V own, typename Tr::V* lds, typename Tr::V* total) {
  using V = typename Tr::V;
  const uint32_t t = threadIdx.x;
  lds[t] = own;
  __syncthreads();
  for (uint32_t off = 1; off < kST; off <<= 1) {
    V x = t >= off ? Tr::op(lds[t - off], lds[t]) : lds[t];
    __syncthreads();
    lds[t] = x;
    __syncthreads();
  }
  *total = lds[kST - 1];
  V ex = t ? lds[t - 1] : Tr::id();
  __syncthreads();
  return ex;
}

template <class Tr>
__global__ void __launch_bounds__(kST) tscan_reduce(Tr tr, uint64_t n, typename Tr::V* sums) {
  using V = typename Tr::V;
  __shared__ V lds[kST];
  const uint64_t base = blockIdx.x * kSTile + (uint64_t)threadIdx.x * kSI;
  V acc = Tr::id();
  for (int k = 0; k < kSI; ++k)
    if (base + k < n) acc = Tr::op(acc, tr.load(base + k));
  V tot;
  block_exclusive<Tr>(acc, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <class Tr>
__global__ void __launch_bounds__(kST) tscan_sums(Tr tr, uint64_t tiles, typename Tr::V* sums, uint64_t n) {
  using V = typename Tr::V;
  __shared__ V lds[kST];
  V carry = Tr::id();
  for (uint64_t c = 0; c < tiles; c += kST) {
    const uint64_t i = c + threadIdx.x;
    const V own = i < tiles ? sums[i] : Tr::id();
    V tot;
    const V ex = block_exclusive<Tr>(own, lds, &tot);
    if (i < tiles) sums[i] = Tr::op(carry, ex);
    carry = Tr::op(carry, tot);
  }
  if (threadIdx.x == 0) tr.store(n, carry, Tr::id());  // the grand total at index n
}

template <class Tr>
__global__ void __launch_bounds__(kST) tscan_apply(Tr tr, uint64_t n, const typename Tr::V* sums) {
  using V = typename Tr::V;
  __shared__ V lds[kST];
  const uint64_t base = blockIdx.x * kSTile + (uint64_t)threadIdx.x * kSI;
  V v[kSI];
  V acc = Tr::id();
#pragma unroll
  for (int k = 0; k < kSI; ++k) {
    v[k] = base + k < n ? tr.load(base + k) : Tr::id();
    acc = Tr::op(acc, v[k]);
  }
  V tot;
  V run = Tr::op(sums[blockIdx.x], block_exclusive<Tr>(acc, lds, &tot));
#pragma unroll
  for (int k = 0; k < kSI; ++k) {
    if (base + k < n) tr.store(base + k, run, v[k]);
    run = Tr::op(run, v[k]);
  }
}

// ------------------------------------------------------------------ encode inputs in HBM
struct EncPos {  // per fold position: its snapshot bytes and byte-reference tables (device pointers)
  const uint8_t* raw;
  const ByteRef *kref, *vref, *mref, *mvref;  // key/value refs by key src; member/value refs by member src
};
struct EncIn {
  // result rows (cdb_merged): key out meta ct ut dt win cref; node out node v t; member out t meta
  const uint64_t *kmeta, *kct, *kut, *kdt, *kwin, *kcref;
  const uint64_t *nnode, *nv, *nt;
  const uint64_t *mt, *mmeta;
  uint64_t nk, nn, nm;
  const EncPos* pos;
};

__device__ __forceinline__ ByteRef key_span(const EncIn& E, uint64_t meta, const uint8_t** p) {
  const EncPos& b = E.pos[meta_pos(meta)];
  const ByteRef r = b.kref[meta_src(meta)];
  *p = b.raw + r.off;
  return r;
}
__device__ __forceinline__ ByteRef val_span(const EncIn& E, uint64_t win, const uint8_t** p) {
  const EncPos& b = E.pos[meta_pos(win)];
  const ByteRef r = b.vref[meta_src(win)];
  *p = b.raw + r.off;
  return r;
}
__device__ __forceinline__ ByteRef mem_span(const EncIn& E, uint64_t meta, const uint8_t** p) {
  const EncPos& b = E.pos[meta_pos(meta)];
  const ByteRef r = b.mref[meta_src(meta)];
  *p = b.raw + r.off;
  return r;
}
__device__ __forceinline__ ByteRef mval_span(const EncIn& E, uint64_t meta, const uint8_t** p) {
  const EncPos& b = E.pos[meta_pos(meta)];
  const ByteRef r = b.mvref[meta_src(meta)];
  *p = b.raw + r.off;
  return r;
}

// host-tier member refs of a device-decoded batch, written into its HBM tables (refs_ready's
// patch step, on the device)
struct RefPatch { uint64_t row; ByteRef m, mv; };
__global__ void patch_refs_kernel(const RefPatch* pt, uint64_t n, ByteRef* mref, ByteRef* mvref) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const RefPatch q = pt[i];
  mref[q.row] = q.m;
  mvref[q.row] = q.mv;
}

// 1. first child row of each key -> key index + 1 (counter keys into nhead, set/dict into mhead)
__global__ void mark_heads_kernel(EncIn E, uint32_t* nhead, uint32_t* mhead) {
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (r >= E.nk) return;
  const uint32_t T = meta_tag(E.kmeta[r]);
  const uint64_t cref = E.kcref[r], cc = cref & 0xFFFFFF, cb = cref >> 24;
  if (!cc) return;
  if (T == TAG_COUNTER && cb < E.nn) nhead[cb] = (uint32_t)(r + 1);
  if ((T == TAG_SET || T == TAG_DICT) && cb < E.nm) mhead[cb] = (uint32_t)(r + 1);
}

struct ParentScan {  // "last non-zero": every child row gets the key index + 1 of its range head
  using V = uint32_t;
  uint32_t* a;
  uint64_t n;
  __device__ static V id() { return 0; }
  __device__ static V op(V x, V y) { return y ? y : x; }
  __device__ V load(uint64_t i) const { return a[i]; }
  __device__ void store(uint64_t i, V ex, V own) const {
    if (i < n) a[i] = op(ex, own);
  }
};

// does child row j lie inside key p's child range? (rows outside every range carry no bytes)
__device__ __forceinline__ bool in_range(const EncIn& E, uint32_t parent, uint64_t j, uint64_t* cb, uint64_t* cc) {
  if (!parent) return false;
  const uint64_t cref = E.kcref[parent - 1];
  *cb = cref >> 24;
  *cc = cref & 0xFFFFFF;
  return j >= *cb && j < *cb + *cc;
}

struct MemV {
  uint64_t a, d, na;  // add-map bytes, del-map bytes, adds
};
// Child sizes, computed once: a member's (kl, k, t[, vl, v]) bytes with its kind in bit 63
// (0 for rows outside every key's range), a node's (node, v, t) bytes. They are written into
// the scans' own output arrays (pd, pn), which the scans then overwrite in place: the apply
// kernel loads a tile's values before storing any of its prefixes.
__global__ void member_size_kernel(EncIn E, const uint32_t* parent, uint64_t* msz) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j >= E.nm) return;
  uint64_t cb, cc;
  const uint32_t p = parent[j];
  if (!in_range(E, p, j, &cb, &cc)) {
    msz[j] = 0;
    return;
  }
  const uint64_t mt = E.mmeta[j];
  const uint8_t* q;
  const ByteRef m = mem_span(E, mt, &q);
  uint64_t sz = vi_len((int64_t)m.len) + m.len + vi_len((int64_t)E.mt[j]);  // (kl, k, t)
  if (meta_tag(mt) == KIND_DEL) {
    msz[j] = sz;
    return;
  }
  if (meta_tag(E.kmeta[p - 1]) == TAG_DICT) {  // dict add: + (vl, v) (lwwhash.rs:194-195)
    const ByteRef v = mval_span(E, mt, &q);
    sz += vi_len((int64_t)v.len) + v.len;
  }
  msz[j] = (1ull << 63) | sz;
}
__global__ void node_size_kernel(EncIn E, const uint32_t* parent, uint64_t* nsz) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j >= E.nn) return;
  uint64_t cb, cc;
  nsz[j] = in_range(E, parent[j], j, &cb, &cc)
               ? vi_len((int64_t)E.nnode[j]) + vi_len((int64_t)E.nv[j]) + vi_len((int64_t)E.nt[j])
               : 0;
}

struct MemberScan {
  using V = MemV;
  uint64_t *pa, *pd, *pc;  // n + 1 entries; pd holds the sizes on entry
  __device__ static V id() { return V{0, 0, 0}; }
  __device__ static V op(V x, V y) { return V{x.a + y.a, x.d + y.d, x.na + y.na}; }
  __device__ V load(uint64_t j) const {
    const uint64_t z = pd[j], sz = z & ~(1ull << 63);
    return z >> 63 ? V{sz, 0, 1} : V{0, sz, 0};
  }
  __device__ void store(uint64_t j, V ex, V) const {
    pa[j] = ex.a;
    pd[j] = ex.d;
    pc[j] = ex.na;
  }
};

struct NodeScan {
  using V = uint64_t;
  uint64_t* pn;  // n + 1 entries; holds the sizes on entry
  __device__ static V id() { return 0; }
  __device__ static V op(V x, V y) { return x + y; }
  __device__ V load(uint64_t j) const { return pn[j]; }
  __device__ void store(uint64_t j, V ex, V) const { pn[j] = ex; }
};

// A key row's encoded entry: head bytes and, for data rows, the children's bytes.
struct KeyLayout {
  uint32_t fam;        // 0 DATAS, 1 EXPIRES, 2 DELETES
  uint64_t head;       // bytes before the children (incl. the add count / node count)
  uint64_t add_bytes;  // set/dict: add map bytes (the del count follows them)
  uint64_t na, nd;
  uint64_t total;
};
__device__ __forceinline__ KeyLayout key_layout(const EncIn& E, const uint64_t* pn, const uint64_t* pa,
                                                const uint64_t* pd, const uint64_t* pc, uint64_t r) {
  KeyLayout L{};
  const uint64_t meta = E.kmeta[r];
  const uint32_t T = meta_tag(meta);
  const uint8_t* q;
  const ByteRef k = key_span(E, meta, &q);
  const uint64_t kb = vi_len((int64_t)k.len) + k.len;
  if (T == TAG_EXPIRE || T == TAG_DELETE) {  // (klen, key, t) (db.rs:127-134)
    L.fam = T == TAG_EXPIRE ? 1 : 2;
    L.head = L.total = kb + vi_len((int64_t)E.kct[r]);
    return L;
  }
  L.fam = 0;
  L.head = kb + vi_len((int64_t)E.kct[r]) + vi_len((int64_t)E.kut[r]) + vi_len((int64_t)E.kdt[r]) + 1;
  const uint64_t cref = E.kcref[r], cb = cref >> 24, cc = cref & 0xFFFFFF;
  if (T == TAG_BYTES) {
    const ByteRef v = val_span(E, E.kwin[r], &q);
    L.head += vi_len((int64_t)v.len) + v.len;
    L.total = L.head;
  } else if (T == TAG_COUNTER) {
    L.head += vi_len((int64_t)cc);
    L.total = L.head + (cc ? pn[cb + cc] - pn[cb] : 0);
  } else {
    L.na = cc ? pc[cb + cc] - pc[cb] : 0;
    L.nd = cc - L.na;
    L.add_bytes = cc ? pa[cb + cc] - pa[cb] : 0;
    const uint64_t del_bytes = cc ? pd[cb + cc] - pd[cb] : 0;
    L.head += vi_len((int64_t)L.na);
    L.total = L.head + L.add_bytes + vi_len((int64_t)L.nd) + del_bytes;
  }
  return L;
}

struct KeyV {
  uint64_t b[3];  // bytes per section
  uint64_t c[3];  // entries per section
};
// per key row: fam << 62 | entry bytes (head + children), read by the key scan
__global__ void key_size_kernel(EncIn E, const uint64_t* pn, const uint64_t* pa, const uint64_t* pd,
                                const uint64_t* pc, uint64_t* ksz) {
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (r >= E.nk) return;
  const KeyLayout L = key_layout(E, pn, pa, pd, pc, r);
  ksz[r] = ((uint64_t)L.fam << 62) | L.total;
}

struct KeyScan {
  using V = KeyV;
  const uint64_t* ksz;
  uint64_t nk;
  uint64_t* koff;   // row offset inside its section
  KeyV* total;
  __device__ static V id() { return V{{0, 0, 0}, {0, 0, 0}}; }
  __device__ static V op(V x, V y) {
    return V{{x.b[0] + y.b[0], x.b[1] + y.b[1], x.b[2] + y.b[2]}, {x.c[0] + y.c[0], x.c[1] + y.c[1], x.c[2] + y.c[2]}};
  }
  __device__ V load(uint64_t r) const {
    const uint64_t z = ksz[r];
    V v = id();
    v.b[z >> 62] = z & ((1ull << 62) - 1);
    v.c[z >> 62] = 1;
    return v;
  }
  __device__ void store(uint64_t r, V ex, V own) const {
    if (r == nk) {
      *total = ex;
      return;
    }
    const uint32_t f = own.c[0] ? 0 : own.c[1] ? 1 : 2;
    koff[r] = ex.b[f];
  }
};

// Byte copy from global memory with dword-aligned loads (keys and values are short and start
// anywhere in the arena).
__device__ __forceinline__ void copy_in(uint8_t* o, const uint8_t* p, uint64_t n) {
  if (!n) return;
  const uintptr_t a0 = (uintptr_t)p & ~(uintptr_t)3;
  const uint32_t* w = (const uint32_t*)a0;
  uint32_t sh = (uint32_t)((uintptr_t)p - a0);
  uint32_t cur = *w;
  for (uint64_t i = 0; i < n; ++i) {
    o[i] = (uint8_t)(cur >> (8 * sh));
    if (++sh == 4 && i + 1 < n) {
      sh = 0;
      cur = *++w;
    }
  }
}

// Writes a key row's head (everything but its children and a Set/Dict's del count).
__device__ __forceinline__ void put_head(const EncIn& E, const KeyLayout& L, uint64_t r, uint8_t* o) {
  const uint64_t meta = E.kmeta[r];
  const uint32_t T = meta_tag(meta);
  const uint8_t* q;
  const ByteRef k = key_span(E, meta, &q);
  o += vi_put(o, (int64_t)k.len);  // write_entry (snapshot.rs:48-52) / db.rs:127-134
  copy_in(o, q, k.len);
  o += k.len;
  o += vi_put(o, (int64_t)E.kct[r]);
  if (L.fam) return;
  o += vi_put(o, (int64_t)E.kut[r]);  // object.rs:86-88
  o += vi_put(o, (int64_t)E.kdt[r]);
  *o++ = (uint8_t)T;
  if (T == TAG_BYTES) {  // len, bytes (the loader's layout, object.rs:114-117)
    const ByteRef v = val_span(E, E.kwin[r], &q);
    o += vi_put(o, (int64_t)v.len);
    copy_in(o, q, v.len);
  } else if (T == TAG_COUNTER) {
    vi_put(o, (int64_t)(E.kcref[r] & 0xFFFFFF));  // type_counter.rs:102
  } else {
    vi_put(o, (int64_t)L.na);  // lwwhash.rs:190 / 326
  }
}

// 5. emit: key heads. The entries of one workgroup's rows of one section are contiguous in the
// stream, so they are assembled in LDS and written out with coalesced dword stores (spans
// larger than the stage are written in place). A staged span also covers the rows' child
// regions: those bytes are garbage here and are written by the node / member kernels, which
// run after this one; the Set/Dict del counts inside them are written after the copies.
constexpr uint32_t kStage = 32768;
__global__ void __launch_bounds__(256) emit_keys_kernel(EncIn E, const uint64_t* pn, const uint64_t* pa,
                                                        const uint64_t* pd, const uint64_t* pc, const uint64_t* koff,
                                                        uint64_t base0, uint64_t base1, uint64_t base2, uint8_t* out,
                                                        uint64_t* childbase) {
  __shared__ uint8_t stage[kStage];
  __shared__ unsigned long long s_lo[3], s_hi[3];
  const uint32_t t = threadIdx.x;
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + t;
  const bool valid = r < E.nk;
  KeyLayout L{};
  uint64_t o = 0;
  if (t < 3) {
    s_lo[t] = ~0ull;
    s_hi[t] = 0;
  }
  __syncthreads();
  if (valid) {
    L = key_layout(E, pn, pa, pd, pc, r);
    o = (L.fam == 0 ? base0 : L.fam == 1 ? base1 : base2) + koff[r];
    atomicMin(&s_lo[L.fam], (unsigned long long)o);
    atomicMax(&s_hi[L.fam], (unsigned long long)(o + L.total));
  }
  __syncthreads();
  for (uint32_t f = 0; f < 3; ++f) {
    const uint64_t lo = s_lo[f], hi = s_hi[f];
    if (lo >= hi) continue;  // no rows of this section (uniform across the workgroup)
    const bool staged = hi - lo <= kStage;
    if (valid && L.fam == f) put_head(E, L, r, staged ? stage + (o - lo) : out + o);
    __syncthreads();
    if (staged) {
      // head bytes up to a dword boundary, then dwords, then the tail
      const uint64_t a = (lo + 3) & ~3ull, span = hi - lo;
      const uint64_t lead = std::min<uint64_t>(a - lo, span);
      if (t < lead) out[lo + t] = stage[t];
      const uint64_t words = (span - lead) / 4;
      for (uint64_t w = t; w < words; w += 256) {
        const uint64_t b = lead + 4 * w;
        const uint32_t v = (uint32_t)stage[b] | ((uint32_t)stage[b + 1] << 8) | ((uint32_t)stage[b + 2] << 16) |
                           ((uint32_t)stage[b + 3] << 24);
        *(uint32_t*)(out + a + 4 * w) = v;
      }
      const uint64_t done = lead + 4 * words;
      if (t < span - done) out[lo + done + t] = stage[done + t];
      __syncthreads();
    }
  }
  if (!valid || L.fam) return;
  const uint32_t T = meta_tag(E.kmeta[r]);
  if (T == TAG_BYTES) return;
  const uint64_t cb = o + L.head;  // where the children start
  childbase[r] = cb;
  if (T != TAG_COUNTER) vi_put(out + cb + L.add_bytes, (int64_t)L.nd);  // lwwhash.rs:198 / 331
}

__global__ void emit_nodes_kernel(EncIn E, const uint32_t* parent, const uint64_t* pn, const uint64_t* childbase,
                                  uint8_t* out) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j >= E.nn) return;
  uint64_t cb, cc;
  const uint32_t p = parent[j];
  if (!in_range(E, p, j, &cb, &cc)) return;
  uint8_t* o = out + childbase[p - 1] + (pn[j] - pn[cb]);
  o += vi_put(o, (int64_t)E.nnode[j]);  // type_counter.rs:104-106
  o += vi_put(o, (int64_t)E.nv[j]);
  vi_put(o, (int64_t)E.nt[j]);
}

__global__ void emit_members_kernel(EncIn E, const uint32_t* parent, const uint64_t* pa, const uint64_t* pd,
                                    const uint64_t* pc, const uint64_t* childbase, uint8_t* out) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j >= E.nm) return;
  uint64_t cb, cc;
  const uint32_t p = parent[j];
  if (!in_range(E, p, j, &cb, &cc)) return;
  const uint64_t mt = E.mmeta[j];
  const bool add = meta_tag(mt) == KIND_ADD;
  uint64_t at;
  if (add) {
    at = pa[j] - pa[cb];
  } else {
    const uint64_t e = cb + cc, na = pc[e] - pc[cb];
    at = (pa[e] - pa[cb]) + vi_len((int64_t)(cc - na)) + (pd[j] - pd[cb]);
  }
  uint8_t* o = out + childbase[p - 1] + at;
  const uint8_t* q;
  const ByteRef m = mem_span(E, mt, &q);
  o += vi_put(o, (int64_t)m.len);  // (kl, k, t[, vl, v]) lwwhash.rs:191-196 / 327-330
  copy_in(o, q, m.len);
  o += m.len;
  o += vi_put(o, (int64_t)E.mt[j]);
  if (add && meta_tag(E.kmeta[p - 1]) == TAG_DICT) {
    const ByteRef v = mval_span(E, mt, &q);
    o += vi_put(o, (int64_t)v.len);
    copy_in(o, q, v.len);
  }
}

// ------------------------------------------------------------------ host side
struct DevMem {
  void* p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};
cdb_status dalloc(cdb_ctx* ctx, DevMem& m, size_t bytes) {
  return hip_check(ctx, hipMalloc(&m.p, std::max<size_t>(bytes, 16)), "hipMalloc(encode)");
}
cdb_status h2d(cdb_ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t s) {
  return staged_h2d(ctx, dst, src, bytes, s);
}

template <class Tr>
cdb_status run_scan(cdb_ctx* ctx, const Tr& tr, uint64_t n, void* scratch, hipStream_t s) {
  const uint64_t tiles = std::max<uint64_t>(1, (n + kSTile - 1) / kSTile);
  auto* S = (typename Tr::V*)scratch;
  tscan_reduce<Tr><<<tiles, kST, 0, s>>>(tr, n, S);
  tscan_sums<Tr><<<1, kST, 0, s>>>(tr, tiles, S, n);
  tscan_apply<Tr><<<tiles, kST, 0, s>>>(tr, n, S);
  return launch_check(ctx, s, "encode scan");
}

struct Varints {
  std::vector<uint8_t> b;
  void integer(int64_t i) {
    uint8_t t[9];
    const uint32_t n = vi_put(t, i);
    b.insert(b.end(), t, t + n);
  }
  void bytes(const void* p, size_t n) {
    const uint8_t* q = (const uint8_t*)p;
    b.insert(b.end(), q, q + n);
  }
  void byte(uint8_t x) { b.push_back(x); }
};

// CRC over dev[0, padded) where padded is a whole number of tiles (zero prefix).
cdb_status crc_device(cdb_ctx* ctx, const uint8_t* dev, uint64_t padded, uint8_t* dst, uint64_t* d_crc, hipStream_t s) {
  // built once; a function-local static's initialisation is thread-safe (contexts may run on
  // different threads at the same time, cdb_merge.h)
  struct CrcTables {
    uint64_t t[8 * 256];
    CrcTables() { crc_tables(t); }
  };
  static const CrcTables tab;
  const uint64_t* tables = tab.t;
  const uint64_t tiles = padded / kCrcTile;
  const uint64_t run = std::max<uint64_t>(1, (tiles + kCrcThreads - 1) / kCrcThreads);
  CrcConsts K;
  for (int k = 0; k < 8; ++k) K.chunk_lvl[k] = x8n_mod((uint64_t)kCrcChunk << k);
  K.tile = x8n_mod(kCrcTile);
  for (int k = 0; k < 8; ++k) K.run_lvl[k] = x8n_mod((kCrcTile * run) << k);
  DevMem dt, dtc;
  cdb_status st;
  if ((st = dalloc(ctx, dt, sizeof tab.t)) != CDB_OK) return st;
  if ((st = dalloc(ctx, dtc, std::max<uint64_t>(tiles, 1) * 8)) != CDB_OK) return st;
  if ((st = h2d(ctx, dt.p, tables, sizeof tab.t, s)) != CDB_OK) return st;
  if (tiles) crc_tile_kernel<<<tiles, kCrcThreads, 0, s>>>(dev, (const uint64_t*)dt.p, K, (uint64_t*)dtc.p);
  crc_final_kernel<<<1, kCrcThreads, 0, s>>>((const uint64_t*)dtc.p, tiles, run, run * kCrcThreads - tiles, K, d_crc,
                                            dst);
  if ((st = launch_check(ctx, s, "crc")) != CDB_OK) return st;
  return hip_check(ctx, hipStreamSynchronize(s), "crc sync");
}

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

struct Events {
  hipEvent_t e[6] = {};
  Events() {
    for (auto& x : e) (void)hipEventCreate(&x);
  }
  ~Events() {
    for (auto& x : e)
      if (x) (void)hipEventDestroy(x);
  }
};

}  // namespace

cdb_status crc64_gpu_impl(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t* crc) {
  if (!len) {
    *crc = 0;
    return CDB_OK;
  }
  hipStream_t s = ctx->stream;
  const uint64_t pad = (kCrcTile - len % kCrcTile) % kCrcTile;
  DevMem d, dc;
  cdb_status st;
  if ((st = dalloc(ctx, d, pad + len)) != CDB_OK) return st;
  if ((st = dalloc(ctx, dc, 8)) != CDB_OK) return st;
  if ((st = hip_check(ctx, hipMemsetAsync(d.p, 0, pad, s), "memset")) != CDB_OK) return st;
  if ((st = h2d(ctx, (uint8_t*)d.p + pad, buf, len, s)) != CDB_OK) return st;
  if ((st = crc_device(ctx, (const uint8_t*)d.p, pad + len, nullptr, (uint64_t*)dc.p, s)) != CDB_OK) return st;
  return hip_check(ctx, hipMemcpy(crc, dc.p, 8, hipMemcpyDeviceToHost), "d2h crc");
}

namespace {

// Steps 1-6 of the encoder over result rows and byte tables already in HBM (E; E.pos set).
// ev.e[0] / e[1] were recorded by the caller around its uploads.
cdb_status encode_rows(cdb_ctx* ctx, const EncIn& E, const cdb_encode_header& hdr, uint8_t** out, size_t* out_len,
                       cdb_encode_stats* stats, Events& ev);

}  // namespace

cdb_status encode_snapshot_impl(cdb_ctx* ctx, const cdb_merged& m, const cdb_encode_header& hdr, uint8_t** out,
                                size_t* out_len, cdb_encode_stats* stats) {
  hipStream_t s = ctx->stream;
  const uint64_t nk = m.k[O_META].size(), nn = m.nd[C_ID1].size(), nm = m.mb[C_META].size();
  if (nk >= 0xFFFFFFFFull) return fail(ctx, CDB_BAD_ARGUMENT, "encode: more than 2^32-2 key rows");
  Events ev;
  (void)hipEventRecord(ev.e[0], s);
  // ---- uploads: result rows, byte arenas and ref tables (one allocation each), position table
  struct Base { uint64_t arena, krow, mrow; };
  std::vector<Base> pb(m.inputs.size());
  uint64_t arena = 0, krow = 0, mrow = 0;
  for (size_t p = 0; p < m.inputs.size(); ++p) {
    const Batch& b = *m.inputs[p];
    pb[p] = Base{arena, krow, mrow};
    arena += b.raw.size();
    krow += b.key_ref.size();
    mrow += b.m_ref.size();
  }
  DevMem dk, dn, dm, dpos, dar, dkr, dvr, dmr, dmvr;
  cdb_status st;
  if ((st = dalloc(ctx, dk, 6 * nk * 8)) != CDB_OK || (st = dalloc(ctx, dn, 3 * nn * 8)) != CDB_OK ||
      (st = dalloc(ctx, dm, 2 * nm * 8)) != CDB_OK || (st = dalloc(ctx, dpos, pb.size() * sizeof(EncPos))) != CDB_OK ||
      (st = dalloc(ctx, dar, arena + 8)) != CDB_OK || (st = dalloc(ctx, dkr, krow * sizeof(ByteRef))) != CDB_OK ||
      (st = dalloc(ctx, dvr, krow * sizeof(ByteRef))) != CDB_OK ||
      (st = dalloc(ctx, dmr, mrow * sizeof(ByteRef))) != CDB_OK ||
      (st = dalloc(ctx, dmvr, mrow * sizeof(ByteRef))) != CDB_OK)
    return st;
  EncIn E{};
  uint64_t* K = (uint64_t*)dk.p;
  const int kcols[6] = {O_META, O_CT, O_UT, O_DT, O_WIN, O_CREF};
  for (int c = 0; c < 6; ++c)
    if ((st = h2d(ctx, K + c * nk, m.k[kcols[c]].data(), nk * 8, s)) != CDB_OK) return st;
  E.kmeta = K;
  E.kct = K + nk;
  E.kut = K + 2 * nk;
  E.kdt = K + 3 * nk;
  E.kwin = K + 4 * nk;
  E.kcref = K + 5 * nk;
  uint64_t* N = (uint64_t*)dn.p;
  const int ncols[3] = {C_ID1, C_ID2, C_T};
  for (int c = 0; c < 3; ++c)
    if ((st = h2d(ctx, N + c * nn, m.nd[ncols[c]].data(), nn * 8, s)) != CDB_OK) return st;
  E.nnode = N;
  E.nv = N + nn;
  E.nt = N + 2 * nn;
  uint64_t* M = (uint64_t*)dm.p;
  if ((st = h2d(ctx, M, m.mb[C_T].data(), nm * 8, s)) != CDB_OK ||
      (st = h2d(ctx, M + nm, m.mb[C_META].data(), nm * 8, s)) != CDB_OK)
    return st;
  E.mt = M;
  E.mmeta = M + nm;
  E.nk = nk;
  E.nn = nn;
  E.nm = nm;
  std::vector<EncPos> pos(m.inputs.size());
  for (size_t p = 0; p < m.inputs.size(); ++p) {
    const Batch& b = *m.inputs[p];
    pos[p] = EncPos{(const uint8_t*)dar.p + pb[p].arena, (const ByteRef*)dkr.p + pb[p].krow,
                    (const ByteRef*)dvr.p + pb[p].krow, (const ByteRef*)dmr.p + pb[p].mrow,
                    (const ByteRef*)dmvr.p + pb[p].mrow};
    if ((st = h2d(ctx, (void*)pos[p].raw, b.raw.data(), b.raw.size(), s)) != CDB_OK ||
        (st = h2d(ctx, (void*)pos[p].kref, b.key_ref.data(), b.key_ref.size() * sizeof(ByteRef), s)) != CDB_OK ||
        (st = h2d(ctx, (void*)pos[p].vref, b.val_ref.data(), b.val_ref.size() * sizeof(ByteRef), s)) != CDB_OK ||
        (st = h2d(ctx, (void*)pos[p].mref, b.m_ref.data(), b.m_ref.size() * sizeof(ByteRef), s)) != CDB_OK ||
        (st = h2d(ctx, (void*)pos[p].mvref, b.m_vref.data(), b.m_vref.size() * sizeof(ByteRef), s)) != CDB_OK)
      return st;
  }
  if ((st = h2d(ctx, dpos.p, pos.data(), pos.size() * sizeof(EncPos), s)) != CDB_OK) return st;
  E.pos = (const EncPos*)dpos.p;
  (void)hipEventRecord(ev.e[1], s);
  return encode_rows(ctx, E, hdr, out, out_len, stats, ev);
}

cdb_status encode_device_impl(cdb_ctx* ctx, const cdb_dev_output& dout, const std::vector<Batch*>& inputs,
                              const cdb_encode_header& hdr, uint8_t** out, size_t* out_len, cdb_encode_stats* stats) {
  hipStream_t s = ctx->stream;
  const uint64_t nk = dout.keys.n, nn = dout.nodes.n, nm = dout.members.n;
  if (nk >= 0xFFFFFFFFull) return fail(ctx, CDB_BAD_ARGUMENT, "encode: more than 2^32-2 key rows");
  if (dout.compact && (dout.keys.stride > 1 || dout.nodes.stride > 1 || dout.members.stride > 1))
    return fail(ctx, CDB_BAD_ARGUMENT, "encode: a compacted result is in plain columns");
  // the byte tables of device-decoded batches stay in HBM for the whole call (refs_ready and
  // another encoder wait); a batch at several positions is locked once
  std::vector<std::shared_ptr<DeviceRefs>> held;
  std::vector<std::unique_lock<std::mutex>> locks;
  for (Batch* b : inputs)
    if (b->dev_refs && std::find(held.begin(), held.end(), b->dev_refs) == held.end()) held.push_back(b->dev_refs);
  std::sort(held.begin(), held.end());  // (one lock order for every caller)
  for (auto& r : held) locks.emplace_back(r->mu);
  for (auto& r : held)
    if ((r->dev || r->raw) && r->device != ctx->device)
      return fail(ctx, CDB_BAD_ARGUMENT, "encode: byte references live on another device");
  Events ev;
  (void)hipEventRecord(ev.e[0], s);
  cdb_status st;
  // ---- result rows: the bucket layout compacted into temporary columns, dense columns as they are
  cdb_dev_output dense;
  std::memset(&dense, 0, sizeof dense);
  struct Release {
    cdb_ctx* c;
    cdb_dev_output* d;
    ~Release() {
      cdb_dev_rows_release(c, &d->keys);
      cdb_dev_rows_release(c, &d->nodes);
      cdb_dev_rows_release(c, &d->members);
    }
  } release{ctx, &dense};
  const cdb_dev_output* rows = &dout;
  if (!dout.compact) {
    if ((st = cdb_dev_rows_alloc(ctx, &dense.keys, nk, kKeyOutCols)) != CDB_OK ||
        (st = cdb_dev_rows_alloc(ctx, &dense.nodes, nn, kNodeCols)) != CDB_OK ||
        (st = cdb_dev_rows_alloc(ctx, &dense.members, nm, kMemberCols)) != CDB_OK ||
        (st = cdb_dev_output_compact(ctx, &dout, &dense, s)) != CDB_OK)
      return st;
    rows = &dense;
  }
  EncIn E{};
  E.kmeta = rows->keys.col[O_META];
  E.kct = rows->keys.col[O_CT];
  E.kut = rows->keys.col[O_UT];
  E.kdt = rows->keys.col[O_DT];
  E.kwin = rows->keys.col[O_WIN];
  E.kcref = rows->keys.col[O_CREF];
  E.nnode = rows->nodes.col[C_ID1];
  E.nv = rows->nodes.col[C_ID2];
  E.nt = rows->nodes.col[C_T];
  E.mt = rows->members.col[C_T];
  E.mmeta = rows->members.col[C_META];
  E.nk = nk;
  E.nn = nn;
  E.nm = nm;
  // ---- per position: snapshot bytes and byte references from HBM where the decode left them,
  // else uploaded (host tables: one allocation per batch)
  std::vector<EncPos> pos(inputs.size());
  std::vector<std::unique_ptr<DevMem>> tmp;
  for (size_t p = 0; p < inputs.size(); ++p) {
    Batch& b = *inputs[p];
    DeviceRefs* r = b.dev_refs.get();
    if (r && r->raw) {
      pos[p].raw = (const uint8_t*)r->raw + r->raw_off;
    } else {
      tmp.emplace_back(new DevMem);
      if ((st = dalloc(ctx, *tmp.back(), b.raw.size() + 8)) != CDB_OK ||
          (st = h2d(ctx, tmp.back()->p, b.raw.data(), b.raw.size(), s)) != CDB_OK)
        return st;
      pos[p].raw = (const uint8_t*)tmp.back()->p;
    }
    if (r && r->dev) {
      ByteRef* d = (ByteRef*)r->dev;
      if (!r->patch.empty()) {  // host-tier member refs: into the HBM tables once
        static_assert(sizeof(RefPatch) == sizeof(DeviceRefs::Patch), "patch layout");
        DevMem dp;
        const uint64_t np = r->patch.size();
        if ((st = dalloc(ctx, dp, np * sizeof(RefPatch))) != CDB_OK ||
            (st = hip_check(ctx, hipMemcpyAsync(dp.p, r->patch.data(), np * sizeof(RefPatch), hipMemcpyHostToDevice, s),
                            "h2d(patch)")) != CDB_OK)
          return st;
        patch_refs_kernel<<<(np + 255) / 256, 256, 0, s>>>((const RefPatch*)dp.p, np, d + 2 * r->n,
                                                            d + 2 * r->n + r->nm);
        if ((st = launch_check(ctx, s, "patch_refs")) != CDB_OK ||
            (st = hip_check(ctx, hipStreamSynchronize(s), "sync(patch)")) != CDB_OK)
          return st;
        r->patch.clear();
      }
      pos[p].kref = d;
      pos[p].vref = d + r->n;
      pos[p].mref = d + 2 * r->n;
      pos[p].mvref = d + 2 * r->n + r->nm;
    } else {
      const uint64_t n = b.key_ref.size(), mn = b.m_ref.size();
      tmp.emplace_back(new DevMem);
      if ((st = dalloc(ctx, *tmp.back(), (2 * n + 2 * mn) * sizeof(ByteRef))) != CDB_OK) return st;
      ByteRef* d = (ByteRef*)tmp.back()->p;
      if ((st = h2d(ctx, d, b.key_ref.data(), n * sizeof(ByteRef), s)) != CDB_OK ||
          (st = h2d(ctx, d + n, b.val_ref.data(), n * sizeof(ByteRef), s)) != CDB_OK ||
          (st = h2d(ctx, d + 2 * n, b.m_ref.data(), mn * sizeof(ByteRef), s)) != CDB_OK ||
          (st = h2d(ctx, d + 2 * n + mn, b.m_vref.data(), mn * sizeof(ByteRef), s)) != CDB_OK)
        return st;
      pos[p].kref = d;
      pos[p].vref = d + n;
      pos[p].mref = d + 2 * n;
      pos[p].mvref = d + 2 * n + mn;
    }
  }
  DevMem dpos;
  if ((st = dalloc(ctx, dpos, pos.size() * sizeof(EncPos))) != CDB_OK ||
      (st = h2d(ctx, dpos.p, pos.data(), pos.size() * sizeof(EncPos), s)) != CDB_OK)
    return st;
  E.pos = (const EncPos*)dpos.p;
  (void)hipEventRecord(ev.e[1], s);
  return encode_rows(ctx, E, hdr, out, out_len, stats, ev);
}

namespace {

cdb_status encode_rows(cdb_ctx* ctx, const EncIn& E, const cdb_encode_header& hdr, uint8_t** out, size_t* out_len,
                       cdb_encode_stats* stats, Events& ev) {
  hipStream_t s = ctx->stream;
  const uint64_t nk = E.nk, nn = E.nn, nm = E.nm;
  cdb_status st;

  // ---- 1-3. sizing scans
  DevMem dnh, dmh, dpn, dpa, dpd, dpc, dko, dtot, dcb;
  if ((st = dalloc(ctx, dnh, (nn + 1) * 4)) != CDB_OK || (st = dalloc(ctx, dmh, (nm + 1) * 4)) != CDB_OK ||
      (st = dalloc(ctx, dpn, (nn + 1) * 8)) != CDB_OK || (st = dalloc(ctx, dpa, (nm + 1) * 8)) != CDB_OK ||
      (st = dalloc(ctx, dpd, (nm + 1) * 8)) != CDB_OK || (st = dalloc(ctx, dpc, (nm + 1) * 8)) != CDB_OK ||
      (st = dalloc(ctx, dko, nk * 8)) != CDB_OK || (st = dalloc(ctx, dtot, sizeof(KeyV))) != CDB_OK ||
      (st = dalloc(ctx, dcb, nk * 8)) != CDB_OK)
    return st;
  uint32_t *nhead = (uint32_t*)dnh.p, *mhead = (uint32_t*)dmh.p;
  if ((st = hip_check(ctx, hipMemsetAsync(nhead, 0, (nn + 1) * 4, s), "memset")) != CDB_OK ||
      (st = hip_check(ctx, hipMemsetAsync(mhead, 0, (nm + 1) * 4, s), "memset")) != CDB_OK)
    return st;
  if (nk) mark_heads_kernel<<<(nk + 255) / 256, 256, 0, s>>>(E, nhead, mhead);
  if ((st = launch_check(ctx, s, "mark_heads")) != CDB_OK) return st;
  DevMem dscr;  // scan tile sums, sized for the largest scan
  const uint64_t max_rows = std::max(std::max(nk, nn), nm);
  if ((st = dalloc(ctx, dscr, ((max_rows + kSTile - 1) / kSTile + 1) * sizeof(KeyV))) != CDB_OK) return st;
  if ((st = run_scan(ctx, ParentScan{nhead, nn}, nn, dscr.p, s)) != CDB_OK) return st;
  if ((st = run_scan(ctx, ParentScan{mhead, nm}, nm, dscr.p, s)) != CDB_OK) return st;
  uint64_t *pn = (uint64_t*)dpn.p, *pa = (uint64_t*)dpa.p, *pd = (uint64_t*)dpd.p, *pc = (uint64_t*)dpc.p;
  if (nn) node_size_kernel<<<(nn + 255) / 256, 256, 0, s>>>(E, nhead, pn);
  if (nm) member_size_kernel<<<(nm + 255) / 256, 256, 0, s>>>(E, mhead, pd);
  if ((st = launch_check(ctx, s, "child sizes")) != CDB_OK) return st;
  if ((st = run_scan(ctx, NodeScan{pn}, nn, dscr.p, s)) != CDB_OK) return st;
  if ((st = run_scan(ctx, MemberScan{pa, pd, pc}, nm, dscr.p, s)) != CDB_OK) return st;
  uint64_t* koff = (uint64_t*)dko.p;
  uint64_t* ksz = (uint64_t*)dcb.p;  // the sizes live in the childbase buffer until the emit
  if (nk) key_size_kernel<<<(nk + 255) / 256, 256, 0, s>>>(E, pn, pa, pd, pc, ksz);
  if ((st = launch_check(ctx, s, "key_size")) != CDB_OK) return st;
  if ((st = run_scan(ctx, KeyScan{ksz, nk, koff, (KeyV*)dtot.p}, nk, dscr.p, s)) != CDB_OK) return st;
  KeyV tot;
  if ((st = hip_check(ctx, hipMemcpyAsync(&tot, dtot.p, sizeof tot, hipMemcpyDeviceToHost, s), "d2h totals")) !=
          CDB_OK ||
      (st = hip_check(ctx, hipStreamSynchronize(s), "sync")) != CDB_OK)
    return st;

  // ---- 4. host: node header, section headers, replica entries (server.rs:189-208)
  Varints A, B, C, D;
  A.bytes("CONSTDB", 7);
  const uint8_t ver[4] = {0, 1, 1, 1};
  A.bytes(ver, 4);
  A.integer((int64_t)hdr.node_id);
  A.integer((int64_t)hdr.alias_len);
  A.bytes(hdr.alias, hdr.alias_len);
  A.integer((int64_t)hdr.addr_len);
  A.bytes(hdr.addr, hdr.addr_len);
  A.integer((int64_t)hdr.last_uuid);
  A.byte(5);  // SNAPSHOT_FLAG_DATAS + len (db.rs:123)
  A.integer((int64_t)tot.c[0]);
  B.byte(6);
  B.integer((int64_t)tot.c[1]);
  C.byte(7);
  C.integer((int64_t)tot.c[2]);
  for (size_t i = 0; i < hdr.n_replicas; ++i) {  // replica.rs:101-110
    const cdb_replica_entry& r = hdr.replicas[i];
    if (!r.has_add) continue;
    const size_t al = r.alias ? std::strlen(r.alias) : 0, ad = r.addr ? std::strlen(r.addr) : 0;
    D.byte(3);
    D.integer((int64_t)r.add_time);
    D.integer((int64_t)r.node_id);
    D.integer((int64_t)al);
    D.bytes(r.alias, al);
    D.integer((int64_t)ad);
    D.bytes(r.addr, ad);
    D.integer((int64_t)r.uuid_he_sent);
  }
  for (size_t i = 0; i < hdr.n_replicas; ++i) {  // replica.rs:112-117
    const cdb_replica_entry& r = hdr.replicas[i];
    if (!r.has_del) continue;
    const size_t ad = r.addr ? std::strlen(r.addr) : 0;
    D.byte(4);
    D.integer((int64_t)ad);
    D.bytes(r.addr, ad);
    D.integer((int64_t)r.del_time);
  }
  D.byte(8);  // SNAPSHOT_FLAG_CHECKSUM
  const uint64_t base0 = A.b.size(), base1 = base0 + tot.b[0] + B.b.size(), base2 = base1 + tot.b[1] + C.b.size();
  const uint64_t tail = base2 + tot.b[2], L = tail + D.b.size();  // bytes the CRC covers
  const uint64_t pad = (kCrcTile - L % kCrcTile) % kCrcTile;
  DevMem dout, dcrc;
  if ((st = dalloc(ctx, dout, pad + L + 8)) != CDB_OK || (st = dalloc(ctx, dcrc, 8)) != CDB_OK) return st;
  uint8_t* dev = (uint8_t*)dout.p + pad;
  if ((st = hip_check(ctx, hipMemsetAsync(dout.p, 0, pad, s), "memset")) != CDB_OK ||
      (st = h2d(ctx, dev, A.b.data(), A.b.size(), s)) != CDB_OK ||
      (st = h2d(ctx, dev + base0 + tot.b[0], B.b.data(), B.b.size(), s)) != CDB_OK ||
      (st = h2d(ctx, dev + base1 + tot.b[1], C.b.data(), C.b.size(), s)) != CDB_OK ||
      (st = h2d(ctx, dev + tail, D.b.data(), D.b.size(), s)) != CDB_OK)
    return st;

  // ---- 5. emit
  uint64_t* childbase = (uint64_t*)dcb.p;
  if (nk)
    emit_keys_kernel<<<(nk + 255) / 256, 256, 0, s>>>(E, pn, pa, pd, pc, koff, base0, base1, base2, dev, childbase);
  if (nn) emit_nodes_kernel<<<(nn + 255) / 256, 256, 0, s>>>(E, nhead, pn, childbase, dev);
  if (nm) emit_members_kernel<<<(nm + 255) / 256, 256, 0, s>>>(E, mhead, pa, pd, pc, childbase, dev);
  if ((st = launch_check(ctx, s, "emit")) != CDB_OK) return st;

  // ---- 6. CRC-64/Jones over [0, L) and its 8 LE bytes at L (server.rs:205-207)
  (void)hipEventRecord(ev.e[2], s);
  if ((st = crc_device(ctx, (const uint8_t*)dout.p, pad + L, dev + L, (uint64_t*)dcrc.p, s)) != CDB_OK) return st;
  (void)hipEventRecord(ev.e[3], s);
  uint8_t* host = (uint8_t*)std::malloc(L + 8);
  if (!host) return fail(ctx, CDB_OUT_OF_MEMORY, "encode: host buffer");
  uint64_t crc = 0;
  advise_huge(host, L + 8);
  if ((st = staged_d2h(ctx, host, dev, L + 8, s)) != CDB_OK ||
      (st = hip_check(ctx, hipMemcpyAsync(&crc, dcrc.p, 8, hipMemcpyDeviceToHost, s), "d2h crc")) != CDB_OK ||
      (st = hip_check(ctx, hipStreamSynchronize(s), "sync")) != CDB_OK) {
    std::free(host);
    return st;
  }
  (void)hipEventRecord(ev.e[4], s);
  (void)hipEventSynchronize(ev.e[4]);
  *out = host;
  *out_len = L + 8;
  if (stats) {
    stats->bytes = L + 8;
    stats->data_entries = tot.c[0];
    stats->expires = tot.c[1];
    stats->deletes = tot.c[2];
    stats->checksum = crc;
    stats->upload_ms = elapsed(ev.e[0], ev.e[1]);
    stats->device_ms = elapsed(ev.e[1], ev.e[3]);
    stats->crc_ms = elapsed(ev.e[2], ev.e[3]);
    stats->download_ms = elapsed(ev.e[3], ev.e[4]);
  }
  return CDB_OK;
}

}  // namespace

// CRC-64/Jones of a device buffer whose length is a multiple of crc_tile_bytes() (leading
// zero bytes do not change it); the result lands in d_crc. Synchronises the stream.
uint64_t crc_tile_bytes() { return kCrcTile; }
cdb_status crc64_device(cdb_ctx* ctx, const uint8_t* dev, uint64_t padded, uint64_t* d_crc, hipStream_t s) {
  return crc_device(ctx, dev, padded, nullptr, d_crc, s);
}

cdb_status crc64_device_queued(cdb_ctx* ctx, const uint8_t* dev, uint64_t padded, uint64_t* d_crc, hipStream_t s) {
  struct CrcTables {
    uint64_t t[8 * 256];
    CrcTables() { crc_tables(t); }
  };
  static const CrcTables tab;
  const uint64_t tiles = padded / kCrcTile;
  const uint64_t run = std::max<uint64_t>(1, (tiles + kCrcThreads - 1) / kCrcThreads);
  CrcConsts K;
  for (int k = 0; k < 8; ++k) K.chunk_lvl[k] = x8n_mod((uint64_t)kCrcChunk << k);
  K.tile = x8n_mod(kCrcTile);
  for (int k = 0; k < 8; ++k) K.run_lvl[k] = x8n_mod((kCrcTile * run) << k);
  cdb_status st = CDB_OK;
  const bool fresh = ctx->ws[WS_CRCTAB].p == nullptr;
  uint64_t* dt = (uint64_t*)ws_get(ctx, WS_CRCTAB, sizeof tab.t, &st);
  if (!dt) return st;
  if (fresh) {  // the tables go up once per context (a synchronous copy: the host table is static)
    if ((st = hip_check(ctx, hipMemcpy(dt, tab.t, sizeof tab.t, hipMemcpyHostToDevice), "h2d(crc tables)")) != CDB_OK)
      return st;
  }
  uint64_t* dtc = (uint64_t*)ws_get(ctx, WS_CRCPART, std::max<uint64_t>(tiles, 1) * 8, &st);
  if (!dtc) return st;
  if (tiles) crc_tile_kernel<<<tiles, kCrcThreads, 0, s>>>(dev, dt, K, dtc);
  crc_final_kernel<<<1, kCrcThreads, 0, s>>>(dtc, tiles, run, run * kCrcThreads - tiles, K, d_crc, nullptr);
  return launch_check(ctx, s, "crc");
}

}  // namespace cdb
