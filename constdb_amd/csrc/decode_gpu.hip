// GPU snapshot decode: snapshot bytes -> the same columnar Batch as
// decode.cpp, with the per-entry work on the GPU.
//
// The wire format (snapshot.rs:25-64,120-295) is a sequential varint stream: an entry's start
// is known only after its predecessor is parsed. Two passes:
//   1. host: index_snapshot() walks the stream once with the reference loader's checks (same
//      status codes and offsets as decode_snapshot), decodes the header, replica entries and
//      checksum, and records each entry's byte offset and kind. It hashes nothing and builds
//      no rows;
//   2. GPU, one thread per entry, over the bytes in HBM:
//      count_kernel   parses the entry and counts the children the loader keeps after its
//                     load-time dedup (type_counter.rs:111-126: the last of a repeated node id;
//                     lwwhash.rs:207-226,341-358: set/rem replay per member);
//      (scan of the counts: child row offsets)
//      emit_kernel    parses it again and writes the key row (hash of the key bytes, times,
//                     counter total, tag | src) and its kept child rows (member hashes).
//   Entries whose children exceed the per-thread dedup limits (a key with thousands of
//   members) are decoded on the host by decode.cpp's own functions into their reserved slots.
#include <hip/hip_runtime.h>
#include <condition_variable>
#include <deque>
#include <mutex>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "batch.h"
#include "engine.h"
#include "partition.hip.h"

namespace cdb {
namespace {

constexpr uint32_t kHostTier = 0xFFFFFFFFu;
constexpr uint32_t kNodeDedupMax = 64;    // nodes per counter deduplicated by one thread
constexpr uint32_t kMemberDedupMax = 32;  // set/dict tags per object deduplicated by one thread
constexpr int kDecThreads = 256;

// read_integer (snapshot.rs:243-264): 2-bit size tag in the flag byte's top bits.
__device__ __forceinline__ int64_t rd_int(const uint8_t* p, uint64_t& o) {
  const uint32_t f = p[o++];
  switch (f >> 6) {
    case 0: return (int64_t)(f & 0x3F);
    case 1: {
      const int64_t v = ((int64_t)(f & 0x3F) << 8) | p[o];
      o += 1;
      return v;
    }
    case 2: {
      const int64_t v = ((int64_t)(f & 0x3F) << 24) | ((int64_t)p[o] << 16) | ((int64_t)p[o + 1] << 8) | p[o + 2];
      o += 3;
      return v;
    }
    default: {
      uint64_t v = 0;
      for (int i = 0; i < 8; ++i) v = (v << 8) | p[o + i];
      o += 8;
      return (int64_t)v;
    }
  }
}
struct Span {
  uint64_t off, len;
};
__device__ __forceinline__ Span rd_span(const uint8_t* p, uint64_t& o) {
  Span s;
  s.len = (uint64_t)rd_int(p, o);
  s.off = o;
  o += s.len;
  return s;
}

struct DecArgs {
  const uint8_t* raw;
  const uint64_t* off;
  const uint8_t* kind;
  uint64_t n;
  uint32_t *ncount, *mcount;        // count pass: kept children per entry (kHostTier: host decodes)
  const uint64_t *noff, *moff;      // emit pass: first child row of each entry
  uint64_t* k[7];                   // kh kf ct ut dt aux meta
  ulonglong2 *kref, *vref;           // byte references as (offset, length): Batch::key_ref / val_ref
  uint64_t* nd[6];                  // pkh pkf node v t meta
  uint64_t* mb[6];                  // pkh pkf mh mf t meta
  ulonglong2 *mref, *mvref;          // Batch::m_ref / m_vref
  uint32_t pos;                     // fold position stamped into meta (device-resident emit)
  const uint32_t* dest;             // device-resident emit: key row of entry i (null: row i)
  uint32_t ks, cs;                  // record strides of k / nd, mb (1: columns; the records layout of
                                    // cdb_dev_rows: field c >= 1 of row r at col[c][r * stride])
};
__device__ __forceinline__ uint64_t& dcell(uint64_t* const* col, uint32_t s, int c, uint64_t r) {
  return col[c][c ? r * s : r];
}
// A whole row: the hash word, then fields 1.. -- in the records layout (s = ncols - 1) as 16-B
// pieces of the record (8-B aligned), not one partial-line store per field.
typedef unsigned long long dec_u64x2 __attribute__((ext_vector_type(2), aligned(8)));
template <int NC>
__device__ __forceinline__ void put_row(uint64_t* const* col, uint32_t s, uint64_t r, const uint64_t (&f)[NC]) {
  col[0][r] = f[0];
  if (s == NC - 1) {
    uint64_t* rec = col[1] + r * (NC - 1);
#pragma unroll
    for (int c = 1; c + 1 < NC; c += 2) {
      dec_u64x2 q;
      q.x = f[c];
      q.y = f[c + 1];
      *reinterpret_cast<dec_u64x2*>(rec + (c - 1)) = q;
    }
    if ((NC - 1) & 1) rec[NC - 2] = f[NC - 1];
  } else {
#pragma unroll
    for (int c = 1; c < NC; ++c) col[c][r] = f[c];
  }
}

struct Head {  // the part of a DATAS entry before the payload
  Span key;
  uint64_t ct, ut, dt;
  uint32_t tag;
};
__device__ __forceinline__ Head rd_head(const uint8_t* p, uint64_t& o) {
  Head h;
  h.key = rd_span(p, o);
  h.ct = (uint64_t)rd_int(p, o);
  h.ut = (uint64_t)rd_int(p, o);
  h.dt = (uint64_t)rd_int(p, o);
  h.tag = p[o++];
  return h;
}


// Keeps, per member, the op the loader's set/rem replay leaves holding the tag (lwwhash.rs:
// 87-128 driven by load_snapshot): the first op, replaced by every later op whose time is
// not older. `keep` bit j set = tag j is emitted.
__device__ __forceinline__ uint32_t member_keep(const uint8_t* p, uint64_t o, bool dict, uint32_t na, uint32_t nd,
                                                uint64_t* keep_lo /*bits 0..31*/) {
  Hash128 h[kMemberDedupMax];
  uint64_t t[kMemberDedupMax];
  const uint32_t n = na + nd;
  uint64_t q = o;
  for (uint32_t j = 0; j < n; ++j) {
    if (j == na) (void)rd_int(p, q);  // the dels' count
    const Span m = rd_span(p, q);
    t[j] = (uint64_t)rd_int(p, q);
    if (dict && j < na) (void)rd_span(p, q);
    h[j] = hash_bytes(p + m.off, m.len, kDomainMember);
  }
  uint64_t keep = 0;
  uint32_t kept = 0;
  for (uint32_t j = 0; j < n; ++j) {
    int st = -1;
    for (uint32_t i = 0; i < n; ++i) {
      if (h[i].h != h[j].h || h[i].f != h[j].f) continue;
      if (st >= 0 && t[st] > t[i]) continue;
      st = (int)i;
    }
    if (st == (int)j) {
      keep |= 1ull << j;
      ++kept;
    }
  }
  *keep_lo = keep;
  return kept;
}

__global__ void __launch_bounds__(kDecThreads) count_kernel(DecArgs A) {
  const uint64_t i = (uint64_t)blockIdx.x * kDecThreads + threadIdx.x;
  if (i >= A.n) return;
  uint32_t nc = 0, mc = 0;
  if (A.kind[i] == 0) {
    const uint8_t* p = A.raw;
    uint64_t o = A.off[i];
    const Head hd = rd_head(p, o);
    if (hd.tag == TAG_COUNTER) {
      const uint64_t cnt = (uint64_t)rd_int(p, o);
      if (cnt > kNodeDedupMax) {
        nc = kHostTier;
      } else {
        // node j is kept unless a later triple repeats its id (HashMap::insert keeps the last)
        uint64_t q = o;
        for (uint32_t j = 0; j < cnt; ++j) {
          const uint64_t id = (uint64_t)rd_int(p, q);
          (void)rd_int(p, q);
          (void)rd_int(p, q);
          uint64_t r = q;
          bool later = false;
          for (uint32_t k = j + 1; k < cnt; ++k) {
            later |= (uint64_t)rd_int(p, r) == id;
            (void)rd_int(p, r);
            (void)rd_int(p, r);
          }
          nc += later ? 0 : 1;
        }
      }
    } else if (hd.tag == TAG_SET || hd.tag == TAG_DICT) {
      const bool dict = hd.tag == TAG_DICT;
      const uint32_t na = (uint32_t)rd_int(p, o);
      uint64_t q = o;
      for (uint32_t j = 0; j < na; ++j) {
        (void)rd_span(p, q);
        (void)rd_int(p, q);
        if (dict) (void)rd_span(p, q);
      }
      const uint32_t nd = (uint32_t)rd_int(p, q);
      if ((uint64_t)na + nd > kMemberDedupMax) {
        mc = kHostTier;
      } else {
        uint64_t keep;
        mc = member_keep(p, o, dict, na, nd, &keep);
      }
    }
  }
  A.ncount[i] = nc;
  A.mcount[i] = mc;
}

__global__ void __launch_bounds__(kDecThreads) emit_kernel(DecArgs A) {
  const uint64_t i = (uint64_t)blockIdx.x * kDecThreads + threadIdx.x;
  if (i >= A.n) return;
  const uint8_t* p = A.raw;
  uint64_t o = A.off[i];
  const uint64_t kr = A.dest ? A.dest[i] : i;  // the key row (its src stays the entry index)
  if (A.kind[i] != 0) {  // EXPIRES / DELETES: key, t (read_key_int, snapshot.rs:289-295)
    const Span key = rd_span(p, o);
    const uint64_t t = (uint64_t)rd_int(p, o);
    const Hash128 h = hash_bytes(p + key.off, key.len, kDomainKey);
    const uint64_t f[7] = {h.h, h.f, t, 0, 0, 0, meta_pack(A.kind[i] == 1 ? TAG_EXPIRE : TAG_DELETE, A.pos, i)};
    put_row<7>(A.k, A.ks, kr, f);
    A.kref[i] = make_ulonglong2(key.off, key.len);
    A.vref[i] = make_ulonglong2(0, 0);
    return;
  }
  const Head hd = rd_head(p, o);
  const Hash128 h = hash_bytes(p + hd.key.off, hd.key.len, kDomainKey);
  uint64_t aux = 0;
  Span val{0, 0};
  if (hd.tag == TAG_BYTES) {
    val = rd_span(p, o);
  } else if (hd.tag == TAG_COUNTER) {
    const uint64_t cnt = (uint64_t)rd_int(p, o);
    const bool host = A.ncount[i] == kHostTier;
    uint64_t row = A.noff[i];
    uint64_t q = o;
    for (uint64_t j = 0; j < cnt; ++j) {
      const uint64_t id = (uint64_t)rd_int(p, q);
      const uint64_t v = (uint64_t)rd_int(p, q);
      const uint64_t t = (uint64_t)rd_int(p, q);
      aux += v;  // Counter::load_snapshot sums every value read (wrapping)
      if (host) continue;
      uint64_t r = q;
      bool later = false;
      for (uint64_t k = j + 1; k < cnt; ++k) {
        later |= (uint64_t)rd_int(p, r) == id;
        (void)rd_int(p, r);
        (void)rd_int(p, r);
      }
      if (later) continue;
      const uint64_t f[6] = {h.h, h.f, id, v, t, meta_pack(0, A.pos, row)};
      put_row<6>(A.nd, A.cs, row, f);
      ++row;
    }
  } else if ((hd.tag == TAG_SET || hd.tag == TAG_DICT) && A.mcount[i] != kHostTier) {
    const bool dict = hd.tag == TAG_DICT;
    const uint32_t na = (uint32_t)rd_int(p, o);
    uint64_t q = o;
    for (uint32_t j = 0; j < na; ++j) {
      (void)rd_span(p, q);
      (void)rd_int(p, q);
      if (dict) (void)rd_span(p, q);
    }
    const uint32_t nd = (uint32_t)rd_int(p, q);
    uint64_t keep;
    member_keep(p, o, dict, na, nd, &keep);
    uint64_t row = A.moff[i];
    q = o;
    for (uint32_t j = 0; j < na + nd; ++j) {
      if (j == na) (void)rd_int(p, q);
      const Span m = rd_span(p, q);
      const uint64_t t = (uint64_t)rd_int(p, q);
      Span v{0, 0};
      if (dict && j < na) v = rd_span(p, q);
      if (!((keep >> j) & 1)) continue;
      const Hash128 mh = hash_bytes(p + m.off, m.len, kDomainMember);
      const uint64_t f[6] = {h.h, h.f, mh.h, mh.f, t, meta_pack(j < na ? KIND_ADD : KIND_DEL, A.pos, row)};
      put_row<6>(A.mb, A.cs, row, f);
      A.mref[row] = make_ulonglong2(m.off, m.len);
      A.mvref[row] = make_ulonglong2(v.off, v.len);
      ++row;
    }
  }
  const uint64_t f[7] = {h.h, h.f, hd.ct, hd.ut, hd.dt, aux, meta_pack(hd.tag, A.pos, i)};
  put_row<7>(A.k, A.ks, kr, f);
  A.kref[i] = make_ulonglong2(hd.key.off, hd.key.len);
  A.vref[i] = make_ulonglong2(val.off, val.len);
}

// ---- key-hash order of a snapshot written from a merge result (decode_snapshots_gpu_device)
// A merge result is in key-hash order, and the writer emits its DATAS, EXPIRES and DELETES rows
// as three sections (server.rs:183-215 -> db.rs:122-136), each in that order. The device rows of
// such a snapshot are made ONE run of key rows -- the three sections merged by hash, DATAS first
// on ties, then EXPIRES -- so that the merge takes the sorted-run path. Its children already are
// one run each: they follow their DATAS entries.
//   key_hash_kernel : every entry's key hash (the first 8 bytes of what emit_kernel writes);
//   order_check     : a section that decreases somewhere sets the flag (no run: the merge then
//                     partitions these rows, as for a snapshot in the reference's HashMap order);
//   dest_kernel     : row of entry i = its index in its section + the rows of the other sections
//                     before it (binary searches: earlier sections count ties, later ones not).
__global__ void __launch_bounds__(kDecThreads) key_hash_kernel(DecArgs A, uint64_t* __restrict__ kh) {
  const uint64_t i = (uint64_t)blockIdx.x * kDecThreads + threadIdx.x;
  if (i >= A.n) return;
  uint64_t o = A.off[i];
  const Span key = rd_span(A.raw, o);  // every entry kind starts with its key
  kh[i] = hash_bytes(A.raw + key.off, key.len, kDomainKey).h;
}

struct Sections {
  uint64_t b[4];  // section s = entries [b[s], b[s + 1]): DATAS, EXPIRES, DELETES
};

// Grid-stride with a bounded grid, one flag update per wave at the end, skipped once the flag is
// set: a snapshot in HashMap order has a descent at every other entry, and one atomic per wave on
// the one flag word serialised ~500K atomics per 34M entries (6 ms).
__global__ void __launch_bounds__(kDecThreads) order_check_kernel(const uint64_t* __restrict__ kh, Sections S,
                                                                  unsigned long long* flag) {
  const uint64_t n = S.b[3];
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * kDecThreads + threadIdx.x; i + 1 < n && !bad;
       i += (uint64_t)gridDim.x * kDecThreads)
    bad = i + 1 != S.b[1] && i + 1 != S.b[2] && kh[i] > kh[i + 1];
  if (__ballot(bad) && (threadIdx.x & 63) == 0 && *(volatile unsigned long long*)flag == 0) atomicOr(flag, 1ull);
}

__device__ __forceinline__ uint64_t count_below(const uint64_t* kh, uint64_t lo, uint64_t hi, uint64_t v, bool ties) {
  uint64_t a = lo, b = hi;  // first row in [lo, hi) whose hash is > v (ties) or >= v (no ties)
  while (a < b) {
    const uint64_t m = (a + b) >> 1;
    if (ties ? kh[m] <= v : kh[m] < v) a = m + 1;
    else b = m;
  }
  return a - lo;
}

__global__ void __launch_bounds__(kDecThreads) dest_kernel(const uint64_t* __restrict__ kh, Sections S,
                                                           uint32_t* __restrict__ dest) {
  const uint64_t i = (uint64_t)blockIdx.x * kDecThreads + threadIdx.x;
  if (i >= S.b[3]) return;
  const int s = i < S.b[1] ? 0 : i < S.b[2] ? 1 : 2;
  const uint64_t v = kh[i];
  uint64_t r = i - S.b[s];
  for (int t = 0; t < 3; ++t)
    if (t != s) r += count_below(kh, S.b[t], S.b[t + 1], v, t < s);
  dest[i] = (uint32_t)r;
}

// ---- the entry index of a large DATAS section on the device
// The format has no sync marks: an entry starts where its predecessor ends. One wave takes a
// chunk of kIdxChunk bytes of the section and speculates, as the host threads of
// decode.cpp::parallel_datas do: the first offset of its chunk from which kIdxSync consecutive
// entries of at most 64 KB parse is taken as an entry start (a wrong offset rarely survives that
// many; the lanes try 64 offsets at a time, at most kIdxSyncTries of them, so a chunk inside one
// large entry gives up quickly), then lane 0 walks entries until one starts past the chunk. The
// host stitches the chains in order from the section start; a chunk whose sync point is not where
// the true chain enters it (or that has none) is walked again on the device from there, in rounds,
// and a last pass writes every offset of the true chain. The checks are the loader's
// (read_integer bounds, negative lengths, the tag byte), plus bounds no valid entry can exceed, so
// a chain the device accepts the host accepts too; any failure on the true chain hands the
// section back to the host index pass.
constexpr uint64_t kIdxChunk = 8192;
constexpr uint32_t kIdxSync = 16;
constexpr uint32_t kIdxSyncTries = 256;  // offsets tried per chunk (4 rounds of 64 lanes)
// The sync search bounds every length it meets by kIdxSyncEntryMax: a wrong offset often reads a
// huge member count or length, and one lane parsing thousands of bogus members held its whole wave
// (and, by the walks' serial order, the snapshot) for milliseconds. A chunk whose entries near its
// start are longer finds its sync later or not at all; the stitch re-walks it from the true chain.
constexpr uint64_t kIdxEntryMax = 1u << 10;
// The walk reads its chunk and the first kIdxTail bytes after it from LDS (one copy per wave).
constexpr uint64_t kIdxTail = 4096, kIdxWin = kIdxChunk + kIdxTail;
// Entries starting in one chunk: a DATAS entry takes at least 6 bytes (key length, three times,
// the tag, one payload length), so at most kIdxChunk / 6 + 1 start in a chunk.
constexpr uint32_t kIdxRelCap = (uint32_t)(kIdxChunk / 6 + 2);

// A cursor over the stream; bytes [wlo, wlo + wlen) come from an LDS copy (the walk's window),
// the rest from global memory.
struct DCur {
  const uint8_t* p;
  uint64_t n, off;
  const uint8_t* lds = nullptr;
  uint64_t wlo = 0, wlen = 0;
  __device__ __forceinline__ uint32_t at(uint64_t i) const {
    const uint64_t r = i - wlo;
    return r < wlen ? lds[r] : p[i];
  }
};
template <class Cur>
__device__ __forceinline__ bool dc_int(Cur& c, int64_t* v) {
  if (c.off >= c.n) return false;
  const uint32_t f = c.at(c.off++);
  const uint32_t sz = (f >> 6) == 0 ? 0 : (f >> 6) == 1 ? 1 : (f >> 6) == 2 ? 3 : 8;
  if (sz > c.n - c.off) return false;
  uint64_t x = sz == 8 ? 0 : (f & 0x3F);
  for (uint32_t i = 0; i < sz; ++i) x = (x << 8) | c.at(c.off + i);
  c.off += sz;
  *v = (int64_t)x;
  return true;
}
template <class Cur>
__device__ __forceinline__ bool dc_len(Cur& c, uint64_t* l) {
  int64_t v;
  if (!dc_int(c, &v) || v < 0) return false;
  *l = (uint64_t)v;
  return true;
}
template <class Cur>
__device__ __forceinline__ bool dc_span(Cur& c, uint64_t lim) {
  uint64_t l;
  if (!dc_len(c, &l) || l > c.n - c.off || l > lim) return false;
  c.off += l;
  return true;
}
// One DATAS entry (read_entry + the load_snapshot payloads), skipped; lim bounds every length.
template <class Cur>
__device__ bool dc_data_entry(Cur& c, uint64_t lim) {
  int64_t v;
  if (!dc_span(c, lim) || !dc_int(c, &v) || !dc_int(c, &v) || !dc_int(c, &v)) return false;
  if (c.off >= c.n) return false;
  const uint32_t tag = c.at(c.off++);
  uint64_t cnt;
  switch (tag) {
    case TAG_COUNTER:
      if (!dc_len(c, &cnt) || cnt > min(c.n - c.off, lim) / 3) return false;
      for (uint64_t i = 0; i < cnt; ++i)
        if (!dc_int(c, &v) || !dc_int(c, &v) || !dc_int(c, &v)) return false;
      return true;
    case TAG_BYTES:
      return dc_span(c, lim);
    case TAG_SET:
    case TAG_DICT: {
      const bool dict = tag == TAG_DICT;
      if (!dc_len(c, &cnt) || cnt > min(c.n - c.off, lim) / 2) return false;
      for (uint64_t i = 0; i < cnt; ++i)
        if (!dc_span(c, lim) || !dc_int(c, &v) || (dict && !dc_span(c, lim))) return false;
      if (!dc_len(c, &cnt) || cnt > min(c.n - c.off, lim) / 2) return false;
      for (uint64_t i = 0; i < cnt; ++i)
        if (!dc_span(c, lim) || !dc_int(c, &v)) return false;
      return true;
    }
    default:
      return false;
  }
}

struct IdxArgs {
  const uint8_t* raw;
  uint64_t n;          // stream length
  uint64_t S;          // the section's first entry
  uint32_t T;          // chunks: chunk t = [S + t kIdxChunk, S + (t + 1) kIdxChunk)
  uint64_t* sync;      // per chunk: the chain's first entry (~0: none found)
  uint32_t* count;     // per chunk: entries from sync until one starts past the chunk
  uint64_t* stop;      // per chunk: where the walk stopped (the first entry past it, or a failure)
  uint8_t* ok;         // per chunk: the walk reached the chunk end
  const uint64_t* tstart;  // record pass: the true chain's first entry in chunk t (~0: not on it)
  const uint64_t* tbase;   // record pass: index of that entry in the section
  const uint32_t* tcount;  // record pass: entries of the true chain in chunk t
  uint64_t* out;           // record pass: entry offsets
  uint16_t* rel;           // per chunk: the walked chain's entry offsets relative to the chunk start
                           // (kIdxRelCap slots per chunk; the record pass expands the true chain's)
};

// One wave per chunk, persistent over the chunks (a launch of one workgroup per 4 chunks spent its
// time dispatching workgroups that had little to do). list == null: the speculative pass over every
// chunk (sync search by the 64 lanes, then the walk by lane 0); else the nlist chunks of `list`,
// walked again by lane 0 from req[t] (the offset at which the true chain enters chunk t).
constexpr uint32_t kIdxWalkBlocks = 768;  // 3 workgroups of 4 waves per CU (48 KB of LDS each)
__global__ void __launch_bounds__(256) idx_walk_kernel(IdxArgs a, const uint64_t* __restrict__ req,
                                                       const uint32_t* __restrict__ list, uint32_t nlist) {
  __shared__ __attribute__((aligned(16))) uint8_t win_all[4][kIdxWin];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* win = win_all[wv];
  const uint32_t total = list ? nlist : a.T;
  for (uint32_t i = blockIdx.x * 4 + wv; i < total; i += gridDim.x * 4) {  // (wave-uniform)
    const uint32_t t = list ? list[i] : i;
    const uint64_t lo = a.S + (uint64_t)t * kIdxChunk, hi = min(a.n, lo + kIdxChunk);
    uint64_t o = list ? req[t] : lo;
    // the window: [lo16, lo16 + kIdxWin) with lo16 = lo rounded down to 16 B, copied in 16-B pieces
    // (a piece that starts before the end of the stream may read up to 15 bytes past it: the device
    // copy has 16 bytes of slack)
    const uint64_t lo16 = lo & ~15ull;
    const uint64_t wend = min(lo16 + kIdxWin, (a.n + 15) & ~15ull);
    __builtin_amdgcn_wave_barrier();  // (the previous chunk's readers are done with the window)
    for (uint64_t q = lo16 + 16ull * lane; q < wend; q += 16 * 64)
      *reinterpret_cast<uint4*>(win + (q - lo16)) = *reinterpret_cast<const uint4*>(a.raw + q);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const uint64_t wlen = min(wend, a.n) > lo16 ? min(wend, a.n) - lo16 : 0;
    if (!list && t > 0) {
      uint64_t found = ~0ull;
      for (uint32_t k = 0; k < kIdxSyncTries && found == ~0ull; k += 64) {  // (wave-uniform)
        const uint64_t at0 = lo + k + lane;
        bool ok = false;
        if (at0 < hi) {
          DCur s{a.raw, a.n, at0, win, lo16, wlen};
          uint32_t q = 0;
          for (; q < kIdxSync && s.off < a.n; ++q) {
            const uint64_t at = s.off;
            if (!dc_data_entry(s, kIdxEntryMax) || s.off - at > kIdxEntryMax) break;
          }
          ok = q == kIdxSync;
        }
        const uint64_t m = __ballot(ok);
        if (m) found = lo + k + __builtin_ctzll(m);
      }
      if (found == ~0ull) {
        if (lane == 0) {
          a.sync[t] = ~0ull;
          a.count[t] = 0;
          a.stop[t] = lo;
          a.ok[t] = 0;
        }
        continue;
      }
      o = found;
    }
    if (lane == 0) {
      DCur c{a.raw, a.n, o, win, lo16, wlen};
      uint16_t* rel = a.rel + (uint64_t)t * kIdxRelCap;
      uint32_t k = 0;
      bool good = true;
      while (c.off < hi) {
        const uint64_t at = c.off;
        if (k < kIdxRelCap) rel[k] = (uint16_t)(at - lo);
        if (!dc_data_entry(c, ~0ull)) {
          c.off = at;
          good = false;
          break;
        }
        ++k;
      }
      a.sync[t] = o;
      a.count[t] = k;
      a.stop[t] = c.off;
      a.ok[t] = good ? 1 : 0;
    }
  }
}

void idx_walk_launch(const IdxArgs& a, const uint64_t* req, const uint32_t* list, uint32_t n, hipStream_t s) {
  idx_walk_kernel<<<std::min<uint32_t>((n + 3) / 4, kIdxWalkBlocks), 256, 0, s>>>(a, req, list, n);
}

// Every offset of the true chain: chunk t's walk started where the chain enters it (the stitch
// re-walks every chunk for which that was not so), so its first tcount[t] relative offsets are the
// chain's. One wave per chunk, coalesced.
__global__ void __launch_bounds__(256) idx_record_kernel(IdxArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6); t < a.T; t += gridDim.x * 4) {
    if (a.tstart[t] == ~0ull) continue;
    const uint64_t lo = a.S + (uint64_t)t * kIdxChunk, b = a.tbase[t];
    const uint16_t* rel = a.rel + (uint64_t)t * kIdxRelCap;
    const uint32_t m = a.tcount[t];
    for (uint32_t k = lane; k < m; k += 64) a.out[b + k] = lo + rel[k];
  }
}

// Any entry left to the host tier (its count is the kHostTier marker)?
__global__ void host_tier_flag_kernel(const uint32_t* __restrict__ nc, const uint32_t* __restrict__ mc, uint64_t n,
                                      unsigned long long* flag) {
  bool any = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    any |= nc[i] == kHostTier || mc[i] == kHostTier;
  if (__ballot(any) && (threadIdx.x & 63) == 0) atomicOr(flag, 1ull);
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
struct EvPair {
  hipEvent_t a = nullptr, b = nullptr;
  EvPair() {
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
  }
  ~EvPair() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
  }
};

}  // namespace

// One snapshot through the GPU decode, in two steps so that several snapshots can be sized
// first and then emitted into one set of device columns (decode_snapshots_gpu_device):
//   prepare : the host index pass, the bytes to the device, the count pass, the stream
//             checksum, the host tier (entries past the per-thread dedup limits), child offsets;
//   emit_*  : the emit pass into the batch's host columns, or into caller device columns.
class GpuDecode {
 public:
  GpuDecode(cdb_ctx* ctx, Batch* out, uint32_t flags) : ctx_(ctx), out_(out), flags_(flags) {}
  int prepare(const uint8_t* buf, size_t len, size_t* err_off, DecodeTiming* tm) {
    const int rc = index(buf, len, err_off, tm);
    return rc != CDB_OK && rc != CDB_INVALID_SNAPSHOT_CHECKSUM ? rc : prepare_device(err_off);
  }
  // the host index pass (several snapshots are indexed on parallel threads). Its HIP calls -- the
  // early upload of a large snapshot and the page-lock of its bytes -- record their failures in
  // this object (st_); fail() serialises the context's last_error
  int index(const uint8_t* buf, size_t len, size_t* err_off, DecodeTiming* tm);
  // the device index of a deferred DATAS section in steps, so that the sections of several
  // snapshots are indexed side by side (decode_snapshots_gpu_device):
  //   dd_launch: the bytes up (context stream), the speculative walk and its results down on ks
  //              (-1: a HIP error, in st_);
  //   dd_step  : after ks: the stitch; another round of re-walks queued on ks (1), or finished (0:
  //              the record pass and the host pass resumed after the section; status in status())
  bool deferred() const { return cursor_ != nullptr; }
  int dd_launch(hipStream_t ks);
  int dd_step(size_t* err_off);
  int dd_host(size_t* err_off);
  int status() const { return st_ != CDB_OK ? (int)st_ : rc_; }
  // everything after it (returns the index pass's status when the device part succeeds)
  int prepare_device(size_t* err_off) {
    const int rc = prepare_launch(err_off);
    if (!prep_.pending) return rc;
    ck(hipStreamSynchronize(s_), "sync(decode)");
    return prepare_finish(err_off);
  }
  // ... in two halves, so that several snapshots' device work is queued before one
  // synchronisation: prepare_launch queues the bytes, counts, scans and checksum and the small
  // words' download (prepare_pending() then says prepare_finish must follow, after the context
  // stream is synchronised); prepare_finish reads them and does the rest
  // pin (may be null): page-locked room for side_bytes() bytes, untouched until the call's end
  int prepare_launch(size_t* err_off, uint8_t* pin = nullptr, uint64_t pin_room = 0);
  uint64_t side_bytes() const { return idx_.offset.size() * 9; }
  int prepare_finish(size_t* err_off);
  bool prepare_pending() const { return prep_.pending; }
  cdb_status emit_host(DecodeTiming* tm);
  cdb_status emit_device(uint64_t* const* k, uint64_t* const* nd, uint64_t* const* mb, uint32_t ks, uint32_t cs,
                         uint32_t pos, bool run, DecodeTiming* tm) {
    if (emit_launch(k, nd, mb, ks, cs, pos, run) != CDB_OK) return st_;
    if (!emit_pending_) return CDB_OK;
    ck(hipStreamSynchronize(s_), "sync(decode)");
    return emit_finish(tm);
  }
  // ... in two halves (several snapshots' emits queued before one synchronisation of the context
  // stream, then emit_finish for each when emit_pending())
  cdb_status emit_launch(uint64_t* const* k, uint64_t* const* nd, uint64_t* const* mb, uint32_t ks, uint32_t cs,
                         uint32_t pos, bool run);
  cdb_status emit_finish(DecodeTiming* tm);
  bool emit_pending() const { return emit_pending_; }
  // (several snapshots, records layout) the rows emitted into rows of the snapshot's own, right
  // after its preparation and sort, while later snapshots still cross PCIe (emit_own queues the
  // emit; emit_finish follows a later synchronisation); once every snapshot is counted, move_rows
  // copies them into the caller's columns at the snapshot's offsets (device copies on the context's
  // stream)
  cdb_status emit_own(uint32_t pos);
  bool emitted_own() const { return own_; }
  cdb_status move_rows(uint64_t* const* k, uint64_t* const* nd, uint64_t* const* mb);
  // key-hash order (after prepare_device): queues the key-hash pass and the sections' order check
  // on the context's stream; the verdict reads after a synchronisation (read_order).
  cdb_status order_check();
  bool read_order() const { return ordered_ && !(prep_.small && prep_.small[4]); }
  // a snapshot not in key-hash order (the reference's HashMap order) made ONE run anyway (after
  // read_order): its entries sorted by key hash on the device, children laid out in that order
  cdb_status sort_to_run();
  bool sorted() const { return sorted_; }
  uint64_t keys() const { return n_; }
  uint64_t nodes() const { return nn_; }
  uint64_t members() const { return nm_; }
  uint32_t index_threads_ = 1;  // threads of the host index pass's DATAS section
  double device_index_ms_ = 0;  // the DATAS section's device index + the resumed host pass

 private:
  struct HostEntry {
    uint64_t i;
    Batch rows;
    uint64_t total;
  };
  void ck(hipError_t e, const char* what) {
    if (e != hipSuccess && st_ == CDB_OK) st_ = hip_check(ctx_, e, what);
  }
  static bool host_register(void* p, size_t bytes) {  // false: not locked, and no pending HIP error
    if (hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess) return true;
    (void)hipGetLastError();
    return false;
  }
  cdb_status alloc(void** p, size_t bytes, const char* what) {  // reported, no pending HIP error
    if (hipMalloc(p, bytes) == hipSuccess) return CDB_OK;
    (void)hipGetLastError();
    *p = nullptr;
    return fail(ctx_, CDB_OUT_OF_MEMORY, what);
  }
  // byte references straight into the batch (pairs as written by the emit pass), then the host
  // tier's member references
  cdb_status refs_to_batch(const DecArgs& A);
  // a deferred DATAS section: its entries indexed on the device, then the host pass resumed after
  // it (or, where the device gives up, the host pass over the whole stream)
  int finish_index(size_t* err_off);
  void dd_download();
  int dd_done(int dv, uint64_t end, size_t* err_off);
  struct DevIndex {
    hipStream_t ks = nullptr;
    bool active = false;
    uint32_t T = 0;
    int round = 0;
    IdxArgs a;
    uint64_t* d_req = nullptr;
    uint32_t* d_list = nullptr;  // re-walk rounds: the requested chunks
    std::vector<uint32_t> list;
    uint64_t last = 0;  // the section's last entry
    DevBuf work, offs;
    EvPair up;  // (a: the snapshot's bytes are on the device)
    std::vector<uint64_t> sync, stop, req;
    std::vector<uint32_t> count;
    std::vector<uint8_t> ok;
    std::chrono::steady_clock::time_point t0;
  } di_;

  cdb_ctx* ctx_;
  Batch* out_;
  uint32_t flags_;
  cdb_status st_ = CDB_OK;
  int rc_ = CDB_OK;
  hipStream_t s_ = nullptr;
  EntryIndex idx_;
  DeferredCrc dcrc_;
  uint64_t n_ = 0, nn_ = 0, nm_ = 0;
  std::vector<uint64_t> noff_, moff_;
  std::vector<HostEntry> hosted_;
  DevBuf d_raw_, d_meta_, d_crc_, d_rows_, d_ord_;
  uint64_t raw_front_ = 0;  // the deferred index uploaded the bytes to d_raw_ + raw_front_
  bool early_up_ = false;   // the index pass queued that upload (from the caller's buffer, or chunked)
 public:
  // The early uploads of a call's snapshots, one after another across their streams (each waits on
  // the one issued before it), so that the first snapshots land -- and their walks run -- while
  // the later ones still cross PCIe.
  struct UpChain {
    std::mutex mu;
    hipEvent_t last = nullptr;
  };
  UpChain* chain_ = nullptr;
  bool early_upload() const { return early_up_; }
 private:
 public:
  hipStream_t up_s_ = nullptr;  // (several snapshots) this snapshot's own stream: the chunked upload
 private:
  // A snapshot over 512 MB: copied into the batch's huge pages in chunks, each chunk page-locked
  // and uploaded on up_s_ as soon as it is copied, so PCIe works while the host copies. False:
  // nothing queued (the call then takes the batch-copy path).
  bool chunked_upload(const uint8_t* buf, size_t len);
  bool pre_chunked_ = false;  // pre_upload() did the chunked upload: index() goes straight to its pass
 public:
  // A snapshot over 512 MB: its chunked copy and upload ahead of (and on another thread than) its
  // host index pass, so that pass overlaps the next snapshot's copy and upload.
  void pre_upload(const uint8_t* buf, size_t len) {
    if (buf && len > (size_t(512) << 20) && up_s_ && hipSetDevice(ctx_->device) == hipSuccess)
      pre_chunked_ = chunked_upload(buf, len);
  }
 private:
  bool emit_pending_ = false;  // emit_launch -> emit_finish
  bool own_ = false;           // emit_own: the rows are in own_rows_ (records: hash column + records)
  DevBuf own_rows_;
  uint64_t* own_k_[kKeyCols] = {};
  uint64_t* own_n_[kNodeCols] = {};
  uint64_t* own_m_[kMemberCols] = {};
  struct HostReg {  // page-locked ranges of the snapshot's bytes (unlocked at the end of the call)
    void* p = nullptr;
    std::vector<void*> more;   // the chunks of a chunked upload
    hipStream_t s = nullptr;   // the stream an upload from them was queued on
    void release() {
      if (!p && more.empty()) return;
      // an upload may still read them when the call ends early (an index pass failed after it
      // was queued): wait for it before the pages are unlocked
      if (s) (void)hipStreamSynchronize(s);
      if (p) (void)hipHostUnregister(p);
      for (void* q : more) (void)hipHostUnregister(q);
      (void)hipGetLastError();
      p = nullptr;
      more.clear();
    }
    ~HostReg() { release(); }
  } reg_;
  uint64_t raw_pad_ = 0;  // d_raw_ + raw_pad_ = byte 0 of the snapshot
 public:
  double lt_[4] = {0, 0, 0, 0};  // dd_launch host time (ms): bytes buffer, upload call, scratch, walk launch
 private:
  DeferredDatas defer_;
  IndexCursor* cursor_ = nullptr;
  struct CursorFree {
    IndexCursor** p;
    ~CursorFree() {
      if (*p) index_cursor_free(*p);
    }
  } cursor_free_{&cursor_};
  uint64_t dev_datas_ = 0;  // leading entries (the DATAS section) whose offsets are only in di_.offs
  bool ordered_ = false;  // the sections are contiguous, in DATAS, EXPIRES, DELETES order
  bool sorted_ = false;   // sort_to_run placed the rows: sort_dest_ is every entry's key row
  uint32_t* sort_dest_ = nullptr;
  DevBuf d_sort_;
  Sections sec_{};
  DecArgs A_;
  uint32_t grid_ = 0;
  EvPair ev_;
  struct PrepState {  // prepare_launch -> prepare_finish
    bool pending = false;
    uint64_t dd = 0, n = 0;
    uint64_t *d_off = nullptr, *d_noff = nullptr, *d_moff = nullptr;
    uint32_t *d_ncnt = nullptr, *d_mcnt = nullptr;
    uint64_t* small = nullptr;  // page-locked words (downloads stay asynchronous): crc | node rows |
                                // member rows | host-tier flag | order flag
    ~PrepState() {
      if (small) (void)hipHostFree(small);
    }
  } prep_;
};

int GpuDecode::index(const uint8_t* buf, size_t len, size_t* err_off, DecodeTiming* tm) {
  const auto t0 = std::chrono::steady_clock::now();
  // A large snapshot's bytes go up at once, from the caller's buffer (page-locked for the call),
  // while this thread copies them into the batch and indexes them: the DMA no longer waits for
  // the host index passes (the walk waits on di_.up.a; prepare_device finds them in d_raw_).
  // CDB_H2D_STAGED=1: through the staging ring after the index pass instead.
  // Up to 512 MB: page-locking the caller's buffer (small pages) costs little; beyond, locking
  // 8 x 2 GB of it took 444 ms of host index time against 179 for the batch's huge-page copy
  // (the C4 shard's decode leg: 935 vs 789 ms), so those take the batch copy after the pass.
  static const bool staged = std::getenv("CDB_H2D_STAGED") != nullptr;
  // (a failed page-lock -- a buffer the caller already locked, a read-only mapping, the same bytes
  // passed twice -- falls back silently: its error is cleared so that no later check reports it)
  if (!staged && buf && len >= (size_t(64) << 20) && len <= (size_t(512) << 20) &&
      hipSetDevice(ctx_->device) == hipSuccess &&
      host_register(const_cast<uint8_t*>(buf), len)) {
    reg_.p = const_cast<uint8_t*>(buf);
    hipStream_t us = up_s_ ? up_s_ : ctx_->stream;  // (its walk queues behind it on the same stream)
    reg_.s = us;
    const uint64_t front = crc_tile_bytes();
    if ((st_ = alloc(&d_raw_.p, front + len + 16, "decode: device buffer for the snapshot bytes")) != CDB_OK)
      return st_;
    raw_front_ = front;
    {
      std::unique_lock<std::mutex> lk;
      if (chain_) {
        lk = std::unique_lock<std::mutex>(chain_->mu);
        if (chain_->last) ck(hipStreamWaitEvent(us, chain_->last, 0), "wait(upload chain)");
      }
      ck(hipMemcpyAsync((uint8_t*)d_raw_.p + front, buf, len, hipMemcpyHostToDevice, us), "h2d(index)");
      ck(hipEventRecord(di_.up.a, us), "event(index)");
      if (chain_) chain_->last = di_.up.a;
    }
    if (st_ != CDB_OK) return st_;
    early_up_ = true;
  }
  const bool chunked = pre_chunked_ || (!early_up_ && !staged && buf && len > (size_t(512) << 20) && up_s_ &&
                                        hipSetDevice(ctx_->device) == hipSuccess && chunked_upload(buf, len));
  if (st_ != CDB_OK) return st_;
  // (chunked: the bytes are in the batch already)
  rc_ = index_snapshot(chunked ? nullptr : buf, len, flags_, out_, &idx_, err_off, &dcrc_, index_threads_, &defer_,
                       &cursor_);
  if (rc_ == kIndexDeferred) rc_ = CDB_OK;  // the DATAS section is indexed in prepare_device
  // otherwise a deferred section's snapshot goes up whole right after: page-lock the batch's bytes
  // here, on this thread (the index passes of several snapshots run side by side, and so do the
  // page-locks; one after another they cost as much as the uploads)
  if (!early_up_ && !staged && cursor_ && out_->raw.size() >= (size_t(64) << 20) &&
      hipSetDevice(ctx_->device) == hipSuccess && host_register(out_->raw.data(), out_->raw.size())) {
    reg_.p = out_->raw.data();
    reg_.s = ctx_->stream;
  }
  if (tm) tm->index_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc_;
}

bool GpuDecode::chunked_upload(const uint8_t* buf, size_t len) {
  Batch* b = out_;
  b->raw.resize(len);  // default-initialised
  advise_huge(b->raw.data(), len);
  const uint64_t front = crc_tile_bytes();
  if ((st_ = alloc(&d_raw_.p, front + len + 16, "decode: device buffer for the snapshot bytes")) != CDB_OK)
    return false;
  uint8_t* const raw = b->raw.data();
  uint8_t* const dst = (uint8_t*)d_raw_.p + front;
  // chunk boundaries at 64 MB-aligned addresses: no two page-locked ranges share a page
  constexpr uintptr_t kChunk = uintptr_t(64) << 20;
  const uintptr_t base = (uintptr_t)raw;
  reg_.s = up_s_;
  bool ok = true;
  for (size_t a = 0; a < len;) {
    const size_t e = std::min<size_t>(len, ((base + a + kChunk) & ~(kChunk - 1)) - base);
    parallel_copy(raw + a, buf + a, e - a);
    if (ok && host_register(raw + a, e - a)) {
      reg_.more.push_back(raw + a);
      ok = hipMemcpyAsync(dst + a, raw + a, e - a, hipMemcpyHostToDevice, up_s_) == hipSuccess;
      if (!ok) (void)hipGetLastError();
    } else {
      ok = false;  // (the rest is only copied)
    }
    a = e;
  }
  if (!ok) {  // a chunk could not be locked or queued: nothing of it is used
    reg_.release();
    (void)hipFree(d_raw_.p);
    d_raw_.p = nullptr;
    return true;  // (the bytes are in the batch)
  }
  raw_front_ = front;
  ck(hipEventRecord(di_.up.a, up_s_), "event(index)");
  early_up_ = st_ == CDB_OK;
  return true;
}

int GpuDecode::dd_launch(hipStream_t ks) {
  DevIndex& d = di_;
  d.t0 = std::chrono::steady_clock::now();
  d.ks = ks;
  const uint64_t len = out_->raw.size(), S = defer_.start;
  hipStream_t s = ctx_->stream;
  auto lap = [t = std::chrono::steady_clock::now()](double* acc) mutable {
    const auto now = std::chrono::steady_clock::now();
    *acc += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  };
  // the bytes go to their final place: one CRC tile of room in front, so prepare_device zero-fills
  // the checksum's leading pad there instead of moving the stream
  if (!early_up_) {  // (else the index pass started the upload)
    const uint64_t front = crc_tile_bytes();
    if ((st_ = alloc(&d_raw_.p, front + len + 16, "decode: device buffer for the snapshot bytes")) != CDB_OK)
      return -1;
    raw_front_ = front;
  }
  uint8_t* const dst = (uint8_t*)d_raw_.p + raw_front_;
  lap(&lt_[0]);
  // bytes page-locked by the index pass go up directly (no second host copy through the staging
  // ring, and this thread does not wait for the upload)
  if (early_up_) {
  } else if (reg_.p) {
    ck(hipMemcpyAsync(dst, out_->raw.data(), len, hipMemcpyHostToDevice, s), "h2d(index)");
    if (st_ != CDB_OK) return -1;
  } else if ((st_ = staged_h2d(ctx_, dst, out_->raw.data(), len, s)) != CDB_OK) {
    return -1;
  }
  if (!early_up_) ck(hipEventRecord(d.up.a, s), "event(index)");
  ck(hipStreamWaitEvent(ks, d.up.a, 0), "wait(index)");
  lap(&lt_[1]);
  const uint32_t T = d.T = (uint32_t)((len - S + kIdxChunk - 1) / kIdxChunk);
  const size_t wbytes = (size_t)T * (8 + 4 + 8 + 1 + 8 + 8 + 4 + 8) + 64 + (size_t)T * kIdxRelCap * 2 + 16 + (size_t)T * 4;
  if ((st_ = alloc(&d.work.p, wbytes, "decode: device entry index scratch")) != CDB_OK) return -1;
  lap(&lt_[2]);
  IdxArgs& a = d.a;
  std::memset(&a, 0, sizeof a);
  a.raw = dst;
  a.n = len;
  a.S = S;
  a.T = T;
  uint8_t* w = (uint8_t*)d.work.p;
  a.sync = (uint64_t*)w;
  a.stop = a.sync + T;
  uint64_t* d_tstart = a.stop + T;
  uint64_t* d_tbase = d_tstart + T;
  d.d_req = d_tbase + T;
  a.count = (uint32_t*)(d.d_req + T);
  uint32_t* d_tcount = a.count + T;
  a.ok = (uint8_t*)(d_tcount + T);
  a.rel = (uint16_t*)(((uintptr_t)(a.ok + T) + 15) & ~(uintptr_t)15);
  d.d_list = (uint32_t*)(a.rel + (size_t)T * kIdxRelCap);
  a.tstart = d_tstart;
  a.tbase = d_tbase;
  a.tcount = d_tcount;
  d.sync.assign(T, 0);
  d.stop.assign(T, 0);
  d.req.assign(T, ~0ull);
  d.count.assign(T, 0);
  d.ok.assign(T, 0);
  d.round = 0;
  idx_walk_launch(a, nullptr, nullptr, T, ks);
  ck(hipGetLastError(), "idx_walk_kernel");
  lap(&lt_[3]);
  d.active = true;
  return st_ == CDB_OK ? 0 : -1;
}

void GpuDecode::dd_download() {  // the walk's results to the host (after the walk: see dd_step)
  DevIndex& d = di_;
  const uint32_t T = d.T;
  ck(hipMemcpyAsync(d.sync.data(), d.a.sync, T * 8ull, hipMemcpyDeviceToHost, d.ks), "d2h(index)");
  ck(hipMemcpyAsync(d.stop.data(), d.a.stop, T * 8ull, hipMemcpyDeviceToHost, d.ks), "d2h(index)");
  ck(hipMemcpyAsync(d.count.data(), d.a.count, T * 4ull, hipMemcpyDeviceToHost, d.ks), "d2h(index)");
  ck(hipMemcpyAsync(d.ok.data(), d.a.ok, T, hipMemcpyDeviceToHost, d.ks), "d2h(index)");
}

// 1: another round of device walks is queued on ks; 2: the section's offsets are in idx_, the host
// part (dd_host: the host pass resumed after the section) remains; 0: finished (status() holds
// the outcome: the index pass's status, as finish_index returns it).
int GpuDecode::dd_step(size_t* err_off) {
  DevIndex& d = di_;
  if (!d.active) return 0;
  // the walk's results come down only now: a copy into pageable host memory queued behind the walk
  // would hold the launching thread until the walk ends (and with it every later snapshot's launch)
  ck(hipStreamSynchronize(d.ks), "sync(index)");
  dd_download();
  ck(hipStreamSynchronize(d.ks), "sync(index)");
  if (st_ != CDB_OK) return dd_done(-1, 0, err_off);
  const uint64_t len = out_->raw.size(), S = defer_.start, cnt = defer_.count;
  const uint32_t T = d.T;
  // stitch: the true chain from the section start, chunk by chunk. A chunk whose sync point is not
  // where the chain enters it (a spurious sync inside an entry's bytes, or none found) is walked
  // again on the device from there; past the first such chunk the chain is speculative (each
  // chunk's own chain, which usually joins the true one, so later chunks keep theirs), and rounds
  // repeat until every chunk on the chain starts where the chain enters it.
  bool consistent = true;
  std::fill(d.req.begin(), d.req.end(), ~0ull);
  {
    uint64_t cur = S, got = 0;
    bool lost = false;  // the speculative chain has no entry point here: adopt the chunk's own
    for (uint32_t t = 0; t < T && got < cnt; ++t) {
      const uint64_t hi = std::min<uint64_t>(len, S + (uint64_t)(t + 1) * kIdxChunk);
      if (!lost && cur >= hi) continue;  // an entry spans the whole chunk
      const uint64_t need = cnt - got;
      if (lost) {
        if (d.sync[t] == ~0ull) continue;
        lost = false;
      } else if (d.sync[t] != cur) {
        d.req[t] = cur;
        consistent = false;
        if (d.sync[t] == ~0ull) {
          lost = true;
          continue;
        }
      } else if (!d.ok[t] && d.count[t] < need) {
        // the chain fails inside the section: on the true chain (every chunk so far consistent)
        // the host pass reports it; after a re-walk request it is a speculative chain, so the
        // round ends here and the next one resumes from the re-walked chunks
        if (consistent) return dd_done(1, 0, err_off);
        break;
      }
      got += std::min<uint64_t>(d.count[t], need);
      cur = d.stop[t];
    }
  }
  if (!consistent) {
    if (++d.round >= 16) return dd_done(1, 0, err_off);  // (3-4 rounds on the generator's streams)
    d.list.clear();
    for (uint32_t t = 0; t < T; ++t)
      if (d.req[t] != ~0ull) d.list.push_back(t);
    const uint32_t nl = (uint32_t)d.list.size();
    ck(hipMemcpyAsync(d.d_req, d.req.data(), T * 8ull, hipMemcpyHostToDevice, d.ks), "h2d(index)");
    ck(hipMemcpyAsync(d.d_list, d.list.data(), nl * 4ull, hipMemcpyHostToDevice, d.ks), "h2d(index)");
    idx_walk_launch(d.a, d.d_req, d.d_list, nl, d.ks);
    ck(hipGetLastError(), "idx_walk_kernel");
    return st_ == CDB_OK ? 1 : dd_done(-1, 0, err_off);
  }
  std::vector<uint64_t> tstart(T, ~0ull), tbase(T, 0);
  std::vector<uint32_t> tcount(T, 0);
  uint64_t got = 0;
  {
    uint64_t cur = S;
    for (uint32_t t = 0; t < T && got < cnt; ++t) {
      const uint64_t hi = std::min<uint64_t>(len, S + (uint64_t)(t + 1) * kIdxChunk);
      if (cur >= hi) continue;
      const uint32_t m = (uint32_t)std::min<uint64_t>(d.count[t], cnt - got);
      if (m > kIdxRelCap) return dd_done(1, 0, err_off);  // (no valid entry is that short)
      tstart[t] = cur;
      tbase[t] = got;
      tcount[t] = m;
      got += m;
      cur = d.stop[t];
    }
  }
  if (got < cnt) return dd_done(1, 0, err_off);  // the stream ends inside the section
  // every offset of the true chain, written on the device, then into the host index
  ck(hipMemcpyAsync((void*)d.a.tstart, tstart.data(), T * 8ull, hipMemcpyHostToDevice, d.ks), "h2d(index)");
  ck(hipMemcpyAsync((void*)d.a.tbase, tbase.data(), T * 8ull, hipMemcpyHostToDevice, d.ks), "h2d(index)");
  ck(hipMemcpyAsync((void*)d.a.tcount, tcount.data(), T * 4ull, hipMemcpyHostToDevice, d.ks), "h2d(index)");
  // the offsets stay on the device (prepare_device copies them into place); the host needs only
  // the last one (where the section ends) unless an entry falls to the host tier
  if ((st_ = alloc(&d.offs.p, cnt * 8, "decode: device entry offsets")) != CDB_OK) return dd_done(-1, 0, err_off);
  d.a.out = (uint64_t*)d.offs.p;
  idx_record_kernel<<<std::min<uint32_t>((T + 3) / 4, 2048), 256, 0, d.ks>>>(d.a);
  ck(hipGetLastError(), "idx_record_kernel");
  ck(hipMemcpyAsync(&d.last, d.a.out + (cnt - 1), 8, hipMemcpyDeviceToHost, d.ks), "d2h(index)");
  ck(hipStreamSynchronize(d.ks), "sync(index)");  // (the host vectors above are copy sources)
  if (st_ != CDB_OK) return dd_done(-1, 0, err_off);
  return 2;  // the host part (dd_host) is left to the caller: several snapshots run it side by side
}

int GpuDecode::dd_host(size_t* err_off) {
  uint64_t end = 0;
  if (!index_data_entry_end(*out_, di_.last, &end)) return dd_done(1, 0, err_off);
  return dd_done(0, end, err_off);
}

// dv 0: the section's offsets are in idx_, the host pass resumes at `end`; 1: the device gave up,
// the host index pass runs over the whole stream; -1: a HIP error (st_).
int GpuDecode::dd_done(int dv, uint64_t end, size_t* err_off) {
  DevIndex& d = di_;
  d.active = false;
  // (the walk's scratch is freed with this object, at the end of the call: a hipFree waits for the
  // device, and while later snapshots upload and walk that wait stalls every thread's HIP calls)
  if (dv == 0) {  // the section's offsets on the device, the side sections' on the host after them
    idx_.offset.clear();
    idx_.kind.clear();
    rc_ = index_resume(cursor_, end, err_off);  // EXPIRES, DELETES, the checksum
    dev_datas_ = defer_.count;
  } else if (dv > 0) {
    if (d.offs.p) (void)hipFree(d.offs.p);
    d.offs.p = nullptr;  // the host index pass over the whole stream: its statuses and offsets
    if (up_s_) (void)hipStreamSynchronize(up_s_);  // (a chunked upload may still write d_raw_)
    if (d_raw_.p) (void)hipFree(d_raw_.p);
    d_raw_.p = nullptr;
    raw_front_ = 0;
    idx_ = EntryIndex{};
    dcrc_ = DeferredCrc{};
    *out_ = Batch{std::move(out_->raw)};
    rc_ = index_snapshot(nullptr, out_->raw.size(), flags_, out_, &idx_, err_off, &dcrc_, index_threads_);
  }
  index_cursor_free(cursor_);
  cursor_ = nullptr;
  device_index_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d.t0).count();
  return 0;
}

int GpuDecode::finish_index(size_t* err_off) {
  if (!cursor_) return rc_;
  if (hipSetDevice(ctx_->device) != hipSuccess) return fail(ctx_, CDB_DEVICE_ERROR, "hipSetDevice");
  if (!di_.active && dd_launch(ctx_->stream) < 0) {
    dd_done(-1, 0, err_off);
    return st_;
  }
  int r;
  while ((r = dd_step(err_off)) == 1) {
  }
  if (r == 2) dd_host(err_off);
  return st_ != CDB_OK ? st_ : rc_;
}

int GpuDecode::prepare_launch(size_t* err_off, uint8_t* pin, uint64_t pin_room) {
  prep_.pending = false;
  if (cursor_) {
    const int rc = finish_index(err_off);
    if (rc != CDB_OK && rc != CDB_INVALID_SNAPSHOT_CHECKSUM) return rc;
  }
  const uint64_t len = out_->raw.size();
  const uint64_t dd = dev_datas_, n = n_ = dd + idx_.offset.size();
  if (n == 0) return rc_;
  if (hipSetDevice(ctx_->device) != hipSuccess) return CDB_DEVICE_ERROR;
  hipStream_t s = s_ = ctx_->stream;
  if (early_up_) ck(hipStreamWaitEvent(s, di_.up.a, 0), "wait(decode)");  // (an upload on another stream)
  // the raw stream sits after `pad` zero bytes, so the checksummed prefix ends on a CRC tile
  const uint64_t tile = crc_tile_bytes();
  const uint64_t pad = dcrc_.pending ? (tile - dcrc_.len % tile) % tile : 0;
  // (the deferred DATAS index already put the bytes on the device, raw_front_ bytes into d_raw_)
  if (!raw_front_ && (st_ = alloc(&d_raw_.p, pad + len + 16, "decode: device buffer for the snapshot bytes")) != CDB_OK)
    return st_;
  raw_pad_ = raw_front_ ? raw_front_ : pad;
  uint8_t* const crc_base = (uint8_t*)d_raw_.p + raw_pad_ - pad;  // pad zero bytes, then the stream
  // small device words: crc | node-row total | member-row total | host-tier flag
  if ((st_ = alloc(&d_crc_.p, 32, "decode: device checksum word")) != CDB_OK) return st_;
  uint64_t* d_small = (uint64_t*)d_crc_.p;
  // one device block: off | noff | moff | ncount | mcount | kind | scan partials
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  const size_t head = n * (8 + 1 + 4 + 4 + 8 + 8) + 16 * tiles + 64;
  if ((st_ = alloc(&d_meta_.p, head, "decode: device entry index")) != CDB_OK) return st_;
  uint8_t* hm = (uint8_t*)d_meta_.p;
  uint64_t* d_off = (uint64_t*)hm;
  uint64_t* d_noff = d_off + n;
  uint64_t* d_moff = d_noff + n;
  uint64_t* d_sums = d_moff + n;  // 2 x tiles
  uint32_t* d_ncnt = (uint32_t*)(d_sums + 2 * tiles);
  uint32_t* d_mcnt = d_ncnt + n;
  uint8_t* d_kind = (uint8_t*)(d_mcnt + n);
  ck(hipEventRecord(ev_.a, s), "event");
  if (pad) ck(hipMemsetAsync(crc_base, 0, pad, s), "memset(decode)");
  ck(hipMemsetAsync(d_small, 0, 32, s), "memset(decode)");
  const uint8_t* raw_dev = (const uint8_t*)d_raw_.p + raw_pad_;
  if (st_ == CDB_OK && !raw_front_) st_ = staged_h2d(ctx_, (void*)raw_dev, out_->raw.data(), len, s);
  if (dd) {  // the DATAS section's offsets from the device index, then the side sections'
    ck(hipMemcpyAsync(d_off, di_.offs.p, dd * 8, hipMemcpyDeviceToDevice, s), "d2d(decode)");
    ck(hipMemsetAsync(d_kind, 0, dd, s), "memset(decode)");
  }
  if (pin && (n - dd) * 9 <= pin_room) {  // page-locked room of the caller's: no staging-ring waits
    std::memcpy(pin, idx_.offset.data(), (n - dd) * 8);
    std::memcpy(pin + (n - dd) * 8, idx_.kind.data(), n - dd);
    ck(hipMemcpyAsync(d_off + dd, pin, (n - dd) * 8, hipMemcpyHostToDevice, s), "h2d(decode)");
    ck(hipMemcpyAsync(d_kind + dd, pin + (n - dd) * 8, n - dd, hipMemcpyHostToDevice, s), "h2d(decode)");
  } else {
    if (st_ == CDB_OK) st_ = staged_h2d(ctx_, d_off + dd, idx_.offset.data(), (n - dd) * 8, s);
    ck(hipMemcpyAsync(d_kind + dd, idx_.kind.data(), n - dd, hipMemcpyHostToDevice, s), "h2d(decode)");
  }
  if (st_ != CDB_OK) return st_;
  std::memset(&A_, 0, sizeof A_);
  A_.raw = raw_dev;
  A_.off = d_off;
  A_.kind = d_kind;
  A_.n = n;
  A_.ncount = d_ncnt;
  A_.mcount = d_mcnt;
  A_.noff = d_noff;
  A_.moff = d_moff;
  grid_ = (uint32_t)((n + kDecThreads - 1) / kDecThreads);
  count_kernel<<<grid_, kDecThreads, 0, s>>>(A_);
  ck(hipGetLastError(), "count_kernel");
  // the child offsets: exclusive scans of the counts on the device (they are only meaningful
  // when no entry is left to the host tier, which the flag reports)
  host_tier_flag_kernel<<<(uint32_t)std::min<uint64_t>(grid_, 1024), kDecThreads, 0, s>>>(d_ncnt, d_mcnt, n,
                                                                                         (unsigned long long*)d_small + 3);
  ck(hipGetLastError(), "host_tier_flag_kernel");
  scan_reduce_kernel<uint32_t><<<(uint32_t)tiles, kScanThreads, 0, s>>>(d_ncnt, n, d_sums);
  scan_sums_kernel<<<1, kScanThreads, 0, s>>>(d_sums, tiles, d_small + 1);
  scan_apply_kernel<uint32_t, uint64_t><<<(uint32_t)tiles, kScanThreads, 0, s>>>(d_ncnt, n, d_sums, d_noff,
                                                                               (uint64_t*)nullptr);
  scan_reduce_kernel<uint32_t><<<(uint32_t)tiles, kScanThreads, 0, s>>>(d_mcnt, n, d_sums + tiles);
  scan_sums_kernel<<<1, kScanThreads, 0, s>>>(d_sums + tiles, tiles, d_small + 2);
  scan_apply_kernel<uint32_t, uint64_t><<<(uint32_t)tiles, kScanThreads, 0, s>>>(d_mcnt, n, d_sums + tiles, d_moff,
                                                                               (uint64_t*)nullptr);
  ck(hipGetLastError(), "decode scans");
  if (dcrc_.pending && st_ == CDB_OK)  // the index pass left the stream checksum to the GPU
    st_ = crc64_device_queued(ctx_, crc_base, pad + dcrc_.len, d_small, s);
  if (!prep_.small && st_ == CDB_OK) ck(hipHostMalloc((void**)&prep_.small, 48, hipHostMallocDefault), "host alloc(decode)");
  if (st_ != CDB_OK) return st_;
  ck(hipMemcpyAsync(prep_.small, d_small, 32, hipMemcpyDeviceToHost, s), "d2h(decode)");
  if (st_ != CDB_OK) return st_;
  prep_.pending = true;
  prep_.dd = dd;
  prep_.n = n;
  prep_.d_off = d_off;
  prep_.d_noff = d_noff;
  prep_.d_moff = d_moff;
  prep_.d_ncnt = d_ncnt;
  prep_.d_mcnt = d_mcnt;
  return rc_;
}

int GpuDecode::prepare_finish(size_t* err_off) {
  prep_.pending = false;
  if (st_ != CDB_OK) return st_;
  const hipStream_t s = s_;
  const uint64_t dd = prep_.dd, n = prep_.n;
  uint64_t* const d_off = prep_.d_off;
  uint64_t* const d_noff = prep_.d_noff;
  uint64_t* const d_moff = prep_.d_moff;
  uint32_t* const d_ncnt = prep_.d_ncnt;
  uint32_t* const d_mcnt = prep_.d_mcnt;
  const uint64_t* small = prep_.small;
  if (dcrc_.pending && small[0] != dcrc_.got) {
    rc_ = CDB_INVALID_SNAPSHOT_CHECKSUM;
    *err_off = dcrc_.err_off;
  }
  if (!small[3]) {  // every entry's children were counted on the device (offs: freed with the object)
    nn_ = small[1];
    nm_ = small[2];
    return rc_;
  }
  if (dd) {  // the host tier re-parses entries by offset: every offset on the host
    std::vector<uint64_t> all(n);
    ck(hipMemcpyAsync(all.data(), d_off, n * 8, hipMemcpyDeviceToHost, s), "d2h(decode)");
    ck(hipStreamSynchronize(s), "sync(decode)");
    if (st_ != CDB_OK) return st_;
    std::vector<uint8_t> kinds(dd, 0);
    kinds.insert(kinds.end(), idx_.kind.begin(), idx_.kind.end());
    idx_.offset.swap(all);
    idx_.kind.swap(kinds);
    dev_datas_ = 0;
  }
  // entries past the per-thread dedup limits: decoded here, into slots reserved by a host scan
  noff_.resize(n);
  moff_.resize(n);
  std::vector<uint32_t> ncnt(n), mcnt(n);
  ck(hipMemcpyAsync(ncnt.data(), d_ncnt, n * 4, hipMemcpyDeviceToHost, s), "d2h(decode)");
  ck(hipMemcpyAsync(mcnt.data(), d_mcnt, n * 4, hipMemcpyDeviceToHost, s), "d2h(decode)");
  ck(hipStreamSynchronize(s), "sync(decode)");
  if (st_ != CDB_OK) return st_;
  for (uint64_t i = 0; i < n; ++i) {
    if (ncnt[i] != kHostTier && mcnt[i] != kHostTier) continue;
    HostEntry he;
    he.i = i;
    uint64_t o = idx_.offset[i];
    // the key's hash, as decode.cpp computes it
    const uint8_t* p = out_->raw.data();
    auto rint = [&](uint64_t& q) {
      const uint32_t f = p[q++];
      uint64_t v = f & 0x3F;
      const int extra = (f >> 6) == 0 ? 0 : (f >> 6) == 1 ? 1 : (f >> 6) == 2 ? 3 : 8;
      if (extra == 8) v = 0;
      for (int k = 0; k < extra; ++k) v = (v << 8) | p[q++];
      return v;
    };
    uint64_t q = o;
    const uint64_t klen = rint(q);
    const Hash128 h = hash_bytes(p + q, klen, kDomainKey);
    if (!decode_entry_children(*out_, o, h.h, h.f, &he.rows, &he.total))
      return st_ = fail(ctx_, CDB_DEVICE_ERROR, "decode: host tier could not re-parse an indexed entry");
    if (ncnt[i] == kHostTier) ncnt[i] = (uint32_t)he.rows.n_pkh.size();
    if (mcnt[i] == kHostTier) mcnt[i] = (uint32_t)he.rows.m_pkh.size();
    hosted_.push_back(std::move(he));
  }
  for (uint64_t i = 0; i < n; ++i) {
    noff_[i] = nn_;
    moff_[i] = nm_;
    nn_ += ncnt[i];
    nm_ += mcnt[i];
  }
  // (the emit pass still sees the host tier's markers in the device copies of the counts)
  if (st_ == CDB_OK) st_ = staged_h2d(ctx_, d_noff, noff_.data(), n * 8, s);
  if (st_ == CDB_OK) st_ = staged_h2d(ctx_, d_moff, moff_.data(), n * 8, s);
  return st_ != CDB_OK ? (int)st_ : rc_;
}


cdb_status GpuDecode::refs_to_batch(const DecArgs& A) {
  static_assert(sizeof(ByteRef) == sizeof(ulonglong2), "byte references download as (offset, length) pairs");
  Batch& b = *out_;
  b.key_ref.resize(n_);
  b.val_ref.resize(n_);
  b.m_ref.resize(nm_);
  b.m_vref.resize(nm_);
  advise_huge(b.key_ref.data(), n_ * sizeof(ByteRef));  // (fresh pages, first touched by the download)
  advise_huge(b.val_ref.data(), n_ * sizeof(ByteRef));
  advise_huge(b.m_ref.data(), nm_ * sizeof(ByteRef));
  advise_huge(b.m_vref.data(), nm_ * sizeof(ByteRef));
  std::vector<HostSeg> segs;
  auto down = [&](void* host, const ulonglong2* dev, uint64_t rows) {
    if (rows) segs.push_back({host, const_cast<ulonglong2*>(dev), rows * 16});
  };
  down(b.key_ref.data(), A.kref, n_);
  down(b.val_ref.data(), A.vref, n_);
  down(b.m_ref.data(), A.mref, nm_);
  down(b.m_vref.data(), A.mvref, nm_);
  if (!segs.empty() && (st_ = staged_copy(ctx_, segs.data(), segs.size(), false, s_)) != CDB_OK) return st_;
  for (const HostEntry& he : hosted_) {
    const Batch& r = he.rows;
    for (size_t j = 0; j < r.m_pkh.size(); ++j) {
      b.m_ref[moff_[he.i] + j] = r.m_ref[j];
      b.m_vref[moff_[he.i] + j] = r.m_vref[j];
    }
  }
  return CDB_OK;
}

DeviceRefs::~DeviceRefs() {
  if (!dev && !raw) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(device);
  if (dev) (void)hipFree(dev);
  if (raw) (void)hipFree(raw);
  (void)hipSetDevice(cur);
}

cdb_status refs_ready(cdb_ctx* ctx, Batch* b) {
  std::shared_ptr<DeviceRefs> r = b->dev_refs;
  if (!r) return CDB_OK;
  std::lock_guard<std::mutex> lock(r->mu);
  if (!r->dev) return CDB_OK;  // (another caller downloaded them)
  if (!ctx) return CDB_BAD_ARGUMENT;
  if (ctx->device != r->device) return fail(ctx, CDB_BAD_ARGUMENT, "byte references live on another device");
  (void)hipSetDevice(ctx->device);
  const uint64_t n = r->n, nm = r->nm;
  const ByteRef* d = (const ByteRef*)r->dev;
  RefVec* dst[4] = {&b->key_ref, &b->val_ref, &b->m_ref, &b->m_vref};
  const uint64_t rows[4] = {n, n, nm, nm};
  const ByteRef* src[4] = {d, d + n, d + 2 * n, d + 2 * n + nm};
  std::vector<HostSeg> segs;
  for (int c = 0; c < 4; ++c) {
    dst[c]->resize(rows[c]);
    advise_huge(dst[c]->data(), rows[c] * sizeof(ByteRef));  // (fresh pages, first touched by the download)
    if (rows[c]) segs.push_back({dst[c]->data(), const_cast<ByteRef*>(src[c]), rows[c] * sizeof(ByteRef)});
  }
  cdb_status st = segs.empty() ? CDB_OK : staged_copy(ctx, segs.data(), segs.size(), false, ctx->stream);
  if (st != CDB_OK) {
    for (int c = 0; c < 4; ++c) dst[c]->clear();
    return st;
  }
  for (const DeviceRefs::Patch& p : r->patch) {
    b->m_ref[p.row] = p.m;
    b->m_vref[p.row] = p.mv;
  }
  (void)hipFree(r->dev);
  r->dev = nullptr;
  r->patch.clear();
  return CDB_OK;
}

cdb_status GpuDecode::emit_host(DecodeTiming* tm) {
  if (n_ == 0) return CDB_OK;
  const uint64_t n = n_, nn = nn_, nm = nm_;
  hipStream_t s = s_;
  const size_t rows_words = n * 11 + nn * 6 + nm * 10 + 8;
  if ((st_ = alloc(&d_rows_.p, rows_words * 8, "decode: device row columns")) != CDB_OK) return st_;
  uint64_t* w = (uint64_t*)d_rows_.p;
  DecArgs& A = A_;
  uint64_t* const w0 = w;
  auto align16 = [&]() { w += (w - w0) & 1; };  // reference pairs are 16-B stores
  for (int c = 0; c < 7; ++c, w += n) A.k[c] = w;
  A.ks = A.cs = 1;  // (the host batch's columns)
  align16();
  A.kref = (ulonglong2*)w; w += 2 * n;
  A.vref = (ulonglong2*)w; w += 2 * n;
  for (int c = 0; c < 6; ++c, w += nn) A.nd[c] = w;
  for (int c = 0; c < 6; ++c, w += nm) A.mb[c] = w;
  align16();
  A.mref = (ulonglong2*)w; w += 2 * nm;
  A.mvref = (ulonglong2*)w; w += 2 * nm;
  A.pos = 0;
  emit_kernel<<<grid_, kDecThreads, 0, s>>>(A);
  ck(hipGetLastError(), "emit_kernel");
  if (st_ != CDB_OK) return st_;
  // rows back into the host batch: one staged download of every column
  Batch& b = *out_;
  std::vector<HostSeg> segs;
  auto down = [&](ColVec* v, const uint64_t* dev, uint64_t rows) {
    v->resize(rows);  // default-initialised: the download overwrites every word
    advise_huge(v->data(), rows * 8);
    if (rows) segs.push_back({v->data(), const_cast<uint64_t*>(dev), rows * 8});
  };
  ColVec* kc[7] = {&b.kh, &b.kf, &b.ct, &b.ut, &b.dt, &b.aux, &b.meta};
  for (int c = 0; c < 7; ++c) down(kc[c], A.k[c], n);
  ColVec* nc[6] = {&b.n_pkh, &b.n_pkf, &b.n_node, &b.n_v, &b.n_t, &b.n_meta};
  ColVec* mc[6] = {&b.m_pkh, &b.m_pkf, &b.m_h, &b.m_f, &b.m_t, &b.m_meta};
  for (int c = 0; c < 6; ++c) {
    down(nc[c], A.nd[c], nn);
    down(mc[c], A.mb[c], nm);
  }
  if ((st_ = staged_copy(ctx_, segs.data(), segs.size(), false, s)) != CDB_OK) return st_;
  if ((st_ = refs_to_batch(A)) != CDB_OK) return st_;
  ck(hipEventRecord(ev_.b, s), "event");
  ck(hipStreamSynchronize(s), "sync(decode)");
  if (st_ != CDB_OK) return st_;
  if (tm) {
    float ms = 0;
    hipEventElapsedTime(&ms, ev_.a, ev_.b);
    tm->device_ms = ms;
  }
  // the host tier's children, src fields made absolute
  for (const HostEntry& he : hosted_) {
    const Batch& r = he.rows;
    for (size_t j = 0; j < r.n_pkh.size(); ++j) {
      const uint64_t row = noff_[he.i] + j;
      b.n_pkh[row] = r.n_pkh[j];
      b.n_pkf[row] = r.n_pkf[j];
      b.n_node[row] = r.n_node[j];
      b.n_v[row] = r.n_v[j];
      b.n_t[row] = r.n_t[j];
      b.n_meta[row] = meta_pack(0, 0, row);
    }
    for (size_t j = 0; j < r.m_pkh.size(); ++j) {
      const uint64_t row = moff_[he.i] + j;
      b.m_pkh[row] = r.m_pkh[j];
      b.m_pkf[row] = r.m_pkf[j];
      b.m_h[row] = r.m_h[j];
      b.m_f[row] = r.m_f[j];
      b.m_t[row] = r.m_t[j];
      b.m_meta[row] = meta_pack(meta_tag(r.m_meta[j]), 0, row);
    }
  }
  return CDB_OK;
}

cdb_status GpuDecode::order_check() {
  ordered_ = false;
  if (!prep_.small) ck(hipHostMalloc((void**)&prep_.small, 48, hipHostMallocDefault), "host alloc(decode)");
  if (st_ != CDB_OK) return st_;
  prep_.small[4] = 0;  // the order flag (written by the download queued below)
  const uint64_t n = n_;
  if (n == 0) {
    ordered_ = true;
    return CDB_OK;
  }
  if (n >= (1ull << 32)) return CDB_OK;
  const uint64_t dd = dev_datas_;  // (leading DATAS entries whose kinds are not on the host)
  uint64_t cnt[3] = {dd, 0, 0};
  uint8_t prev = 0;
  for (uint64_t i = dd; i < n; ++i) {
    const uint8_t k = idx_.kind[i - dd];
    if (k < prev || k > 2) return CDB_OK;  // sections out of the writer's order: no run
    prev = k;
    ++cnt[k];
  }
  sec_.b[0] = 0;
  sec_.b[1] = cnt[0];
  sec_.b[2] = cnt[0] + cnt[1];
  sec_.b[3] = n;
  if ((st_ = alloc(&d_ord_.p, n * 12 + 64, "decode: key-hash order scratch")) != CDB_OK) return st_;
  uint64_t* kh = (uint64_t*)d_ord_.p;
  unsigned long long* flag = (unsigned long long*)(kh + n);
  ck(hipMemsetAsync(flag, 0, 8, s_), "memset(decode order)");
  key_hash_kernel<<<grid_, kDecThreads, 0, s_>>>(A_, kh);
  ck(hipGetLastError(), "key_hash_kernel");
  order_check_kernel<<<std::min<uint32_t>(grid_, 2048), kDecThreads, 0, s_>>>(kh, sec_, flag);
  ck(hipGetLastError(), "order_check_kernel");
  ck(hipMemcpyAsync(prep_.small + 4, flag, 8, hipMemcpyDeviceToHost, s_), "d2h(decode order)");
  ordered_ = st_ == CDB_OK;
  return st_;
}

// ---- a snapshot in the reference's HashMap order made one run (sort_to_run)
// perm: sorted position -> entry. dest[entry] = its key row; the children counts in sorted order.
__global__ void __launch_bounds__(kDecThreads) sort_perm_kernel(const uint32_t* __restrict__ perm, uint64_t n,
                                                                const uint32_t* __restrict__ ncnt,
                                                                const uint32_t* __restrict__ mcnt,
                                                                uint32_t* __restrict__ dest, uint32_t* __restrict__ ns,
                                                                uint32_t* __restrict__ ms) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t e = perm[j];
    dest[e] = (uint32_t)j;
    ns[j] = ncnt[e];
    ms[j] = mcnt[e];
  }
}
// every entry's first child rows: the scans in sorted order, back to entry order
__global__ void __launch_bounds__(kDecThreads) sort_off_kernel(const uint32_t* __restrict__ perm, uint64_t n,
                                                               const uint64_t* __restrict__ nso,
                                                               const uint64_t* __restrict__ mso,
                                                               uint64_t* __restrict__ noff, uint64_t* __restrict__ moff) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t e = perm[j];
    noff[e] = nso[j];
    moff[e] = mso[j];
  }
}
// After a stable sort on the top 32 key-hash bits: every run of equal top halves (a few entries --
// a key's DATAS / EXPIRES / DELETES entries, or a 2^-32 coincidence) is insertion-sorted on the
// whole hash by the thread at its first position, stably, so the pairs end in the order the full
// 64-bit stable sort gives.
__global__ void __launch_bounds__(kDecThreads) sort_low_fixup_kernel(uint64_t* __restrict__ k, uint32_t* __restrict__ v,
                                                                     uint64_t n) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j + 1 < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t hi = k[j] >> 32;
    if ((k[j + 1] >> 32) != hi || (j > 0 && (k[j - 1] >> 32) == hi)) continue;  // not a run's first
    uint64_t e = j + 2;
    while (e < n && (k[e] >> 32) == hi) ++e;
    for (uint64_t a = j + 1; a < e; ++a) {
      const uint64_t x = k[a];
      const uint32_t y = v[a];
      uint64_t b = a;
      while (b > j && k[b - 1] > x) {
        k[b] = k[b - 1];
        v[b] = v[b - 1];
        --b;
      }
      k[b] = x;
      v[b] = y;
    }
  }
}
__global__ void __launch_bounds__(kDecThreads) iota32_kernel(uint32_t* __restrict__ v, uint64_t n) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x)
    v[j] = (uint32_t)j;
}

// The reference dumps its DB by iterating a HashMap (db.rs:122-136), so a peer running it sends
// DATAS, EXPIRES and DELETES in no key order. Such a snapshot still becomes ONE sorted run: a stable
// sort of (key hash, entry) pairs over all its entries (4 radix passes on the top 32 bits, then the
// few runs of equal top halves insertion-sorted on the whole hash; equal hashes keep stream order,
// so DATAS precede EXPIRES precede DELETES, as dest_kernel orders a hash-ordered
// snapshot), then every entry's key row is its sorted position and its children are laid out in
// that order (the count scans redone in sorted order). Entries left to the host tier keep the
// snapshot in stream order (no run).
cdb_status GpuDecode::sort_to_run() {
  sorted_ = false;
  const uint64_t n = n_;
  if (!ordered_ || !hosted_.empty() || n < 2 || n >= (1ull << 32)) return CDB_OK;
  uint64_t* kh = (uint64_t*)d_ord_.p;
  uint32_t* dest = (uint32_t*)(kh + n + 8);
  if ((st_ = alloc(&d_sort_.p, n * (8 + 4 + 4 + 4 + 4 + 8 + 8) + 64, "decode: key-hash sort scratch")) != CDB_OK)
    return st_;
  uint64_t* k2 = (uint64_t*)d_sort_.p;
  uint64_t* nso = k2 + n;
  uint64_t* mso = nso + n;
  uint32_t* v = (uint32_t*)(mso + n);
  uint32_t* v2 = v + n;
  uint32_t* ns = v2 + n;
  uint32_t* ms = ns + n;
  const uint32_t g = (uint32_t)std::min<uint64_t>(grid_, 4096);
  iota32_kernel<<<g, kDecThreads, 0, s_>>>(v, n);
  ck(hipGetLastError(), "iota32_kernel");
  uint64_t* kk = kh;
  uint32_t* vv = v;
  // (4 passes on the top half, then the equal-top runs fixed up: the 8-pass sort's order)
  if (st_ == CDB_OK) st_ = radix_sort_pairs(ctx_, &kk, &vv, k2, v2, n, 32, 64, s_);
  if (st_ != CDB_OK) return st_;
  sort_low_fixup_kernel<<<g, kDecThreads, 0, s_>>>(kk, vv, n);
  ck(hipGetLastError(), "sort_low_fixup_kernel");
  sort_perm_kernel<<<g, kDecThreads, 0, s_>>>(vv, n, A_.ncount, A_.mcount, dest, ns, ms);
  ck(hipGetLastError(), "sort_perm_kernel");
  if (st_ == CDB_OK) st_ = exclusive_scan_u32(ctx_, ns, n, nso, nullptr, s_);
  if (st_ == CDB_OK) st_ = exclusive_scan_u32(ctx_, ms, n, mso, nullptr, s_);
  if (st_ != CDB_OK) return st_;
  sort_off_kernel<<<g, kDecThreads, 0, s_>>>(vv, n, nso, mso, (uint64_t*)A_.noff, (uint64_t*)A_.moff);
  ck(hipGetLastError(), "sort_off_kernel");
  sort_dest_ = dest;
  sorted_ = st_ == CDB_OK;
  return st_;
}

// Host-decoded child rows [at, at + n) of a 6-field family into device rows: one upload per column,
// or (records, stride s) the hash column and the interleaved records.
template <typename Val>
static void up_rows(std::vector<ColVec>& up, std::vector<HostSeg>& segs, uint64_t* const* dst, uint32_t s,
                    uint64_t at, uint64_t n, Val&& val) {
  if (s <= 1) {
    for (int c = 0; c < 6; ++c) {
      up.emplace_back(n);
      ColVec& v = up.back();
      for (uint64_t j = 0; j < n; ++j) v[j] = val(c, j);
      segs.push_back({v.data(), dst[c] + at, n * 8});
    }
    return;
  }
  up.emplace_back(n);
  for (uint64_t j = 0; j < n; ++j) up.back()[j] = val(0, j);
  segs.push_back({up.back().data(), dst[0] + at, n * 8});
  up.emplace_back(n * s);
  ColVec& r = up.back();
  for (uint64_t j = 0; j < n; ++j)
    for (int c = 1; c < 6; ++c) r[j * s + (c - 1)] = val(c, j);
  segs.push_back({r.data(), dst[1] + at * s, n * s * 8});
}

cdb_status GpuDecode::emit_launch(uint64_t* const* k, uint64_t* const* nd, uint64_t* const* mb, uint32_t ks,
                                  uint32_t cs, uint32_t pos, bool run) {
  emit_pending_ = false;
  out_->rows_on_device = true;
  out_->dev_rows[0] = n_;
  out_->dev_rows[1] = nn_;
  out_->dev_rows[2] = nm_;
  if (n_ == 0) return CDB_OK;
  const uint64_t n = n_, nn = nn_, nm = nm_;
  hipStream_t s = s_;
  // the byte references only: the rows go to the caller's columns
  const size_t ref_words = n * 4 + nm * 4 + 8;
  if ((st_ = alloc(&d_rows_.p, ref_words * 8, "decode: device byte references")) != CDB_OK) return st_;
  uint64_t* w = (uint64_t*)d_rows_.p;
  DecArgs& A = A_;
  for (int c = 0; c < 7; ++c) A.k[c] = k[c];
  for (int c = 0; c < 6; ++c) {
    A.nd[c] = nd[c];
    A.mb[c] = mb[c];
  }
  A.kref = (ulonglong2*)w; w += 2 * n;
  A.vref = (ulonglong2*)w; w += 2 * n;
  A.mref = (ulonglong2*)w; w += 2 * nm;
  A.mvref = (ulonglong2*)w; w += 2 * nm;
  A.pos = pos;
  A.ks = ks;
  A.cs = cs;
  A.dest = nullptr;
  if (run && sorted_) {
    A.dest = sort_dest_;
  } else if (run && n > 1 && sec_.b[1] != n) {  // side sections to merge into the DATAS order
    const uint64_t* kh = (const uint64_t*)d_ord_.p;
    uint32_t* dest = (uint32_t*)(kh + n + 8);
    dest_kernel<<<grid_, kDecThreads, 0, s>>>(kh, sec_, dest);
    ck(hipGetLastError(), "dest_kernel");
    A.dest = dest;
  }
  emit_kernel<<<grid_, kDecThreads, 0, s>>>(A);
  ck(hipGetLastError(), "emit_kernel");
  if (st_ != CDB_OK) return st_;
  // the host tier's children go up into their reserved rows
  std::vector<ColVec> up;
  up.reserve(hosted_.size() * 12);
  std::vector<HostSeg> segs;
  for (const HostEntry& he : hosted_) {
    const Batch& r = he.rows;
    const uint64_t nr = r.n_pkh.size(), mr = r.m_pkh.size();
    if (nr) {
      const ColVec* src[6] = {&r.n_pkh, &r.n_pkf, &r.n_node, &r.n_v, &r.n_t, nullptr};
      auto val = [&](int c, uint64_t j) { return c < 5 ? (*src[c])[j] : meta_pack(0, pos, noff_[he.i] + j); };
      up_rows(up, segs, nd, cs, noff_[he.i], nr, val);
    }
    if (mr) {
      const ColVec* src[6] = {&r.m_pkh, &r.m_pkf, &r.m_h, &r.m_f, &r.m_t, nullptr};
      auto val = [&](int c, uint64_t j) {
        return c < 5 ? (*src[c])[j] : meta_pack(meta_tag(r.m_meta[j]), pos, moff_[he.i] + j);
      };
      up_rows(up, segs, mb, cs, moff_[he.i], mr, val);
    }
  }
  if (!segs.empty() && (st_ = staged_copy(ctx_, segs.data(), segs.size(), true, s)) != CDB_OK) return st_;
  ck(hipEventRecord(ev_.b, s), "event");
  if (st_ != CDB_OK) return st_;
  emit_pending_ = true;
  return CDB_OK;
}

cdb_status GpuDecode::emit_own(uint32_t pos) {
  const uint64_t n = n_, nn = nn_, nm = nm_;
  auto words = [](uint64_t rows, int nc) { return ((rows + 2 + 1) & ~1ull) + (((rows * (nc - 1)) + 2 + 1) & ~1ull); };
  const uint64_t w = words(n, kKeyCols) + words(nn, kNodeCols) + words(nm, kMemberCols);
  if ((st_ = alloc(&own_rows_.p, w * 8 + 64, "decode: the snapshot's own device rows")) != CDB_OK) return st_;
  uint64_t* q = (uint64_t*)(((uintptr_t)own_rows_.p + 15) & ~(uintptr_t)15);
  auto lay = [&](uint64_t** col, uint64_t rows, int nc) {  // the records layout of cdb_dev_rows
    col[0] = q;
    q += (rows + 2 + 1) & ~1ull;
    for (int c = 1; c < nc; ++c) col[c] = q + (c - 1);
    q += ((rows * (nc - 1)) + 2 + 1) & ~1ull;
  };
  lay(own_k_, n, kKeyCols);
  lay(own_n_, nn, kNodeCols);
  lay(own_m_, nm, kMemberCols);
  // (the snapshot alone decides its row order: a run if it is one; the merge takes the rows of
  // every snapshot in any order when not all of them are runs)
  if (emit_launch(own_k_, own_n_, own_m_, kKeyCols - 1, kNodeCols - 1, pos, sorted_ || read_order()) != CDB_OK)
    return st_;
  own_ = st_ == CDB_OK;  // (emit_finish after the caller's next synchronisation of the stream)
  return st_;
}

cdb_status GpuDecode::move_rows(uint64_t* const* k, uint64_t* const* nd, uint64_t* const* mb) {
  const hipStream_t s = s_ ? s_ : ctx_->stream;
  auto mv = [&](uint64_t* const* dst, uint64_t* const* src, uint64_t rows, int nc) {
    if (!rows) return;
    ck(hipMemcpyAsync(dst[0], src[0], rows * 8, hipMemcpyDeviceToDevice, s), "d2d(decode rows)");
    ck(hipMemcpyAsync(dst[1], src[1], rows * (nc - 1) * 8, hipMemcpyDeviceToDevice, s), "d2d(decode rows)");
  };
  mv(k, own_k_, n_, kKeyCols);
  mv(nd, own_n_, nn_, kNodeCols);
  mv(mb, own_m_, nm_, kMemberCols);
  return st_;
}

cdb_status GpuDecode::emit_finish(DecodeTiming* tm) {
  emit_pending_ = false;
  if (st_ != CDB_OK) return st_;
  const uint64_t n = n_, nn = nn_, nm = nm_;
  if (tm) {
    float ms = 0;
    hipEventElapsedTime(&ms, ev_.a, ev_.b);
    tm->device_ms = ms;
  }
  // the byte references stay in HBM until the canonical dump or the encoder asks (refs_ready)
  auto r = std::make_shared<DeviceRefs>();
  r->device = ctx_->device;
  r->n = n;
  r->nm = nm;
  for (const HostEntry& he : hosted_) {
    const Batch& hr = he.rows;
    for (size_t j = 0; j < hr.m_pkh.size(); ++j) r->patch.push_back({moff_[he.i] + j, hr.m_ref[j], hr.m_vref[j]});
  }
  r->dev = d_rows_.p;
  d_rows_.p = nullptr;
  if (flags_ & CDB_DECODE_KEEP_BYTES) {
    r->raw = d_raw_.p;
    r->raw_off = raw_pad_;
    d_raw_.p = nullptr;
  }
  out_->dev_refs = std::move(r);
  (void)nn;
  return CDB_OK;

}

uint32_t host_index_threads() {
  static const uint32_t t = [] {
    const char* e = std::getenv("CDB_INDEX_THREADS");
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    return e ? (uint32_t)std::max(1, std::atoi(e)) : std::min(16u, hw);
  }();
  return t;
}

int decode_snapshot_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint32_t flags, Batch* out, size_t* err_off,
                        DecodeTiming* tm) {
  GpuDecode d(ctx, out, flags);
  d.index_threads_ = host_index_threads();
  const int rc = d.prepare(buf, len, err_off, tm);
  if (rc != CDB_OK && rc != CDB_INVALID_SNAPSHOT_CHECKSUM) return rc;
  const cdb_status st = d.emit_host(tm);
  return st != CDB_OK ? (int)st : rc;
}

namespace {
struct PhaseClock {
  const char* path = std::getenv("CDB_DECODE_TRACE");
  std::chrono::steady_clock::time_point last;
  std::string json;
  explicit PhaseClock(std::chrono::steady_clock::time_point t0) : last(t0) {}
  void mark(const char* name) {
    if (!path) return;
    const auto now = std::chrono::steady_clock::now();
    char b[96];
    std::snprintf(b, sizeof b, "%s\"%s_ms\": %.3f", json.empty() ? "" : ", ", name,
                  std::chrono::duration<double, std::milli>(now - last).count());
    json += b;
    last = now;
  }
  void add(const char* key, const std::vector<double>& v) {
    if (!path) return;
    std::string a;
    for (double x : v) {
      char b[32];
      std::snprintf(b, sizeof b, "%s%.3f", a.empty() ? "" : ", ", x);
      a += b;
    }
    json += std::string(json.empty() ? "" : ", ") + "\"" + key + "\": [" + a + "]";
  }
  void write(uint32_t n, uint64_t bytes, const uint64_t* rows, bool runs) {
    if (!path) return;
    if (FILE* f = std::fopen(path, "a")) {
      std::fprintf(f, "{\"snapshots\": %u, \"bytes\": %llu, \"rows\": [%llu, %llu, %llu], \"runs\": %d, %s}\n", n,
                   (unsigned long long)bytes, (unsigned long long)rows[0], (unsigned long long)rows[1],
                   (unsigned long long)rows[2], runs ? 1 : 0, json.c_str());
      std::fclose(f);
    }
  }
};
}  // namespace

int decode_snapshots_gpu_device(cdb_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, uint32_t n,
                                uint32_t flags, Batch* const* outs, cdb_dev_input* din, uint32_t* failed,
                                size_t* err_off, DecodeTiming* tm) {
  const auto t_start = std::chrono::steady_clock::now();
  GpuDecode::UpChain up_chain;  // (outlives the decoders that point at it)
  std::vector<std::unique_ptr<GpuDecode>> dec;
  int rc_all = CDB_OK;
  uint64_t tot[3] = {0, 0, 0};
  // the sequential host index passes of the snapshots run side by side (one thread each, at most
  // 16 at once); their statuses are then taken in snapshot order, as one pass after another would
  std::vector<int> irc(n, CDB_OK);
  std::vector<size_t> ieo(n, 0);
  // every snapshot's own stream (kept in the context): its chunked upload, then its walks
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CDB_DEVICE_ERROR, "hipSetDevice");
  if (ctx->idx_streams.size() < n) ctx->idx_streams.resize(n, nullptr);
  for (uint32_t i = 0; i < n; ++i)
    if (!ctx->idx_streams[i]) {
      const cdb_status st = hip_check(ctx, hipStreamCreateWithFlags(&ctx->idx_streams[i], hipStreamNonBlocking),
                                      "stream(index)");
      if (st != CDB_OK) return st;
    }
  for (uint32_t i = 0; i < n; ++i) {
    dec.emplace_back(new GpuDecode(ctx, outs[i], flags));
    // several snapshots are indexed side by side: a few split their DATAS sections over their
    // share of the threads; 8 snapshots measured faster unsplit (271 vs 311 ms in all)
    dec.back()->index_threads_ = n <= 4 ? std::max(1u, host_index_threads() / std::max(1u, n)) : 1u;
    dec.back()->up_s_ = ctx->idx_streams[i];
    dec.back()->chain_ = &up_chain;
  }
  // the deferred DATAS sections: every snapshot's bytes go up with its speculative walk queued
  // behind them on its own stream; the stitch rounds then run per snapshot (below, or on the
  // after-walk thread)
  std::vector<hipStream_t> ks(n, nullptr);
  std::vector<uint32_t> live;
  // launch(i): snapshot i's walk, after its index pass. True: its stitch rounds remain (dd_step)
  auto launch = [&](uint32_t i) {
    if ((irc[i] != CDB_OK && irc[i] != CDB_INVALID_SNAPSHOT_CHECKSUM) || !dec[i]->deferred()) return false;
    ks[i] = ctx->idx_streams[i];
    if (dec[i]->dd_launch(ks[i]) < 0) {
      (void)dec[i]->dd_step(&ieo[i]);
      irc[i] = dec[i]->status();
      return false;
    }
    return true;
  };
  // Snapshots over 512 MB, one after another: copied into their batches by every host thread and
  // uploaded chunk by chunk on their own streams (GpuDecode::chunked_upload), indexed, and their
  // walks launched at once, so the walk of snapshot i runs while snapshot i + 1 crosses PCIe (side
  // by side, every upload ended near the last one and the walks queued behind them). What follows
  // a walk -- the stitch rounds, the host pass resumed after the section, the device preparation
  // (counts, checksum), the order check and the key-hash sort -- runs for such a snapshot on the
  // after-walk thread, in snapshot order, while later snapshots still cross PCIe; it alone uses the
  // context's stream until it is joined. The other snapshots are indexed side by side, one thread
  // each, and take the steps below.
  static const bool staged = std::getenv("CDB_H2D_STAGED") != nullptr;
  std::vector<char> seq(n, 0);
  std::vector<int> prc(n, CDB_OK), erc(n, CDB_OK);
  std::vector<size_t> peo(n, 0);
  {
    // two stages, each a thread taking snapshots in order from its queue: the walk stage (stitch
    // rounds on the snapshot's stream, the host pass resumed after the section) hands each snapshot
    // to the device stage (preparation, order check, sort, emit on the context's stream), so one
    // snapshot's host pass overlaps the previous one's device work
    struct Queue {
      std::mutex mu;
      std::condition_variable cv;
      std::deque<uint32_t> q;
      bool closed = false;
      void push(uint32_t i) {
        {
          std::lock_guard<std::mutex> lk(mu);
          q.push_back(i);
        }
        cv.notify_one();
      }
      void close() {
        {
          std::lock_guard<std::mutex> lk(mu);
          closed = true;
        }
        cv.notify_one();
      }
      bool pop(uint32_t* i) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return closed || !q.empty(); });
        if (q.empty()) return false;
        *i = q.front();
        q.pop_front();
        return true;
      }
    } walked, launched_q;
    // the host pass resumed after a walked section runs on a thread of its own per snapshot (they
    // take 15-20 ms each on C4's snapshots: in line they held back the next snapshot's stitch)
    std::vector<std::thread> resume(n);
    auto walk_stage = [&]() {
      (void)hipSetDevice(ctx->device);
      for (uint32_t i; launched_q.pop(&i);) {
        GpuDecode& d = *dec[i];
        if (d.deferred()) {
          int r;
          while ((r = d.dd_step(&ieo[i])) == 1) {
          }
          if (r == 2) {
            resume[i] = std::thread([&, i] {
              (void)hipSetDevice(ctx->device);
              dec[i]->dd_host(&ieo[i]);
              irc[i] = dec[i]->status();
            });
          } else {
            irc[i] = d.status();
          }
        }
        walked.push(i);
      }
      walked.close();
    };
    auto device_stage = [&]() {
      (void)hipSetDevice(ctx->device);
      for (uint32_t i; walked.pop(&i);) {
        if (resume[i].joinable()) resume[i].join();
        GpuDecode& d = *dec[i];
        peo[i] = ieo[i];
        int rc = irc[i];
        if (rc == CDB_OK || rc == CDB_INVALID_SNAPSHOT_CHECKSUM) rc = d.prepare_launch(&peo[i]);
        // the order check is queued behind the preparation: one synchronisation reads both
        const bool ordered = d.prepare_pending() && n <= CDB_MAX_RUNS && d.order_check() == CDB_OK;
        if (d.prepare_pending()) {
          if (hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync(decode)") != CDB_OK) rc = CDB_DEVICE_ERROR;
          else rc = d.prepare_finish(&peo[i]);
        }
        prc[i] = rc;
        if ((rc != CDB_OK && rc != CDB_INVALID_SNAPSHOT_CHECKSUM) || !ordered)
          continue;  // (the order and the sort are taken again below, where an error is reported)
        if (!d.read_order() && !(flags & CDB_DECODE_STREAM_ORDER) && d.sort_to_run() != CDB_OK) continue;
        // the emit is queued, not waited for: its finish runs after the call's last synchronisation
        if (flags & CDB_DECODE_ROWS_RECORDS) erc[i] = d.emit_own(i);
      }
    };
    std::thread walk_th(walk_stage), device_th(device_stage);
    // snapshots over 512 MB: this thread copies and uploads them one after another; a thread of
    // their own runs each one's host index pass (and launches its walk) as soon as its bytes are
    // in the batch, while the next one copies and uploads
    Queue uploaded;
    std::thread index_th([&]() {
      (void)hipSetDevice(ctx->device);
      for (uint32_t i; uploaded.pop(&i);) {
        irc[i] = dec[i]->index(bufs[i], lens[i], &ieo[i], nullptr);
        launch(i);
        launched_q.push(i);
      }
    });
    for (uint32_t i = 0; i < n; ++i) {
      if (staged || lens[i] <= (size_t(512) << 20)) continue;
      seq[i] = 1;
      dec[i]->pre_upload(bufs[i], lens[i]);
      uploaded.push(i);
    }
    uploaded.close();
    std::vector<uint32_t> par;
    for (uint32_t i = 0; i < n; ++i)
      if (!seq[i]) par.push_back(i);
    const uint32_t nt = std::min<uint32_t>((uint32_t)par.size(), 16);
    std::atomic<uint32_t> next{0};
    // (a snapshot whose bytes went up from the index pass -- 64 to 512 MB -- joins the two stages
    // as soon as it is indexed: its walk runs while later snapshots still upload)
    auto work = [&]() {
      (void)hipSetDevice(ctx->device);
      for (uint32_t j; (j = next.fetch_add(1)) < par.size();) {
        const uint32_t i = par[j];
        irc[i] = dec[i]->index(bufs[i], lens[i], &ieo[i], nullptr);
        if (!staged && dec[i]->early_upload()) {
          launch(i);
          seq[i] = 1;
          launched_q.push(i);
        }
      }
    };
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < nt; ++t) th.emplace_back(work);
    if (nt) work();
    for (auto& t : th) t.join();
    index_th.join();
    launched_q.close();
    walk_th.join();
    device_th.join();
  }
  if (tm) tm->index_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  // CDB_DECODE_TRACE=<file>: one JSON line of phase times (host clock, ms) appended per call
  PhaseClock clk(t_start);
  clk.mark("index");
  {
    cdb_status st = CDB_OK;
    for (uint32_t i = 0; i < n; ++i)
      if (!seq[i] && launch(i)) live.push_back(i);
    std::vector<uint32_t> host;  // sections whose host part (the pass resumed after them) remains
    while (!live.empty()) {
      std::vector<uint32_t> next;
      for (uint32_t i : live) {
        const int r = dec[i]->dd_step(&ieo[i]);
        if (r == 1) next.push_back(i);
        else if (r == 2) host.push_back(i);
        else irc[i] = dec[i]->status();
      }
      live.swap(next);
    }
    {  // the host parts side by side (one thread each, at most 16 at once)
      std::atomic<uint32_t> nx{0};
      auto work = [&]() {
        for (uint32_t j; (j = nx.fetch_add(1)) < host.size();) {
          const uint32_t i = host[j];
          dec[i]->dd_host(&ieo[i]);
          irc[i] = dec[i]->status();
        }
      };
      std::vector<std::thread> th;
      for (uint32_t t = 1; t < std::min<uint32_t>((uint32_t)host.size(), 16); ++t) th.emplace_back(work);
      work();
      for (auto& t : th) t.join();
    }
    if (st != CDB_OK) return st;
  }
  clk.mark("deferred_datas");
  for (int k = 0; k < 4; ++k) {
    static const char* names[4] = {"dd_alloc_bytes_ms", "dd_upload_call_ms", "dd_alloc_scratch_ms", "dd_walk_launch_ms"};
    std::vector<double> v;
    for (uint32_t i = 0; i < n; ++i) v.push_back(dec[i]->lt_[k]);
    clk.add(names[k], v);
  }
  // every snapshot's device preparation queued, one synchronisation, then the halves that read
  // back; statuses are taken in snapshot order (a launch failure stops the launches after it)
  for (uint32_t i = 0; i < n; ++i)
    if (!seq[i]) peo[i] = ieo[i];
  bool any_pending = false;
  // the side sections' offsets and kinds go up from one page-locked region (kept in the context)
  std::vector<uint64_t> pin_at(n + 1, 0);
  for (uint32_t i = 0; i < n; ++i)
    pin_at[i + 1] = pin_at[i] + (seq[i] ? 0 : ((dec[i]->side_bytes() + 63) & ~uint64_t(63)));
  if (pin_at[n] > ctx->dec_pin_bytes) {
    if (ctx->dec_pin) (void)hipHostFree(ctx->dec_pin);
    ctx->dec_pin = nullptr;
    ctx->dec_pin_bytes = 0;
    const size_t want = pin_at[n] + pin_at[n] / 4;
    if (hipHostMalloc(&ctx->dec_pin, want, hipHostMallocDefault) == hipSuccess) ctx->dec_pin_bytes = want;
    else ctx->dec_pin = nullptr;  // (the staging ring then)
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (seq[i]) {  // (prepared on the after-walk thread)
      if (prc[i] != CDB_OK && prc[i] != CDB_INVALID_SNAPSHOT_CHECKSUM) break;
      continue;
    }
    int rc = irc[i];
    uint8_t* pin = ctx->dec_pin ? (uint8_t*)ctx->dec_pin + pin_at[i] : nullptr;
    if (rc == CDB_OK || rc == CDB_INVALID_SNAPSHOT_CHECKSUM)
      rc = dec[i]->prepare_launch(&peo[i], pin, pin ? pin_at[i + 1] - pin_at[i] : 0);
    prc[i] = rc;
    any_pending |= dec[i]->prepare_pending();
    if (rc != CDB_OK && rc != CDB_INVALID_SNAPSHOT_CHECKSUM) break;
  }
  if (any_pending && hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync(decode)") != CDB_OK)
    return CDB_DEVICE_ERROR;
  for (uint32_t i = 0; i < n; ++i) {
    size_t eo = peo[i];
    int rc = prc[i];
    if (dec[i]->prepare_pending()) rc = dec[i]->prepare_finish(&eo);
    if (rc != CDB_OK && rc != CDB_INVALID_SNAPSHOT_CHECKSUM) {
      *failed = i;
      *err_off = eo;
      return rc;
    }
    if (rc != CDB_OK && rc_all == CDB_OK) {  // a checksum mismatch: the rows are still merged
      rc_all = rc;
      *failed = i;
      *err_off = eo;
    }
    tot[0] += dec[i]->keys();
    tot[1] += dec[i]->nodes();
    tot[2] += dec[i]->members();
  }
  if (tot[0] >= (1ull << 32) || tot[1] >= (1ull << 32) || tot[2] >= (1ull << 32))
    return fail(ctx, CDB_BAD_ARGUMENT, "decoded rows exceed 2^32 per family");
  clk.mark("prepare_device");
  cdb_status st;
  // one run per snapshot when every snapshot is in key-hash order (written from a merge result)
  bool runs = n <= CDB_MAX_RUNS;
  for (uint32_t i = 0; i < n && runs; ++i)  // (a snapshot the after-walk thread sorted is checked again)
    if ((!seq[i] || !dec[i]->sorted()) && (st = dec[i]->order_check()) != CDB_OK) return st;
  if (runs) {
    if ((st = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync(decode order)")) != CDB_OK) return st;
    for (uint32_t i = 0; i < n && runs; ++i) {
      if (seq[i] && dec[i]->sorted()) continue;
      if (dec[i]->read_order()) continue;
      // the reference's HashMap order: sorted into a run unless the caller keeps stream order
      if (!(flags & CDB_DECODE_STREAM_ORDER) && (st = dec[i]->sort_to_run()) != CDB_OK) return st;
      runs = dec[i]->sorted();
    }
  }
  clk.mark("order_sort");
  std::memset(din, 0, sizeof *din);
  const bool rec = flags & CDB_DECODE_ROWS_RECORDS;
  auto alloc = [&](cdb_dev_rows* r, uint64_t rows, int nc) {
    return rec ? cdb_dev_rows_alloc_records(ctx, r, rows, nc) : cdb_dev_rows_alloc(ctx, r, rows, nc);
  };
  clk.mark("order_sort_sync");
  if ((st = alloc(&din->keys, tot[0], kKeyCols)) != CDB_OK || (st = alloc(&din->nodes, tot[1], kNodeCols)) != CDB_OK ||
      (st = alloc(&din->members, tot[2], kMemberCols)) != CDB_OK) {
    cdb_dev_rows_release(ctx, &din->keys);
    cdb_dev_rows_release(ctx, &din->nodes);
    cdb_dev_rows_release(ctx, &din->members);
    return st;
  }
  clk.mark("alloc_rows");
  uint64_t o[3] = {0, 0, 0};
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t* k[kKeyCols];
    uint64_t* nd[kNodeCols];
    uint64_t* mb[kMemberCols];
    // (records: field c >= 1 of row r at col[c][r * stride], so the offset scales by the stride)
    const uint64_t ks = std::max<uint32_t>(din->keys.stride, 1), cs = std::max<uint32_t>(din->nodes.stride, 1);
    for (int c = 0; c < kKeyCols; ++c) k[c] = din->keys.col[c] + o[0] * (c ? ks : 1);
    for (int c = 0; c < kNodeCols; ++c) nd[c] = din->nodes.col[c] + o[1] * (c ? cs : 1);
    for (int c = 0; c < kMemberCols; ++c) mb[c] = din->members.col[c] + o[2] * (c ? cs : 1);
    if (runs)
      for (int f = 0; f < 3; ++f) din->run_start[f][i] = o[f];
    // (every snapshot's emit queued, one synchronisation, then the halves that read back; a snapshot
    // the after-walk thread emitted into rows of its own is copied into place)
    if (erc[i] != CDB_OK || (dec[i]->emitted_own() ? (st = dec[i]->move_rows(k, nd, mb))
                                                   : (st = dec[i]->emit_launch(k, nd, mb, (uint32_t)ks,
                                                                               (uint32_t)cs, i, runs))) != CDB_OK) {
      if (erc[i] != CDB_OK) st = (cdb_status)erc[i];
      (void)hipStreamSynchronize(ctx->stream);
      cdb_dev_rows_release(ctx, &din->keys);
      cdb_dev_rows_release(ctx, &din->nodes);
      cdb_dev_rows_release(ctx, &din->members);
      *failed = i;
      return st;
    }
    o[0] += dec[i]->keys();
    o[1] += dec[i]->nodes();
    o[2] += dec[i]->members();
  }
  st = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync(decode emit)");
  for (uint32_t i = 0; i < n && st == CDB_OK; ++i) {
    DecodeTiming t1;
    if (dec[i]->emit_pending() && (st = dec[i]->emit_finish(&t1)) != CDB_OK) *failed = i;
  }
  if (st != CDB_OK) {
    cdb_dev_rows_release(ctx, &din->keys);
    cdb_dev_rows_release(ctx, &din->nodes);
    cdb_dev_rows_release(ctx, &din->members);
    return st;
  }
  din->n_pos = n;
  if (runs) {
    din->n_runs = n;
    for (int f = 0; f < 3; ++f) din->run_start[f][n] = o[f];
  }
  clk.mark("emit");
  {
    uint64_t bytes = 0;
    for (uint32_t i = 0; i < n; ++i) bytes += lens[i];
    clk.write(n, bytes, tot, runs);
  }
  if (tm)  // everything but the host index passes (the snapshots' device work overlaps)
    tm->device_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count() - tm->index_ms;
  return rc_all;
}

}  // namespace cdb
