// Shared row layouts, packing helpers and hashes for the ConstDB MI355X merge engine.
// Compiled for the host (g++/hipcc host pass) and for gfx950 (hipcc device pass).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CDB_HD __host__ __device__ __forceinline__
#else
#define CDB_HD inline
#endif

namespace cdb {

// Object encodings (object.rs:19-22) and the two side-map families carried in the
// same key-row stream (db.rs:12-13).
enum : uint8_t {
  TAG_COUNTER = 0, TAG_BYTES = 3, TAG_DICT = 4, TAG_SET = 5,
  TAG_EXPIRE = 6,  // expires[key] = t        (db.rs:68-71)
  TAG_DELETE = 7,  // deletes[key] = t        (db.rs:73-76)
};
CDB_HD uint32_t tag_family(uint32_t tag) { return tag <= TAG_SET ? 0u : tag - 5u; }  // 0 data, 1 exp, 2 del

// Member tag kinds (lwwhash.rs:14-15): a loaded member carries exactly one tag.
enum : uint8_t { KIND_ADD = 0, KIND_DEL = 1 };

// meta word: tag/kind:8 | pos:8 | src:48. `pos` = fold position (0 = local DB, then
// remotes in apply order); `src` = the row's index inside its decoded batch.
CDB_HD uint64_t meta_pack(uint32_t tag, uint32_t pos, uint64_t src) {
  return ((uint64_t)(tag & 0xFF) << 56) | ((uint64_t)(pos & 0xFF) << 48) | (src & 0xFFFFFFFFFFFFull);
}
CDB_HD uint32_t meta_tag(uint64_t m) { return (uint32_t)(m >> 56); }
CDB_HD uint32_t meta_pos(uint64_t m) { return (uint32_t)(m >> 48) & 0xFF; }
CDB_HD uint64_t meta_src(uint64_t m) { return m & 0xFFFFFFFFFFFFull; }
CDB_HD uint64_t meta_order(uint64_t m) { return m & 0x00FFFFFFFFFFFFFFull; }  // (pos, src)

// Maximum replicas per merge call: pos < 63; vmask bit 63 is the counter "merged" flag.
constexpr int kMaxPos = 63;
constexpr uint64_t kVmaskMerged = 1ull << 63;

// Column counts per row family (device SoA, every column u64).
//   key rows   : kh kf ct ut dt aux meta           (aux = counter load-time sum)
//   node rows  : pkh pkf node v t meta             (counter children, type_counter.rs:21)
//   member rows: pkh pkf mh mf t meta              (set/dict tags, lwwhash.rs:14-15)
// Outputs:
//   key out    : kh kf ct ut dt meta win cref      (win: Bytes winner (pos,src) /
//                                                   counter sum / side-map winner;
//                                                   cref: child begin:40 | count:24)
//   node out   : pkh pkf node v t meta             (meta: head (pos,src) of the segment)
//   member out : pkh pkf mh mf t meta              (meta: kind | winner (pos,src))
constexpr int kKeyCols = 7, kNodeCols = 6, kMemberCols = 6, kKeyOutCols = 8;
// Partitioned rows as the bucket kernels read them (AoS records, columns in the order above):
// a key row is 8 words (the 8th is padding: one aligned 64-B line), a child row 6 words.
constexpr int kKeyStride = 8, kChildStride = 6;
enum KeyCol { K_KH = 0, K_KF, K_CT, K_UT, K_DT, K_AUX, K_META };
enum ChildCol { C_PKH = 0, C_PKF, C_ID1, C_ID2, C_T, C_META };  // node: ID2 = v
enum KeyOutCol { O_KH = 0, O_KF, O_CT, O_UT, O_DT, O_META, O_WIN, O_CREF };

CDB_HD uint64_t cref_pack(uint64_t begin, uint64_t count) {
  return (begin << 24) | (count & 0xFFFFFF);
}

// Input rows come in two layouts (cdb_dev_rows.stride): plain columns, or the (parent) key-hash
// column col[0] plus one record of s = ncols - 1 words per row (col[c] = col[1] + c - 1). Field c
// of row i in either (s = 1 for columns).
CDB_HD uint64_t row_field(const uint64_t* const* col, uint32_t s, int c, uint64_t i) {
  return col[c][c ? i * s : i];
}

// ---------------------------------------------------------------- hashing
// splitmix64 finalizer: full-avalanche 64-bit mix.
// A child's order key inside its key (every merge tier writes a key's children in ascending
// child_order(id1), then id2): the id's bits reversed, so that the leading bits that the chip-wide
// tiers sort on are the id's low bits -- distinct for small counter node ids as for member hashes.
// A merge result's children are then sorted by every prefix of it, which is what lets the chip-wide
// path merge the runs of such inputs instead of sorting them (hot.hip.h).
CDB_HD uint64_t child_order(uint64_t id1) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_bitreverse64(id1);
#else
  uint64_t r = 0;
  for (int i = 0; i < 64; ++i) r |= ((id1 >> i) & 1) << (63 - i);
  return r;
#endif
}
CDB_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

// 128-bit identity of a byte string: two independently seeded 64-bit hashes computed in
// one pass over 8-byte little-endian words (tail zero-padded, length folded into the
// seed). Grouping is by the pair; a false merge needs a 128-bit collision.
struct Hash128 { uint64_t h, f; };
CDB_HD Hash128 hash_bytes(const uint8_t* p, uint64_t n, uint64_t domain) {
  uint64_t a = 0x9E3779B97F4A7C15ull ^ domain ^ (n * 0xC2B2AE3D27D4EB4Full);
  uint64_t b = 0xD6E8FEB86659FD93ull ^ (domain * 0x9E3779B97F4A7C15ull) ^ n;
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) w |= (uint64_t)p[i + k] << (8 * k);
    a = mix64(a ^ w) + 0x632BE59BD9B4E019ull;
    b = mix64(b + w) ^ 0x85EBCA77C2B2AE63ull;
  }
  if (i < n) {
    uint64_t w = 0;
    for (int k = 0; i + k < n; ++k) w |= (uint64_t)p[i + k] << (8 * k);
    a = mix64(a ^ w) + 0x632BE59BD9B4E019ull;
    b = mix64(b + w) ^ 0x85EBCA77C2B2AE63ull;
  }
  Hash128 r;
  r.h = mix64(a ^ (b >> 17));
  r.f = mix64(b ^ (a << 13) ^ 0x27D4EB2F165667C5ull);
  return r;
}
constexpr uint64_t kDomainKey = 0x4B4559ull, kDomainMember = 0x4D454Dull;

// Multi-GPU owner of a (parent) key hash: its top `bits` bits. In a run (rows in
// key-hash order) the rows owned by device d are one slice: this is its first row in [lo, hi).
CDB_HD uint64_t owner_lower_bound(const uint64_t* kh, uint64_t lo, uint64_t hi, uint32_t d, int bits) {
  uint64_t x = lo, y = hi;
  while (x < y) {
    const uint64_t m = (x + y) >> 1;
    if ((bits ? kh[m] >> (64 - bits) : 0) < d) x = m + 1;
    else y = m;
  }
  return x;
}

// Bucket hash of every row family: the parent KEY hash, so that a key and all its
// children land in the same bucket (the fused bucket kernel needs no lookups).
CDB_HD uint64_t bucket_of(uint64_t kh, int bits) { return bits ? kh >> (64 - bits) : 0; }

// Sub-digit inside a bucket used by the in-LDS counting sort (next `db` bits of kh).
CDB_HD uint32_t sub_digit(uint64_t kh, int bucket_bits, int db) {
  const int sh = 64 - bucket_bits - db;
  return sh >= 0 ? (uint32_t)(kh >> sh) & ((1u << db) - 1) : (uint32_t)(kh << (-sh)) & ((1u << db) - 1);
}

}  // namespace cdb
