// Host-side columnar batch: one decoded snapshot (SoA rows + the byte arena they refer to).
#pragma once
#include <stdint.h>

#include <memory>
#include <mutex>
#include <utility>
#include <string>
#include <vector>

#include "../../include/cdb_merge.h"
#include "common.h"

namespace cdb {

// Allocator whose resize() leaves new elements uninitialised: result columns are overwritten
// whole by device downloads, so zero-filling them first only costs a sequential pass.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind { using other = DefaultInitAlloc<U>; };
  DefaultInitAlloc() = default;
  template <class U>
  DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
using ColVec = std::vector<uint64_t, DefaultInitAlloc<uint64_t>>;


struct ByteRef {  // a byte range inside Batch::raw
  uint64_t off, len;
};
using RefVec = std::vector<ByteRef, DefaultInitAlloc<ByteRef>>;

struct ReplicaAdd { uint64_t add_time, node_id; std::string alias, addr; uint64_t uuid; uint32_t seq; };
struct ReplicaDel { std::string addr; uint64_t t; uint32_t seq; };  // seq: order among the replica entries

struct DeviceRefs;

struct Batch {
  std::vector<uint8_t, DefaultInitAlloc<uint8_t>> raw;  // the snapshot bytes: arena for keys, values, members

  // Key rows in stream order: DATAS entries, then EXPIRES, then DELETES (db.rs:122-136).
  // The GPU sees kh kf ct ut dt aux meta; key_ref/val_ref stay on the host.
  ColVec kh, kf, ct, ut, dt, aux, meta;
  RefVec key_ref, val_ref;
  uint64_t n_data = 0, n_expires = 0, n_deletes = 0;

  // Counter children (type_counter.rs:21): pkh pkf node v t meta.
  ColVec n_pkh, n_pkf, n_node, n_v, n_t, n_meta;

  // Set/Dict member tags after load-time reconstruction: pkh pkf mh mf t meta (+ refs).
  ColVec m_pkh, m_pkf, m_h, m_f, m_t, m_meta;
  RefVec m_ref, m_vref;

  // Node header and replica metadata (snapshot.rs:140-179).
  std::string version;
  uint64_t node_id = 0, uuid_he_sent = 0;
  std::string alias, addr;
  std::vector<ReplicaAdd> replica_add;
  std::vector<ReplicaDel> replica_del;

  // cdb_decode_snapshots_device: the row columns above stay empty, the rows live in HBM
  // (dev_rows = keys, nodes, members there); byte references, header and replicas are here.
  bool rows_on_device = false;
  uint64_t dev_rows[3] = {0, 0, 0};
  // ... and until a consumer asks (refs_ready), the byte references too.
  std::shared_ptr<DeviceRefs> dev_refs;

  uint64_t n_keys() const { return kh.size(); }
  uint64_t n_nodes() const { return n_pkh.size(); }
  uint64_t n_members() const { return m_pkh.size(); }
};

// Byte references cdb_decode_snapshots_device left in HBM: key_ref | val_ref (n pairs each),
// then m_ref | m_vref (nm pairs each) in one allocation on `device`; host-tier member rows are
// patched in on download. Only the canonical dump and the encoder resolve bytes, so decoding
// into HBM for a merge does not pay the 32 B/row trip back to the host.
struct DeviceRefs {
  struct Patch { uint64_t row; ByteRef m, mv; };
  int device = 0;
  void* dev = nullptr;
  uint64_t n = 0, nm = 0;
  std::vector<Patch> patch;
  // CDB_DECODE_KEEP_BYTES: the snapshot bytes stay in HBM too (raw + raw_off = byte 0), for
  // cdb_encode_device; freed with the batch
  void* raw = nullptr;
  uint64_t raw_off = 0;
  std::mutex mu;
  ~DeviceRefs();
};
// Downloads b's byte references if they are still in HBM (decode_gpu.hip); thread-safe.
cdb_status refs_ready(cdb_ctx* ctx, Batch* b);

// Copies a large host buffer with the staging ring's copy threads (capi.cpp).
void parallel_copy(void* dst, const void* src, size_t bytes);
// Fills b->raw with the caller's snapshot bytes (uninitialised storage, huge pages, parallel copy).
void adopt_raw(Batch* b, const uint8_t* buf, size_t len);

// Decoder (decode.cpp). Returns a cdb_status value.
int decode_snapshot(const uint8_t* buf, size_t len, uint32_t flags, Batch* out, size_t* err_off);

// GPU decode (decode_gpu.hip): the host validates the stream and indexes its entries (same
// errors and offsets as decode_snapshot; header, replica entries and checksum decoded as
// usual, no key rows), then kernels parse every entry.
struct EntryIndex {
  std::vector<uint64_t> offset;    // byte offset of the entry (its key's length varint)
  std::vector<uint8_t> kind;       // 0 DATAS, 1 EXPIRES, 2 DELETES (stream order)
};
// The stream checksum, left for the GPU: CRC-64/Jones of raw[0, len) must equal `got`
// (otherwise CDB_INVALID_SNAPSHOT_CHECKSUM at err_off).
struct DeferredCrc {
  bool pending = false;
  uint64_t len = 0, got = 0;
  size_t err_off = 0;
};
// A large DATAS section met before any other entry, left to the device index (decode_gpu.hip):
// the host pass stops at its first entry (index_snapshot returns kIndexDeferred and a cursor),
// the device finds the entries' offsets, and index_resume continues after the section's last
// entry (the sections after it, the checksum) with the same checks and error offsets.
constexpr int kIndexDeferred = -100;
constexpr uint64_t kDeviceIndexMinEntries = 1u << 17;
struct DeferredDatas {
  bool pending = false;
  uint64_t start = 0;  // byte offset of the section's first entry
  uint64_t count = 0;  // the section's entry count
};
struct IndexCursor;
// With `crc` non-null and at least one entry indexed, the checksum is not computed here but
// described in *crc for the caller to check.
// threads > 1: a large DATAS section is indexed by that many threads (speculative sync points,
// stitched in order; the result is the sequential pass's, entry for entry).
// defer and cursor non-null: a large first DATAS section is deferred as described above. buf may
// be null when `out` already holds the bytes (a second, host-only pass after a device fallback).
int index_snapshot(const uint8_t* buf, size_t len, uint32_t flags, Batch* out, EntryIndex* idx, size_t* err_off,
                   DeferredCrc* crc = nullptr, uint32_t threads = 1, DeferredDatas* defer = nullptr,
                   IndexCursor** cursor = nullptr);
int index_resume(IndexCursor* ic, uint64_t datas_end, size_t* err_off);
void index_cursor_free(IndexCursor* ic);
// The end offset of the DATAS entry at `off` (false: it does not parse).
bool index_data_entry_end(const Batch& b, uint64_t off, uint64_t* end);
struct DecodeTiming {
  double index_ms = 0;   // host pass
  double device_ms = 0;  // uploads, both kernels, downloads (HIP events)
};
bool decode_entry_children(const Batch& b, uint64_t off, uint64_t kh, uint64_t kf, Batch* side, uint64_t* total);


}  // namespace cdb

// A merge (or op-apply) result, host-resident; bytes resolve through inputs[pos].
struct cdb_merged {
  std::vector<std::shared_ptr<cdb::Batch>> inputs;  // pos -> decoded batch (byte arenas)
  cdb::ColVec k[cdb::kKeyOutCols], nd[cdb::kNodeCols], mb[cdb::kMemberCols];
  // DB::garbages (db.rs:14, LinkedList<(key, field, uuid)>): every Deletes entry applied to this
  // state (DB::delete, db.rs:73-76, from each merged snapshot's DELETES section in fold order),
  // less what DB::gc popped (db.rs:82-119). Kept across cdb_merge_into chains, so that a GC after
  // a chain pops exactly what the reference's list holds -- including stale entries of keys
  // deleted again later, and never the entry a previous gc lost at its stop.
  struct Garbage {
    uint64_t kh, kf, t;
  };
  std::vector<Garbage> garbage;
  // replica-metadata merge, computed on first request
  bool replicas_done = false;
  std::vector<std::string> rep_str;          // addr / alias storage (stable: reserved up front)
  std::vector<cdb_replica_entry> replicas;
};
