/*
 * cdb_merge.h — C ABI of the MI355X-native ConstDB snapshot-merge engine (libcdbmerge.so).
 *
 * Drop-in boundary for the reference's replica-sync hot path (fxsjy/ConstDB, Rust):
 *   - decode:  SnapshotLoader::next            src/snapshot.rs:120-220
 *              Object::load_snapshot            src/object.rs:110-129
 *              Counter/Set/Dict::load_snapshot  src/type_counter.rs:111, src/crdt/lwwhash.rs:207,341
 *   - merge:   the per-entry loop of Puller::merge_replicates_in_main
 *              src/replica/pull.rs:120-158, i.e. DB::merge_entry (src/db.rs:31-43),
 *              Object::merge (src/object.rs:63-83), Counter::merge (src/type_counter.rs:59-91),
 *              Set::merge / Dict::merge (src/crdt/lwwhash.rs:319-323 / 176-181),
 *              DB::delete / DB::expire_at (src/db.rs:68-76), DB::gc (src/db.rs:82-119).
 * Instead of one FFI call per entry (which would defeat a GPU), a whole snapshot is
 * decoded into a columnar batch and R batches are merged in one call. Binding examples
 * for a Rust host (the reference's language) are in INTEGRATION.md.
 *
 * Plain C types only: pointers, sizes, fixed-width integers. No torch types.
 * Threading: a cdb_ctx is used from one thread at a time (like the reference's single
 * main task, src/server.rs:95,128-130); no callbacks into the host.
 * Ownership: input buffers are caller-owned and read-only; everything returned by a
 * cdb_* call is library-owned and released with the matching *_free.
 */
#ifndef CDB_MERGE_H
#define CDB_MERGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes map 1:1 onto the decode-path CstError variants (src/lib.rs:146-175). */
typedef enum cdb_status {
  CDB_OK = 0,
  CDB_INVALID_SNAPSHOT = 1,          /* CstError::InvalidSnapshot(offset)      lib.rs:158 */
  CDB_INVALID_SNAPSHOT_CHECKSUM = 2, /* CstError::InvalidSnapshotChecksum      lib.rs:174 */
  CDB_INVALID_TYPE = 3,              /* CstError::InvalidType (unknown tag)    lib.rs:152, object.rs:121 */
  CDB_IO_ERROR = 4,                  /* CstError::IoError (truncated stream)   lib.rs:162 */
  CDB_DICT_MERGE_UNIMPLEMENTED = 5,  /* Dict::merge's unimplemented!() panic,  lwwhash.rs:180 (strict mode) */
  CDB_BAD_ARGUMENT = 6,
  CDB_DEVICE_ERROR = 7,              /* a HIP call failed */
  CDB_OUT_OF_MEMORY = 8,
  CDB_NO_DEVICE = 9,                 /* no gfx950 device visible: the engine never falls back to the CPU */
  CDB_INVALID_REQUEST_MSG = 10,      /* CstError::InvalidRequestMsg: malformed RESP  lib.rs:156, conn/buf_read.rs:114-200 */
  CDB_NEED_MORE_MSG = 11             /* CstError::NeedMoreMsg: the stream ends inside a message  lib.rs:154 */
} cdb_status;

typedef struct cdb_ctx cdb_ctx;       /* device, streams, workspace */
typedef struct cdb_batch cdb_batch;   /* one decoded snapshot (columnar, host + device) */
typedef struct cdb_merged cdb_merged; /* a merge result (device-resident, host-readable) */

/* ------------------------------------------------------------------ context */
/* Creates a context on HIP device `device`. Fails with CDB_NO_DEVICE when no device. */
cdb_status cdb_ctx_create(cdb_ctx** out, int device);
void cdb_ctx_destroy(cdb_ctx* ctx);
/* Human-readable last error of this context (static storage, valid until the next call). With
 * ctx == NULL: why the last cdb_ctx_create_multi of the process failed (no context exists then). */
const char* cdb_last_error(const cdb_ctx* ctx);

/* ------------------------------------------------------------------ decode
 * Replaces SnapshotLoader::next (snapshot.rs:120-220) + the load_snapshot functions.
 * Decodes the WRITER layout of server.rs:183-215 (CRC-64/Jones over every byte up to and
 * including flag 0x08, then 8 raw little-endian CRC bytes). Bytes values use the
 * loader's `len, bytes` layout (object.rs:114-117; the writer at object.rs:94-97 omits
 * the length, which the reference itself cannot read back).
 * On CDB_INVALID_SNAPSHOT_CHECKSUM the batch is still returned in *out (the reference
 * merges every entry before it reaches the checksum, replica/pull.rs:64-79), so the
 * caller decides; for every other error *out is NULL and *err_offset = byte offset. */
enum {
  CDB_DECODE_REFERENCE_CHECKSUM = 1u << 0, /* reproduce snapshot.rs:207-213 exactly: read the
                                              checksum as a varint and CRC it too (rejects
                                              practically every well-formed dump) */
  CDB_DECODE_ROWS_RECORDS = 1u << 1,       /* cdb_decode_snapshots_device: emit the rows in the
                                              records layout (cdb_dev_rows) instead of columns */
  CDB_DECODE_STREAM_ORDER = 1u << 2,       /* cdb_decode_snapshots_device: leave a snapshot that is not
                                              in key-hash order in stream order (n_runs = 0) instead
                                              of sorting it into a run */
  CDB_DECODE_KEEP_BYTES = 1u << 3          /* cdb_decode_snapshots_device: keep the snapshot bytes in
                                              HBM with the batch (for cdb_encode_device; the host
                                              copy stays too) */
};
cdb_status cdb_decode_snapshot(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint32_t flags,
                               cdb_batch** out, size_t* err_offset);

/* The same decode with the per-entry work on the GPU: a host pass validates
 * the stream (identical status codes and offsets) and indexes its entries; HIP kernels parse
 * every entry in parallel (varints, key and member hashes, the loader's load-time dedup) and
 * emit the rows. The batch is identical to cdb_decode_snapshot's, field for field. Needs a
 * device (CDB_NO_DEVICE otherwise). *index_ms / *device_ms (may be NULL) receive the host
 * pass time and the device time (transfers included). */
cdb_status cdb_decode_snapshot_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint32_t flags,
                                   cdb_batch** out, size_t* err_offset, double* index_ms,
                                   double* device_ms);

/* GPU decode of n snapshots straight into HBM, for cdb_merge_device (replica/pull.rs:64-79
 * followed by :120-128 with no host round trip of the rows). Every snapshot is validated and
 * indexed exactly as by cdb_decode_snapshot_gpu; then all are sized, ONE set of device columns
 * is allocated (*out; release each family with cdb_dev_rows_release) and snapshot i's rows are
 * emitted into it at fold position i -- row for row what cdb_upload_batches leaves from the
 * host-decoded batches. batches[i] receives snapshot i's host side (bytes, byte references,
 * header, replica entries, cdb_batch_info) to resolve merge outputs by src; its row columns
 * stay in HBM, so cdb_merge, cdb_upload_batches and cdb_batch_column reject it. Its byte
 * references stay in HBM too, until the first cdb_merged_canonical_dump or cdb_encode_snapshot
 * of a result behind it downloads them (on that call's ctx, which must be this ctx's device).
 * Sorted runs: snapshot i's key rows are placed as ONE run in key-hash order (meta src still names
 * the entry), its node and member rows as one run each in their parents' order, and out->n_runs = n
 * with run_start set, so cdb_merge_device takes the sorted-run path. A snapshot whose DATAS, EXPIRES
 * and DELETES sections are each in key-hash order (one cdb_encode_snapshot wrote from a merge
 * result) is placed by merging the three sections (DATAS first on equal hashes); one in the
 * reference's HashMap order (db.rs:122-136) is sorted on the device (a stable radix sort of its
 * entries' key hashes: the same order). Snapshots with entries left to the host decoder (objects
 * past 3000 members or 1500 nodes), or CDB_DECODE_STREAM_ORDER, keep stream order: n_runs = 0 (the
 * partition path; the same result). Errors: *failed
 * is the snapshot, *err_offset the byte offset in it, and nothing is allocated; a checksum
 * mismatch (CDB_INVALID_SNAPSHOT_CHECKSUM) still returns every batch and the rows, as the
 * reference merges a snapshot's entries before it reaches the checksum. A snapshot of 64 MB to
 * 512 MB is uploaded straight from bufs[i], which the call page-locks (hipHostRegister) for its
 * duration; where that fails, from the batch's copy. The buffers must not be freed or written
 * during the call. */
struct cdb_dev_input; /* below, with cdb_merge_device */
cdb_status cdb_decode_snapshots_device(cdb_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, uint32_t n,
                                       uint32_t flags, cdb_batch** batches, struct cdb_dev_input* out,
                                       uint32_t* failed, size_t* err_offset, double* index_ms, double* device_ms);

typedef struct cdb_batch_info {
  uint64_t n_data;        /* SnapshotEntry::Data entries   (snapshot.rs:309) */
  uint64_t n_expires;     /* SnapshotEntry::Expires        (snapshot.rs:310) */
  uint64_t n_deletes;     /* SnapshotEntry::Deletes        (snapshot.rs:311) */
  uint64_t n_nodes;       /* counter children (node, v, t) (type_counter.rs:21) */
  uint64_t n_members;     /* set/dict member tags after load-time reconstruction (lwwhash.rs:207-226,341-358) */
  uint64_t node_id;       /* SnapshotEntry::Node           (snapshot.rs:306) */
  uint64_t uuid_he_sent;
  uint32_t n_replica_add; /* SnapshotEntry::ReplicaAdd     (snapshot.rs:307) */
  uint32_t n_replica_del; /* SnapshotEntry::ReplicaDel     (snapshot.rs:308) */
  char version[16];       /* SnapshotEntry::Version, "a.b.c.d" */
} cdb_batch_info;
cdb_status cdb_batch_info_get(const cdb_batch* b, cdb_batch_info* info);
/* Read-only view of one decoded column (host memory, valid while the batch lives).
 * family 0 = key rows (kh kf ct ut dt aux meta), 1 = counter nodes (pkh pkf node v t meta),
 * 2 = set/dict members (pkh pkf mh mf t meta). */
cdb_status cdb_batch_column(const cdb_batch* b, int family, int col, const uint64_t** data, uint64_t* n);
void cdb_batch_free(cdb_batch* b);

/* ------------------------------------------------------------------ merge
 * Replaces the per-entry loop of replica/pull.rs:120-158: folds `n` decoded snapshots in
 * array order (pos 0 = the local DB state, then remotes in apply order) exactly as R
 * sequential applications of DB::merge_entry / DB::delete / DB::expire_at would.
 * Deterministic: the result does not depend on row order inside a batch. */
enum {
  CDB_MERGE_STRICT_DICT_PANIC = 1u << 0, /* report Dict-on-Dict merges (where the reference
                                            panics, lwwhash.rs:180) as CDB_DICT_MERGE_UNIMPLEMENTED;
                                            default: apply the pre-panic loop (code intent) */
  CDB_MERGE_GC_DELETES = 1u << 1,        /* run DB::gc(gc_watermark) after the merge (db.rs:82-119;
                                            garbage list = Deletes entries in fold order) */
  CDB_MERGE_GC_MEMBERS = 1u << 2         /* BUILD EXTENSION: drop del-only set/dict members
                                            whose tag time < gc_watermark (the field path of
                                            db.rs:96-115, which the reference never enqueues) */
};
typedef struct cdb_merge_opts {
  uint32_t flags;
  uint32_t force_tier;   /* testing only: 0 = automatic; 1 = every bucket through the LDS
                            workgroup tier; 2 = every bucket through the global-scratch tier;
                            3 = every bucket through the wide (128-key-row) wave kernel;
                            4 = every bucket through the one-workgroup global-scratch kernel
                            (tier 2 sends children through the chip-wide child path) */
  uint64_t gc_watermark; /* ReplicaManager::min_uuid (replica/replica.rs:87-89) */
  uint32_t key_shift;    /* multi-GPU: the top `key_shift` bits of every key hash are the owner
                            rank (all equal on one device), so local buckets use the bits below */
  uint32_t pipe_ranges;  /* testing only: 0 = automatic (the bucket phase runs in 8 ranges, each
                            compacted while the next merges, for merges of >= 64M rows); n >= 1 =
                            exactly n ranges whatever the size */
} cdb_merge_opts;

typedef struct cdb_merge_stats {
  uint64_t key_rows_in, node_rows_in, member_rows_in;
  uint64_t key_rows_out, node_rows_out, member_rows_out;
  uint64_t type_conflicts;   /* db.rs:38-40 error! log events (local kept) */
  uint64_t dict_merges;      /* Dict-on-Dict merges (the reference panics at lwwhash.rs:180) */
  uint64_t deletes_gced;
  uint64_t members_gced;
  uint64_t duplicate_rows;   /* same key twice in one snapshot (never written by db.rs:122-136) */
  uint64_t orphan_children;  /* child rows whose key row is missing (malformed input) */
  uint64_t hot_buckets;      /* buckets handled by the over-capacity path */
  uint64_t wide_buckets;     /* buckets handled by the wide wave kernel (65..128 key rows) */
  uint64_t mid_buckets;      /* buckets handled by the LDS workgroup tier */
  double   device_ms;        /* device time of the whole merge pipeline (HIP events) */
  double   partition_ms;     /* bucket partition of the three row families */
  double   bucket_ms;        /* fused bucket-merge kernel (the dominant kernel) */
  double   finish_ms;        /* over-capacity buckets + dense compaction */
  uint64_t sorted_runs;      /* 1 when the sorted-run path ran (partition_ms = its run directories) */
  uint64_t hot_slow_runs;    /* chip-wide path: (key, id-bits) runs folded by successor selection
                                (ids sharing the sort tag's id bits, or runs of > 8 rows) */
  uint64_t hot_merged_children; /* chip-wide path: children whose runs arrived in child order
                                (a merge result's) and were merged instead of radix-sorted */
  uint64_t wave_pipe_buckets;   /* buckets folded by the persistent wave tier (bucket_wave_pipe_kernel) */
  uint64_t wave_pipe_units;     /* its units: groups of consecutive buckets merged by one wave */
} cdb_merge_stats;

cdb_status cdb_merge(cdb_ctx* ctx, cdb_batch* const* inputs, uint32_t n,
                     const cdb_merge_opts* opts, cdb_merged** out, cdb_merge_stats* stats);

/* Merges n decoded snapshots into an existing result, the way the reference merges every peer
 * snapshot into its live DB (replica/pull.rs:120-128 -> DB::merge_entry, db.rs:31-43, which
 * mutates server.db): `state` is fold position 0, inputs[i] position i + 1. The same as cdb_merge
 * over [decode(encode(state)), inputs...] without the round trip: state's rows go to the device
 * as input rows (a counter's load-time total is its sum, every other field as stored). *out is
 * a new result (state is unchanged) whose bytes resolve through state's inputs, then `inputs`
 * (at most 255 in all behind one result; encode + decode starts a fresh chain). */
cdb_status cdb_merge_into(cdb_ctx* ctx, cdb_merged* state, cdb_batch* const* inputs, uint32_t n,
                          const cdb_merge_opts* opts, cdb_merged** out, cdb_merge_stats* stats);

/* DB::gc(tombstone) (db.rs:82-119; Server::gc, server.rs:257-262, with ReplicaManager::min_uuid) on a
 * merge result, in place. Every result keeps the reference's garbage list (DB::garbages, db.rs:14):
 * the Deletes entries of every snapshot merged into it (DB::delete, db.rs:73-76), in fold order,
 * across cdb_merge_into chains, less what earlier gcs popped. The gc pops it from the back while
 * t <= tombstone, removes a key's Deletes row when its time equals a popped entry's, and stops at
 * the first entry with t > tombstone, which is popped and lost (the list keeps the entries before
 * it). *removed (may be NULL) receives the rows removed. CDB_MERGE_GC_DELETES in a cdb_merge /
 * cdb_merge_into is this gc after the merge. A result from cdb_merged_from_device lists only the
 * host-resident batches' entries (after its state's): a device merge's own GC flag applies the
 * rule to that call's inputs alone. */
cdb_status cdb_merged_gc(cdb_ctx* ctx, cdb_merged* m, uint64_t tombstone, uint64_t* removed);
/* Entries in a result's garbage list (DB::garbages.len()). */
uint64_t cdb_merged_garbage_count(const cdb_merged* m);

/* Canonical dump of a merge result: keys sorted by bytes, members by bytes, counter nodes
 * by id, then expires and deletes (the text format of oracle/constdb_oracle.py's
 * canonical_dump). *out is released with cdb_free. */
cdb_status cdb_merged_canonical_dump(cdb_ctx* ctx, cdb_merged* m, char** out, size_t* len);

/* Replica-metadata merge: the ReplicaManager's LWWHash<addr, ReplicaMeta>
 * (replica/replica.rs:16-35) after the same fold. Input 0 is the local node: its ReplicaAdd /
 * ReplicaDel entries are installed verbatim (its own add and del maps). Every later input's
 * entries are then applied in stream order. A ReplicaAdd goes through add_replica ->
 * LWWHash::set (lwwhash.rs:87-107) unless it names input 0's node id (pull.rs:133-135); a
 * ReplicaDel goes through remove_replica -> LWWHash::rem (lwwhash.rs:109-128). The result is
 * sorted by addr; strings are NUL-terminated and live as long as the merged result. Host-side:
 * a few entries per snapshot. */
typedef struct cdb_replica_entry {
  const char* addr;
  const char* alias;      /* ReplicaMeta.he.alias of the add tag ("" without one) */
  uint64_t node_id;       /* ReplicaMeta.he.id of the add tag */
  uint64_t uuid_he_sent;  /* ReplicaMeta.uuid_he_sent of the add tag */
  uint64_t add_time;      /* add tag time (has_add) */
  uint64_t del_time;      /* del tag time (has_del) */
  uint32_t has_add, has_del;
} cdb_replica_entry;
cdb_status cdb_merged_replicas(cdb_merged* m, const cdb_replica_entry** out, size_t* n);

/* ------------------------------------------------------------------ snapshot encode
 * Replaces Server::dump_all (src/server.rs:183-215) -> DB::dump (src/db.rs:122-136) ->
 * SnapshotWriter::write_entry / Object::save_snapshot (src/snapshot.rs:25-64,
 * src/object.rs:85-108, src/type_counter.rs:101-109, src/crdt/lwwhash.rs:189-205,325-339) ->
 * ReplicaManager::dump_snapshot (src/replica/replica.rs:100-119), and the CRC-64/Jones of the
 * whole stream (snapshot.rs:62-64, server.rs:205-207), for a merge result. The entries are
 * sized, laid out by prefix scans and written by HIP kernels; the checksum is computed on the
 * GPU (per-chunk CRC + GF(2) combination). Order: DATAS in the result's row order, then
 * EXPIRES, then DELETES; within a Set/Dict the add map precedes the del map (the reference's
 * HashMap order is unspecified, so any order is a valid dump). Bytes values carry their
 * length (the loader's layout, object.rs:114-117). Replica entries are written
 * as in dump_snapshot: every has_add entry as 0x03, then every has_del entry as 0x04, in array
 * order (pass the cdb_merged_replicas result, or any other list). *out is released with
 * cdb_free. */
typedef struct cdb_encode_header {
  uint64_t node_id;                   /* server.rs:193 */
  const char* alias; size_t alias_len;
  const char* addr; size_t addr_len;
  uint64_t last_uuid;                 /* get_repl_last_uuid(), server.rs:198 */
  const cdb_replica_entry* replicas; size_t n_replicas;
} cdb_encode_header;
typedef struct cdb_encode_stats {
  uint64_t bytes;                     /* stream length incl. the 8 checksum bytes */
  uint64_t data_entries, expires, deletes;
  uint64_t checksum;                  /* CRC-64/Jones over bytes [0, len-8) */
  double upload_ms;                   /* H2D of result rows, refs and byte arenas */
  double device_ms;                   /* sizing scans + emit kernels + CRC (HIP events) */
  double crc_ms;                      /* the CRC kernels alone */
  double download_ms;                 /* D2H of the stream */
} cdb_encode_stats;
cdb_status cdb_encode_snapshot(cdb_ctx* ctx, cdb_merged* m, const cdb_encode_header* hdr, uint8_t** out,
                               size_t* len, cdb_encode_stats* stats);
/* CRC-64/Jones (reflected, init 0, no xorout; crc64 2.0.0 as used at snapshot.rs:3) of a
 * host buffer, computed on the GPU with the same kernels. */
cdb_status cdb_crc64_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t* crc);

void cdb_merged_free(cdb_merged* m);
void cdb_free(void* p);

/* ------------------------------------------------------------------ op-stream apply
 * Partial replication: after the snapshot, a replica receives `replicate` messages (RESP arrays
 * `replicate <nodeid> <last_uuid> <uuid> <command> <args...>`, server.rs:290-314) and `replack`
 * messages, and applies them one at a time (Puller::apply_his_replicates, replica/pull.rs:184-235).
 *
 * cdb_decode_ops replaces the per-message front half on the host: RESP framing
 * (conn/buf_read.rs:114-210), the uuid gate against uuid_he_sent (pull.rs:199-209: a message
 * whose last_uuid is behind is a duplicate and skipped; one that is ahead means lost commands
 * and is dropped), the command lookup (cmd.rs:39-41) and each handler's argument parsing.
 * It yields op rows in stream order. Replayed commands: set delbytes incr decr delcnt sadd srem
 * delset hset hdel deldict. spop (random member on the replica, type_set.rs:82-111), del (never
 * replicated) and the read/control commands are counted as `unsupported` and skipped; names not
 * in the command table are `unknown` and skipped with the uuid advanced, like the reference.
 * Returns CDB_INVALID_REQUEST_MSG (*err_offset = the message's offset) on malformed RESP, and
 * CDB_NEED_MORE_MSG when the stream ends inside a message: then *out still holds every complete
 * message before it and *err_offset = the bytes consumed.
 *
 * cdb_apply_ops replaces the handlers (cmd.rs:188-309, type_counter.rs:142-204,
 * type_set.rs:13-134, type_hash.rs:11-119, DB::query db.rs:52-66) for the whole batch at once,
 * on the device, on top of `state` (a merge result: the DB the snapshot sync produced, or an
 * earlier apply). The result is a new merge result over the same inputs plus the op stream
 * (its fold position = state's input count); `state` is left unchanged. */
typedef struct cdb_ops cdb_ops;
typedef struct cdb_ops_info {
  uint64_t n_messages;     /* RESP messages decoded */
  uint64_t n_ops;          /* op rows (commands that reach the DB) */
  uint64_t n_node_args;    /* counter (node, delta) arguments: incr/decr (1), delcnt pairs */
  uint64_t n_member_args;  /* set members / dict fields */
  uint64_t applied;        /* replicate messages whose handler ran (pull.rs:218-222) */
  uint64_t duplicates;     /* uuid_he_sent > last_uuid: skipped (pull.rs:205-206) */
  uint64_t lost;           /* uuid_he_sent < last_uuid, or a malformed replicate: dropped (pull.rs:201-204) */
  uint64_t unknown;        /* not in the command table (pull.rs:213-217) */
  uint64_t unsupported;    /* in the table, not replayed (see above) */
  uint64_t cmd_errors;     /* argument errors (WrongArity ...): logged by the reference, uuid advanced */
  uint64_t replacks;
  uint64_t uuid_he_sent;   /* after the stream */
  uint64_t uuid_he_acked;
} cdb_ops_info;
cdb_status cdb_decode_ops(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t uuid_he_sent, cdb_ops** out,
                          size_t* err_offset);
/* The same decode with the per-message work on the GPU (the framing being replaced
 * is conn/buf_read.rs:102-111): every '*' at a line start is a candidate message start, one
 * thread per candidate parses the RESP value there, the host follows the chain of sizes from
 * byte 0 (candidates inside bulk payloads are never reached), one thread per message decodes
 * pull.rs:184-235 up to the uuid gate and the handler's arguments, the host runs the gate
 * (sequential: it carries uuid_he_sent), and one thread per applied op writes its rows and
 * hashes. The result equals cdb_decode_ops's field for field, statuses and offsets included.
 * Streams the device path leaves to the host (an integer argument whose decimal form differs
 * from its digits, top-level values that are not arrays, nesting deeper than 16) are decoded by
 * cdb_decode_ops; *used_gpu (may be NULL) tells which ran. *host_ms / *device_ms (may be NULL):
 * the host part (chain walk, gate, arena copy) and the rest of the call. */
cdb_status cdb_decode_ops_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t uuid_he_sent, cdb_ops** out,
                              size_t* err_offset, double* host_ms, double* device_ms, uint32_t* used_gpu);
/* Read-only view of one column of a decoded op stream (family 0: kh kf ct ut dt aux meta, then
 * key_ref and val_ref as (offset, length) pairs; 1: pkh pkf node v t meta; 2: pkh pkf mh mf t meta,
 * then m_ref and m_vref as pairs). *n counts u64 words. */
cdb_status cdb_ops_column(const cdb_ops* ops, int family, int col, const uint64_t** data, uint64_t* n);
cdb_status cdb_ops_info_get(const cdb_ops* ops, cdb_ops_info* info);
/* Testing only (no device needed): the GPU decode's host index pass with a large DATAS section
 * split over `threads` threads (speculative sync points, stitched in order) against the
 * sequential pass: CDB_OK when status, error offset, entry offsets and kinds, section counts
 * and the deferred checksum are identical. *entries = the entries indexed. */
cdb_status cdb_snapshot_index_selftest(const uint8_t* buf, size_t len, uint32_t flags, uint32_t threads,
                                       uint64_t* entries);
void cdb_ops_free(cdb_ops* ops);

typedef struct cdb_apply_stats {
  uint64_t ops_in, node_args_in, member_args_in, key_rows_in;
  uint64_t key_rows_out, node_rows_out, member_rows_out;
  uint64_t type_errors;       /* CstError::InvalidType from a handler (as_mut_* on another type) */
  uint64_t expired_on_query;  /* DB::query turned an expired key into a delete (db.rs:58-63) */
  double device_ms;           /* device time of the apply pipeline (HIP events; transfers excluded) */
} cdb_apply_stats;
cdb_status cdb_apply_ops(cdb_ctx* ctx, cdb_merged* state, const cdb_ops* ops, cdb_merged** out,
                         cdb_apply_stats* stats);

/* ------------------------------------------------------------------ device level
 * The same merge over rows already resident in HBM (what bench.py times, and what a multi-GPU
 * driver calls after its RCCL all-to-all). Every field is a u64; layouts are documented in
 * DESIGN.md §Data layout and constdb_amd/csrc/common.h. Rows may come in any order and from up
 * to 63 fold positions (pos in the meta word).
 *
 * Two input layouts (cdb_dev_rows.stride):
 *   columns (stride 0): col[c] is a plain array, row i's field c = col[c][i];
 *   records (stride = ncols - 1): col[0] is the (parent) key-hash column and the other fields of
 *     row i are one record of `stride` words, col[c] = col[1] + (c - 1), field c = col[c][i * stride]
 *     (keys: a 48-B record kf ct ut dt aux meta; nodes / members: a 40-B record). Same bytes per row
 *     as columns, but a bucket's rows of one run are ONE contiguous byte range, which the merge
 *     copies into LDS in 16-B pieces (the sorted-run path); the hash column alone is
 *     what the run directories stream. Arrays 16-B aligned, readable up to the next 16-B boundary
 *     (cdb_dev_rows_alloc* allocate so). */
typedef struct cdb_dev_rows {
  uint64_t* col[8]; /* keys: kh kf ct ut dt aux meta | nodes: pkh pkf node v t meta |
                       members: pkh pkf mh mf t meta */
  uint64_t n;
  uint32_t stride;  /* words from one row to the next in col[1..7]: 0 (or 1) plain columns */
  uint32_t stride0; /* the same for col[0]; inputs: 0. A merge's own bucket-layout outputs
                       (cdb_dev_output.compact = 0) are whole rows: stride0 = stride = row words */
} cdb_dev_rows;
#define CDB_MAX_RUNS 64
typedef struct cdb_dev_input {
  cdb_dev_rows keys, nodes, members;
  uint32_t n_pos;
  uint32_t n_runs;  /* 0: rows in any order (the partition path). 1..64: the rows of every family
                       are n_runs consecutive runs, run r = rows [run_start[f][r], run_start[f][r+1])
                       of family f (0 keys, 1 nodes, 2 members), each non-decreasing in column 0
                       (the key hash; children: the parent key hash) -- one run per replica.
                       Producers: cdb_dev_state_rows (a merge result as position 0), and
                       cdb_decode_snapshots_device over snapshots cdb_encode_snapshot wrote
                       (their three key sections merged back into one run on decode). Then the
                       merge reads the runs in place (no partition pass). A run found out of
                       order, or more than 32 runs, send the merge to the partition path; the
                       result is the same. */
  uint64_t run_start[3][CDB_MAX_RUNS + 1];
} cdb_dev_input;
/* The merge's buckets (the engine's native result layout, cdb_dev_output.compact = 0): bucket b
 * owns a hash range (ascending in b); its output rows of family f (0 keys, 1 nodes, 2 members) are
 * count[f][b] whole rows at row slots first[f][b] ..; dense[f][b] is the index the bucket's first
 * row has in the dense result (an exclusive scan of count). Library-owned, in the ctx workspace. */
typedef struct cdb_dev_buckets {
  uint64_t nb;
  const uint32_t* first[3];
  const uint32_t* count[3];
  const uint32_t* dense[3];
} cdb_dev_buckets;

/* Merge outputs.
 *   compact = 1: dense plain columns in caller-allocated keys / nodes / members (at least the
 *     input row counts), keys in key-hash order, cref = (absolute child row, count);
 *   either layout: a key's children follow in ascending bit-reversed child id (id1), then id2, so
 *     a result kept as the next merge's input brings its hot keys' children as sorted lists (the
 *     chip-wide path merges those instead of sorting them; stats.hot_merged_children);
 *   compact = 0: the engine's bucket layout, no compaction pass: the merge points keys / nodes /
 *     members at its own row slots (whole AoS rows: stride0 = stride = 8 words per key row, 6 per
 *     child row; library-owned, valid until the next merge on the ctx) and fills `buckets`. Every row
 *     of a bucket lies in its slot range, in key-hash order; a key row's cref child begin is relative
 *     to its bucket's first child slot. ->n = the dense row counts. Consumers read this layout
 *     directly: cdb_dev_state_rows (the next merge's position 0), cdb_merged_from_device (canonical
 *     dump, encode, op apply, cdb_merge_into). */
typedef struct cdb_dev_output {
  cdb_dev_rows keys;    /* kh kf ct ut dt meta win cref */
  cdb_dev_rows nodes;   /* pkh pkf node v t meta */
  cdb_dev_rows members; /* pkh pkf mh mf t meta */
  uint32_t compact;
  uint32_t reserved;
  cdb_dev_buckets buckets; /* compact = 0 only */
} cdb_dev_output;

/* Owner grouping for inputs that are not in runs: a counting-sort scatter of one
 * family's rows by owner = the top `owner_bits` bits (0..9) of column 0 (key hash, or parent key
 * hash for children, so a key and its children share an owner) into `out` (caller-allocated,
 * >= in->n rows, `ncols` = 6, 7 or 8 fields, either input layout on either side); the 2^owner_bits
 * per-owner row counts go to the host array `counts`, so owner d's rows are out's rows
 * [sum(counts[<d]), sum(counts[<=d])). cdb_merge_sharded calls it for such inputs (their owner
 * slices then travel as one unsorted run each); inputs in runs need no grouping: their owner
 * slices are found by binary search (cdb_shard_splits). */
cdb_status cdb_partition_owner(cdb_ctx* ctx, const cdb_dev_rows* in, int ncols, int owner_bits,
                               cdb_dev_rows* out, uint64_t* counts, void* stream);

/* Uploads decoded batches [0, n) into freshly allocated device rows (*out; release each family
 * with cdb_dev_rows_release), batch i at fold position i, so that a caller can keep a decoded
 * replica set resident in HBM and merge it with cdb_merge_device (what cdb_merge does per call). */
cdb_status cdb_upload_batches(cdb_ctx* ctx, cdb_batch* const* inputs, uint32_t n, cdb_dev_input* out);

/* The host view of a cdb_merge_device result (compacted): its rows are downloaded, and bytes
 * resolve through inputs[i] for fold position i -- or, with `state` non-NULL (the result the
 * device merge's position 0 came from, via cdb_dev_state_rows), position 0 through state and
 * position i >= 1 through inputs[i - 1], as cdb_merge_into. inputs may be batches whose rows are
 * in HBM (cdb_decode_snapshots_device). The result supports everything a cdb_merge result does
 * (canonical dump, replicas, encode, op apply, cdb_merge_into). */
cdb_status cdb_merged_from_device(cdb_ctx* ctx, cdb_merged* state, cdb_batch* const* inputs, uint32_t n,
                                  const cdb_dev_output* out, cdb_merged** m);

/* cdb_encode_snapshot of a cdb_merge_device result without its host view (server.rs:183-215 for a
 * node whose state is in HBM): the result rows (either output layout) are read where the merge left
 * them, fold position i resolves through inputs[i] -- their byte references from HBM while a device
 * decode still holds them there (cdb_decode_snapshots_device; host-tier member references are
 * patched into those tables), their snapshot bytes from HBM when decoded with
 * CDB_DECODE_KEEP_BYTES, everything else uploaded. No result row crosses PCIe; the stream comes
 * back once. Byte for byte the stream cdb_encode_snapshot writes for
 * cdb_merged_from_device(ctx, NULL, inputs, n, out). A result whose position 0 was a previous
 * result (cdb_dev_state_rows) needs that chain's host view: use cdb_merged_from_device. */
cdb_status cdb_encode_device(cdb_ctx* ctx, const cdb_dev_output* out, cdb_batch* const* inputs, uint32_t n,
                             const cdb_encode_header* hdr, uint8_t** bytes, size_t* len, cdb_encode_stats* stats);

/* A merge result kept in HBM as fold position 0 of the next cdb_merge_device (the reference's
 * persistent server.db, replica/pull.rs:120-128): `state` rows (either output layout) are copied
 * into caller-allocated input rows (columns or records, 7 / 6 / 6 fields, at least state's row
 * counts; ->n is set) as key rows kh kf ct ut dt aux meta (aux = a counter's sum) and children
 * unchanged, every meta word with pos 0 and src = the row's dense index in `state`. A merge
 * result is in key-hash order, so these rows are ONE run of every family for the next merge
 * (run_start[f] = {0, n, ...}). */
cdb_status cdb_dev_state_rows(cdb_ctx* ctx, const cdb_dev_output* state, cdb_dev_rows* keys, cdb_dev_rows* nodes,
                              cdb_dev_rows* members, void* stream);

/* Appends every family of `src` (any input layout) behind dst's rows (dst->keys.n etc.; dst's
 * columns must have room: the caller allocated them), converting to dst's layout and raising each
 * row's fold position by pos_offset; dst's row counts, n_pos and runs follow (src's runs after dst's
 * when both are in runs, else dst->n_runs = 0). With cdb_dev_state_rows this chains a merge result
 * (position 0) and newly decoded snapshots (positions 1..) into the next cdb_merge_device input. */
cdb_status cdb_dev_input_append(cdb_ctx* ctx, cdb_dev_input* dst, const cdb_dev_input* src, uint32_t pos_offset,
                                void* stream);

/* The dense form (compact = 1) of a bucket-layout result `src` in caller-allocated columns
 * (8 / 6 / 6, at least src's row counts): what the compaction pass of a compact = 1 merge does. */
cdb_status cdb_dev_output_compact(cdb_ctx* ctx, const cdb_dev_output* src, cdb_dev_output* dst, void* stream);

/* Allocates device columns for `rows` rows of a family (ncols u64 columns, 1..8) in *r. */
cdb_status cdb_dev_rows_alloc(cdb_ctx* ctx, cdb_dev_rows* r, uint64_t rows, int ncols);
/* The records layout (above) for `rows` rows of an ncols-field family (6 or 7): a hash column and
 * records of ncols - 1 words, in one allocation released by cdb_dev_rows_release. */
cdb_status cdb_dev_rows_alloc_records(cdb_ctx* ctx, cdb_dev_rows* r, uint64_t rows, int ncols);
void cdb_dev_rows_release(cdb_ctx* ctx, cdb_dev_rows* r);
/* Runs the merge pipeline on the context's stream (or `stream` if non-NULL, a hipStream_t).
 * out->*.n receive the output row counts. Synchronises before returning. */
cdb_status cdb_merge_device(cdb_ctx* ctx, const cdb_dev_input* in, const cdb_merge_opts* opts,
                            cdb_dev_output* out, cdb_merge_stats* stats, void* stream);

/* ------------------------------------------------------------------ several GPUs in one process
 * SURVEY §8b/§8e. The reference merges in ONE server process (server.rs:95,128-130); a node's GPUs
 * are driven the same way: one context over device_count devices (one stream set and workspace
 * per device), with RCCL communicators between them (ncclCommInitAll; RCCL is loaded on first use).
 * Keys shard by owner = the top log2(device_count) bits of the key hash (children follow their
 * parent key), so every §8a rule stays local to one device: no collective beyond the row exchange.
 * Device slot i may name any visible device; a device listed twice gives two shards on one GPU
 * (testing), whose rows then move by device copies instead of RCCL. device_count must be a power
 * of two, at most 8. The single-device functions take a multi-device context as its slot 0.
 * Distinct devices whose RCCL cannot be loaded (CDB_RCCL_LIB names the library, default
 * librccl.so.1) or whose communicators cannot be created are refused with CDB_DEVICE_ERROR and
 * the reason in cdb_last_error(NULL) -- never a silent change of transport; the environment
 * variable CDB_SHARD_TRANSPORT=peer asks for HIP peer copies instead (cdb_exchange_stats.transport
 * 2). */
cdb_status cdb_ctx_create_multi(cdb_ctx** out, int device_count, const int* devices);
int cdb_ctx_device_count(const cdb_ctx* ctx);
/* The context of device slot i (slot 0: ctx itself), for per-device calls (cdb_gen_device,
 * cdb_dev_rows_alloc, cdb_decode_snapshots_device, ...). Owned by ctx; NULL if out of range. */
cdb_ctx* cdb_ctx_shard(cdb_ctx* ctx, int i);

typedef struct cdb_exchange_stats {
  uint32_t n_devices;
  uint32_t transport;        /* 0 none (one device), 1 RCCL point-to-point, 2 device/peer copies */
  uint32_t packed;           /* devices whose input was not in sorted runs: rows grouped by owner first */
  uint32_t reserved;
  double split_ms;           /* owner splits of every input (+ run order check / owner pack), host wall */
  double exchange_ms;        /* the row transfers until every device holds its rows, host wall */
  double merge_ms;           /* the slowest device's merge pipeline (HIP events) */
  double total_ms;           /* the whole call, host wall */
  uint64_t bytes_moved;      /* bytes that crossed between devices */
  uint64_t bytes_local;      /* bytes a device kept (its own owner slices, device copies) */
  uint64_t transfers;        /* point-to-point operations (or peer copies) posted */
  uint64_t link_bytes[8][8]; /* [source slot][destination slot] */
} cdb_exchange_stats;

/* One sharded merge step over every device of ctx (replica/pull.rs:120-128 for a whole node):
 * in[i] are the rows resident on device slot i (fold positions are global across slots: slot i's
 * replicas must not reuse a position another slot's rows carry, or the merge folds them as one
 * replica; n_runs >= 1 for key-hash-
 * ordered runs, each run's owner slices then move as they are; n_runs = 0, or runs found out of
 * order, are grouped by owner on that device first). Each device receives the rows it owns -- as
 * runs when every source was in runs, so its merge takes the sorted-run path -- and merges them
 * (cdb_merge_device with key_shift = log2(device_count); opts->key_shift is ignored). out[i]
 * receives device slot i's compacted result (keys in key-hash order): library-owned columns in
 * that device's workspace, valid until the next cdb_merge_sharded on ctx or cdb_ctx_destroy; cref
 * child ranges index out[i]'s own child rows. stats (may be NULL) is an array of device_count;
 * xs (may be NULL) the exchange figures. */
cdb_status cdb_merge_sharded(cdb_ctx* ctx, const cdb_dev_input* in, const cdb_merge_opts* opts, cdb_dev_output* out,
                             cdb_merge_stats* stats, cdb_exchange_stats* xs);

/* The exchange plan of a sharded merge, as host functions (cdb_merge_sharded computes the splits on
 * the devices; constdb_amd/dist.py, one process per GPU, with torch.searchsorted, and takes its
 * receive layout from cdb_shard_recv_plan: one plan for both drivers). No device needed.
 * cdb_shard_splits: the owner slices of n_runs key-hash-ordered runs of one family (rows
 * [run_start[r], run_start[r + 1]) of the hash column kh, a host array): out[r * (n_devices + 1) + d]
 * = the first row of run r owned by device d or later (owner = the top log2(n_devices) hash bits).
 * cdb_shard_recv_plan: the receive layout of one destination. counts = every source's rows for it,
 * source after source, each as [3][n_runs[i]] (family-major). The destination receives one run per
 * (source, source run) with rows in any family, in that order: recv_src / recv_run name them and
 * run_start[f * (cap + 1) + k] is run k's first row of family f (run_start[f * (cap + 1) + n] the
 * family's total, also in totals[f]). CDB_BAD_ARGUMENT (with *n_recv_runs set) when more than cap
 * runs. */
cdb_status cdb_shard_splits(const uint64_t* kh, const uint64_t* run_start, uint32_t n_runs, uint32_t n_devices,
                            uint64_t* out);
cdb_status cdb_shard_recv_plan(uint32_t n_sources, const uint32_t* n_runs, const uint64_t* counts, uint32_t cap,
                               uint32_t* n_recv_runs, uint32_t* recv_src, uint32_t* recv_run, uint64_t* run_start,
                               uint64_t* totals);

/* ------------------------------------------------------------------ synthetic inputs
 * Seeded generator of replica states. Writes snapshot bytes
 * (for the decode path and the oracle) or device rows (for HBM-resident benches). */
typedef struct cdb_gen_config {
  uint64_t seed;
  uint64_t universe;      /* number of distinct keys */
  uint32_t n_replicas;    /* R */
  uint32_t key_permille;  /* probability (x1000) that a replica holds a key */
  uint32_t mix_bytes, mix_counter, mix_set, mix_dict; /* type mix weights */
  uint32_t conflict_ppm;  /* cross-replica type-conflict probability (x1e6) */
  uint32_t tie_permille;  /* probability (x1000) that a time is forced to tie */
  uint32_t max_nodes;     /* counter nodes per key: 1..max_nodes */
  uint32_t mean_members;  /* set/dict members per key (uniform 0..2*mean) */
  uint32_t member_universe; /* members drawn from this many per key */
  uint32_t del_permille;  /* probability (x1000) that a member tag is a del */
  uint32_t side_permille; /* probability (x1000) of an expires / deletes entry per key */
  uint32_t value_min, value_max; /* Bytes value length range */
  uint32_t shard, n_shards;      /* generate only keys with owner(kh) == shard (multi-GPU) */
  uint32_t replica_lo, replica_hi; /* generate replicas [lo, hi) */
  uint32_t flags;                /* CDB_GEN_* below */
  uint32_t hot_zipf_milli;       /* config C5: children per key follow rank^-(s/1000) over key index
                                    rank i + 1 (0 = off; then max_nodes / mean_members apply) */
  uint32_t stream;               /* cdb_gen_ops: salt of the per-op draws (command, key, members,
                                    uuids) so replicas sharing a seed -- and so every key's type --
                                    replay different streams (0: the unsalted stream) */
  uint64_t hot_events;           /* config C5: expected node/member rows over all replicas */
} cdb_gen_config;
enum {
  CDB_GEN_NODE_PER_REPLICA = 1u << 0, /* counters carry one node, the replica's own id r + 1 (the
                                         2-node MEET shape of config C1, bin/test.rs:85-106) */
  CDB_GEN_OPS_ZIPF_MEMBERS = 1u << 1, /* cdb_gen_ops: zipf_milli skews member choice, keys uniform */
  CDB_GEN_OPS_TAGS_ONLY = 1u << 2,    /* cdb_gen_ops: only sadd/srem/hset/hdel (config C3): no
                                         whole-key deletes, no other types */
  CDB_GEN_ROWS_RECORDS = 1u << 3      /* cdb_gen_device: rows in the records layout (cdb_dev_rows) */
};
void cdb_gen_default(cdb_gen_config* cfg);
/* Snapshot bytes of replica r (writer layout). *out released with cdb_free. */
cdb_status cdb_gen_snapshot(const cdb_gen_config* cfg, uint32_t replica, uint8_t** out, size_t* len);
/* A replicate stream of n_ops commands (the RESP messages server.rs:290-314 sends) over the
 * same key universe: per key the generator's type (0.2 % other types: InvalidType), set/delbytes,
 * incr/decr/delcnt, sadd/srem/delset, hset/hdel/deldict; uuids chained from uuid_he_sent, 5 %
 * older than the snapshot times. Keys uniform (zipf_milli = 0) or power-law skewed (exponent
 * zipf_milli/1000 < 1). *out released with cdb_free. */
cdb_status cdb_gen_ops(const cdb_gen_config* cfg, uint64_t n_ops, uint64_t uuid_he_sent, uint32_t zipf_milli,
                       uint8_t** out, size_t* len);
/* Device rows for replicas [replica_lo, replica_hi) generated directly in HBM. */
cdb_status cdb_gen_device(cdb_ctx* ctx, const cdb_gen_config* cfg, cdb_dev_input* in);

#ifdef __cplusplus
}
#endif
#endif /* CDB_MERGE_H */
