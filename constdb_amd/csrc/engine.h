// Internal engine interface shared by the HIP driver (engine.hip) and the host C-ABI
// glue (capi.cpp). Not part of the public ABI (include/cdb_merge.h is).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/cdb_merge.h"

namespace cdb {
struct Node;  // RCCL communicators of a multi-device context (shard.hip)
}

struct cdb_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_part = nullptr, ev_bucket = nullptr;
  hipStream_t side = nullptr;                         // the wide tier runs beside the wave tier;
  hipStream_t side2 = nullptr;                        // node / member partitions beside the keys'
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;    // (timing disabled)
  hipEvent_t ev_pfork = nullptr, ev_pn = nullptr, ev_pm = nullptr;
  hipEvent_t ev_cs = nullptr, ev_cw = nullptr, ev_cdone = nullptr;  // pipelined compaction (side2)
  std::mutex pin_mu;  // staged_copy's pinned ring (pin, pin_next, pin_ev): the decoder's threads share it
  std::string last_error;
  struct Buf { void* p = nullptr; size_t bytes = 0; };
  Buf ws[48];  // named workspace slots, grown on demand, reused across calls
  void* pin = nullptr;                                // pinned staging ring of host<->device copies
  hipEvent_t pin_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  uint64_t pin_next = 0;                              // next slot of the ring (continues across calls)
  uint64_t runs_host[3 * 65] = {};                    // sorted-run path: run starts staged for the device
  uint32_t runs_err = 0;                              // sorted-run path: run_mark_kernel's verdict
  void* dec_pin = nullptr;                            // decode: page-locked side-section offsets and
  size_t dec_pin_bytes = 0;                           // kinds of every snapshot (grown, kept)
  std::vector<hipStream_t> idx_streams;               // decode: one stream per snapshot's entry index
                                                      // (created on first use, kept: creating and
                                                      // destroying 8 cost 13 ms per call)
  // multi-device context (cdb_ctx_create_multi): this context is device slot 0; shards[i - 1] is
  // the context of device slot i; node holds the RCCL communicators (shard.hip)
  std::vector<cdb_ctx*> shards;
  cdb::Node* node = nullptr;
};

namespace cdb {

enum WsSlot {
  WS_KA = 0, WS_KB, WS_NA, WS_NB, WS_MA, WS_MB,         // partition ping-pong per family
  WS_DIR,                                               // bucket directories + hist/cursor
  WS_MISC,                                              // stats, last_bad, hot list
  WS_HOT,                                               // hot-bucket scratch slab
  WS_SCAN,                                              // scan partials (keys, merge)
  WS_SCAN2, WS_SCAN3,                                   // scan partials (nodes, members)
  WS_OWNER,                                             // owner-partition directory
  WS_PERM,                                              // final-level row permutations (u32)
  WS_STATS,                                             // statistic shards
  WS_KHCOL,                                             // key-hash column of the row level
  WS_HOST_IN_K, WS_HOST_IN_N, WS_HOST_IN_M,             // cdb_merge: uploaded batches
  WS_HOST_OUT_K, WS_HOST_OUT_N, WS_HOST_OUT_M,          // cdb_merge: device-side result
  WS_RUNDIR, WS_RUNMISC,                                // sorted-run path: run directories, gap lists
  WS_HOTC3, WS_HOTMETA, WS_HOTK, WS_HOTCH, WS_RADIX,    // over-capacity child path (hot.hip.h)
  WS_MAT,                                               // sorted-run path: materialisation counts
  WS_PIPE,                                              // pipelined bucket phase: range bases, totals
  WS_XK, WS_XN, WS_XM,                                  // sharded merge: received rows per family
  WS_YK, WS_YN, WS_YM,                                  // sharded merge: this device's output rows
  WS_PK, WS_PN, WS_PM,                                  // sharded merge: owner-packed rows (inputs not in runs)
  WS_SPLIT,                                             // sharded merge: owner splits of the runs
  WS_CRCTAB, WS_CRCPART,                                // decode: CRC tables, per-tile CRC partials
  WS_WIDE,                                              // wide tier: group counters per range
  WS_STATE,                                             // cdb_dev_state_rows: zero bases, error word
  WS_RUNBDIR,                                           // sorted-run path: bucket-major run directory
  WS_UNITS,                                             // persistent wave tier: unit-start bitmap
  WS_HOTMERGE,                                          // chip-wide path: list bounds, merge tiles
  WS_COUNT
};
static_assert(WS_COUNT <= 48, "cdb_ctx::ws has 48 slots");

struct Batch;
struct DecodeTiming;
int decode_snapshot_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint32_t flags, Batch* out, size_t* err_off,
                        DecodeTiming* tm);
int decode_snapshots_gpu_device(cdb_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, uint32_t n,
                                uint32_t flags, Batch* const* outs, cdb_dev_input* din, uint32_t* failed,
                                size_t* err_off, DecodeTiming* tm);
cdb_status fail(cdb_ctx* ctx, cdb_status st, const std::string& msg);
// Records why a context could not be created (cdb_last_error(NULL)); returns st.
cdb_status set_create_error(cdb_status st, const std::string& msg);
// The device merge pipeline (engine.hip) on stream s of ctx's device.
cdb_status merge_device_impl(cdb_ctx* ctx, const cdb_dev_input* in, const cdb_merge_opts* opts, cdb_dev_output* out,
                             cdb_merge_stats* stats, hipStream_t s);
// Releases a multi-device context's node (RCCL communicators; shard.hip).
void node_destroy(Node* n);
cdb_status hip_check(cdb_ctx* ctx, hipError_t e, const char* what);
cdb_status launch_check(cdb_ctx* ctx, hipStream_t s, const char* what);
void* ws_get(cdb_ctx* ctx, int slot, size_t bytes, cdb_status* st);
// One host<->device copy of pageable memory (a column or a piece of one).
struct HostSeg {
  void* host;
  void* dev;
  size_t bytes;
};
// Moves `segs` through the context's pinned staging ring: host threads copy chunk k into (out
// of) a pinned slot while the DMA engine moves chunk k-1 on stream s. H2D returns once every
// chunk is queued (the sources may be freed); D2H returns with every copy complete.
cdb_status staged_copy(cdb_ctx* ctx, const HostSeg* segs, size_t nseg, bool h2d, hipStream_t s);
// Single-segment forms; copies under 1 MB go straight through hipMemcpyAsync.
cdb_status staged_h2d(cdb_ctx* ctx, void* dev, const void* host, size_t bytes, hipStream_t s);
cdb_status staged_d2h(cdb_ctx* ctx, void* host, const void* dev, size_t bytes, hipStream_t s);
// Asks for transparent huge pages on a fresh host buffer about to be filled by a download.
void advise_huge(void* p, size_t bytes);
uint64_t crc_tile_bytes();
cdb_status crc64_device(cdb_ctx* ctx, const uint8_t* dev, uint64_t padded, uint64_t* d_crc, hipStream_t s);
// The same, queued only (no synchronisation): tables and partials in the context's workspace, so
// calls on one stream may follow each other without waiting.
cdb_status crc64_device_queued(cdb_ctx* ctx, const uint8_t* dev, uint64_t padded, uint64_t* d_crc, hipStream_t s);
cdb_status stamp_pos(cdb_ctx* ctx, uint64_t* meta, uint64_t n, uint32_t pos, hipStream_t s);
// Stable LSD radix sort of n (u64 key, u32 value) pairs on key bits [lo, bits) (radix.hip.h; workspace
// slots WS_RADIX, WS_SCAN); *k / *v receive whichever buffers hold the result.
cdb_status radix_sort_pairs(cdb_ctx* ctx, uint64_t** k, uint32_t** v, uint64_t* k2, uint32_t* v2, uint64_t n,
                            int lo, int bits, hipStream_t s);
// Exclusive scan of n u32 into u64 (workspace slot WS_SCAN); *d_total (device, may be null) = the sum.
cdb_status exclusive_scan_u32(cdb_ctx* ctx, const uint32_t* in, uint64_t n, uint64_t* out, uint64_t* d_total,
                              hipStream_t s);
// A merge result's family as fold position 0 of the next merge, in place in the input rows:
// meta <- tag | pos 0 | src = row; for keys (aux != null) also aux <- the counter sum (the
// result's win, staged in aux) for counters, 0 otherwise.
cdb_status state_rows(cdb_ctx* ctx, uint64_t* meta, uint64_t* aux, uint64_t n, hipStream_t s);

}  // namespace cdb
