// Op-stream apply: op rows decoded from a replicate stream (ops.cpp) and
// applied on the device (ops_apply.hip). Internal; the ABI is include/cdb_merge.h.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/cdb_merge.h"
#include "batch.h"

namespace cdb {

// Replayed write commands (cmd.rs:97-133). The code is the op row's meta tag.
enum OpCode : uint32_t {
  OP_SET = 1,       // cmd.rs:188-210
  OP_DELBYTES = 2,  // cmd.rs:290-309
  OP_INCR = 3,      // type_counter.rs:169-186
  OP_DECR = 4,      // type_counter.rs:188-204
  OP_DELCNT = 5,    // type_counter.rs:142-167
  OP_SADD = 6,      // type_set.rs:13-40
  OP_SREM = 7,      // type_set.rs:42-63
  OP_DELSET = 8,    // type_set.rs:115-134
  OP_HSET = 9,      // type_hash.rs:11-45
  OP_HDEL = 10,     // type_hash.rs:47-68
  OP_DELDICT = 11,  // type_hash.rs:100-119
};

// One decoded stream: a Batch holding the op rows in stream order:
//   kh kf (key hash), ct = uuid (current_uuid), ut = node id of the replicate message,
//   aux = byte offset of the message, meta = code | pos | row; key_ref, val_ref (SET value).
// Children in stream order (within an op: argument order):
//   nodes   n_pkh n_pkf (parent key) n_node n_v (delta, i64) n_t = op row
//   members m_pkh m_pkf m_h m_f (member hash) m_t = op row, m_ref (member), m_vref (HSET value)
// raw = the stream bytes, then the decimal forms of integer arguments (get_int_bytes).
int decode_ops(const uint8_t* buf, size_t len, uint64_t uuid_he_sent, Batch* out, cdb_ops_info* info,
               size_t* err_off);

// The same decode with the per-message work on the GPU (ops_gpu.hip). Returns 1 when the
// stream needs decode_ops instead (rare shapes, or a device failure); otherwise 0 with the
// decode's status in *rc (CDB_OK, CDB_NEED_MORE_MSG or CDB_INVALID_REQUEST_MSG).
int decode_ops_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t uuid_he_sent, Batch* out,
                   cdb_ops_info* info, size_t* err_off, int* rc, double* host_ms, double* device_ms);

// Device apply (ops_apply.hip): state = merge-result columns (host), ops = the op batch at fold
// position pos_ops; out = merge-result columns (host).
cdb_status apply_ops_impl(cdb_ctx* ctx, const ColVec* sk, const ColVec* sn, const ColVec* sm, const Batch& ops, uint32_t pos_ops,
                          ColVec* ok, ColVec* on, ColVec* om,
                          cdb_apply_stats* stats);

}  // namespace cdb
