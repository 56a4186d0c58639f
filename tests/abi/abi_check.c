/* C-ABI check of libcdbmerge (include/cdb_merge.h), compiled with the system C compiler.
 *
 * 1. Pins the layout of every public struct that a binding mirrors by hand (the Rust #[repr(C)]
 *    structs of INTEGRATION.md, the ctypes structs of constdb_amd/__init__.py): a change to the
 *    header that moves a field fails this file at compile time.
 * 2. Runs the boundary as a C host would: cdb_gen_snapshot -> cdb_decode_snapshot (no device
 *    needed) -> cdb_ctx_create -> cdb_merge -> cdb_merged_canonical_dump. Without a device it
 *    stops after the decode with "no device" (cdb_ctx_create must say CDB_NO_DEVICE); with one
 *    it writes the canonical dump to argv[1] for the caller to compare with the oracle.
 */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cdb_merge.h"

#define PIN_SIZE(T, n) _Static_assert(sizeof(T) == (n), "sizeof(" #T ") changed")
#define PIN_OFF(T, f, n) _Static_assert(offsetof(T, f) == (n), "offsetof(" #T ", " #f ") changed")

PIN_SIZE(cdb_merge_opts, 24);
PIN_OFF(cdb_merge_opts, gc_watermark, 8);
PIN_OFF(cdb_merge_opts, key_shift, 16);
PIN_SIZE(cdb_merge_stats, 168);
PIN_OFF(cdb_merge_stats, hot_slow_runs, 160);
PIN_OFF(cdb_merge_stats, mid_buckets, 112);
PIN_OFF(cdb_merge_stats, device_ms, 120);
PIN_OFF(cdb_merge_stats, sorted_runs, 152);
PIN_SIZE(cdb_batch_info, 80);
PIN_OFF(cdb_batch_info, n_replica_add, 56);
PIN_OFF(cdb_batch_info, version, 64);
PIN_SIZE(cdb_replica_entry, 56);
PIN_OFF(cdb_replica_entry, node_id, 16);
PIN_OFF(cdb_replica_entry, has_add, 48);
PIN_SIZE(cdb_encode_header, 64);
PIN_OFF(cdb_encode_header, last_uuid, 40);
PIN_OFF(cdb_encode_header, replicas, 48);
PIN_SIZE(cdb_encode_stats, 72);
PIN_OFF(cdb_encode_stats, upload_ms, 40);
PIN_SIZE(cdb_ops_info, 104);
PIN_SIZE(cdb_apply_stats, 80);
PIN_OFF(cdb_apply_stats, device_ms, 72);
PIN_SIZE(cdb_dev_rows, 72);
PIN_OFF(cdb_dev_rows, n, 64);
PIN_SIZE(cdb_dev_input, 1784);
PIN_OFF(cdb_dev_input, n_pos, 216);
PIN_OFF(cdb_dev_input, n_runs, 220);
PIN_OFF(cdb_dev_input, run_start, 224);
PIN_SIZE(cdb_dev_output, 224);
PIN_OFF(cdb_dev_output, compact, 216);
PIN_SIZE(cdb_gen_config, 112);
PIN_OFF(cdb_gen_config, replica_hi, 88);
PIN_OFF(cdb_gen_config, flags, 92);
PIN_OFF(cdb_gen_config, hot_events, 104);
PIN_SIZE(cdb_exchange_stats, 584);
PIN_OFF(cdb_exchange_stats, split_ms, 16);
PIN_OFF(cdb_exchange_stats, bytes_moved, 48);
PIN_OFF(cdb_exchange_stats, link_bytes, 72);
_Static_assert(CDB_NEED_MORE_MSG == 11 && CDB_INVALID_REQUEST_MSG == 10 && CDB_DEVICE_ERROR == 7,
               "status codes are part of the ABI");

int main(int argc, char** argv) {
  cdb_gen_config cfg;
  cdb_gen_default(&cfg);
  cfg.seed = 17;
  cfg.universe = 3000;
  cfg.n_replicas = 3;
  cfg.replica_hi = 3;
  cdb_batch* batches[3];
  for (uint32_t r = 0; r < 3; ++r) {
    uint8_t* buf = NULL;
    size_t len = 0, off = 0;
    if (cdb_gen_snapshot(&cfg, r, &buf, &len) != CDB_OK) return 10;
    const cdb_status st = cdb_decode_snapshot(NULL, buf, len, 0, &batches[r], &off);
    cdb_free(buf);
    if (st != CDB_OK) {
      fprintf(stderr, "decode %u: status %d at %zu\n", r, (int)st, off);
      return 11;
    }
    cdb_batch_info info;
    if (cdb_batch_info_get(batches[r], &info) != CDB_OK || info.n_data == 0 || info.node_id != r + 1) return 12;
  }
  cdb_ctx* ctx = NULL;
  const cdb_status cs = cdb_ctx_create(&ctx, 0);
  if (cs == CDB_NO_DEVICE) {
    for (int r = 0; r < 3; ++r) cdb_batch_free(batches[r]);
    printf("no device\n");
    return 0;
  }
  if (cs != CDB_OK) return 13;
  cdb_merge_opts opts;
  memset(&opts, 0, sizeof opts);
  cdb_merge_stats stats;
  cdb_merged* m = NULL;
  cdb_status st = cdb_merge(ctx, batches, 3, &opts, &m, &stats);
  if (st != CDB_OK) {
    fprintf(stderr, "merge: %d %s\n", (int)st, cdb_last_error(ctx));
    return 14;
  }
  char* dump = NULL;
  size_t dlen = 0;
  if (cdb_merged_canonical_dump(ctx, m, &dump, &dlen) != CDB_OK) return 15;
  FILE* f = fopen(argc > 1 ? argv[1] : "abi_dump.txt", "wb");
  if (!f || fwrite(dump, 1, dlen, f) != dlen) return 16;
  fclose(f);
  printf("merged %llu key rows -> %llu, dump %zu bytes\n", (unsigned long long)stats.key_rows_in,
         (unsigned long long)stats.key_rows_out, dlen);
  cdb_free(dump);
  cdb_merged_free(m);
  for (int r = 0; r < 3; ++r) cdb_batch_free(batches[r]);
  cdb_ctx_destroy(ctx);
  return 0;
}
