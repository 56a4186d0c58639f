/* C-ABI check of libcdbmerge (include/cdb_merge.h), compiled with the system C compiler.
 *
 * 1. Pins the layout of every public struct that a binding mirrors by hand (the Rust #[repr(C)]
 *    structs of INTEGRATION.md, the ctypes structs of constdb_amd/__init__.py): a change to the
 *    header that moves a field fails this file at compile time.
 * 2. Runs the boundary as a C host would: cdb_gen_snapshot -> cdb_decode_snapshot (no device
 *    needed) -> cdb_ctx_create -> cdb_merge -> cdb_merged_canonical_dump. Without a device it
 *    stops after the decode with "no device" (cdb_ctx_create must say CDB_NO_DEVICE); with one
 *    it writes the canonical dump to argv[1] for the caller to compare with the oracle.
 * 3. With a device and argv[2]: the HBM-resident pull (decode into HBM -> merge into the bucket
 *    layout -> state rows + append -> second merge -> host view -> dump to argv[2]).
 * 4. With argv[3]: a two-slot multi-device context on device 0 (cdb_ctx_create_multi ->
 *    cdb_merge_sharded), each slot's dump to argv[3].<slot>.
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
PIN_SIZE(cdb_merge_stats, 192);
PIN_OFF(cdb_merge_stats, hot_merged_children, 168);
PIN_OFF(cdb_merge_stats, wave_pipe_buckets, 176);
PIN_OFF(cdb_merge_stats, wave_pipe_units, 184);
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
PIN_SIZE(cdb_dev_rows, 80);
PIN_OFF(cdb_dev_rows, n, 64);
PIN_OFF(cdb_dev_rows, stride, 72);
PIN_OFF(cdb_dev_rows, stride0, 76);
PIN_SIZE(cdb_dev_input, 1808);
PIN_OFF(cdb_dev_input, n_pos, 240);
PIN_OFF(cdb_dev_input, n_runs, 244);
PIN_OFF(cdb_dev_input, run_start, 248);
PIN_SIZE(cdb_dev_buckets, 80);
PIN_OFF(cdb_dev_buckets, count, 32);
PIN_OFF(cdb_dev_buckets, dense, 56);
PIN_SIZE(cdb_dev_output, 328);
PIN_OFF(cdb_dev_output, compact, 240);
PIN_OFF(cdb_dev_output, buckets, 248);
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

static int write_dump(cdb_ctx* ctx, cdb_merged* m, const char* path) {
  char* dump = NULL;
  size_t dlen = 0;
  if (cdb_merged_canonical_dump(ctx, m, &dump, &dlen) != CDB_OK) return 1;
  FILE* f = fopen(path, "wb");
  const int bad = !f || fwrite(dump, 1, dlen, f) != dlen;
  if (f) fclose(f);
  cdb_free(dump);
  return bad;
}

static void release_input(cdb_ctx* ctx, cdb_dev_input* in) {
  cdb_dev_rows_release(ctx, &in->keys);
  cdb_dev_rows_release(ctx, &in->nodes);
  cdb_dev_rows_release(ctx, &in->members);
}

/* The HBM-resident pull of INTEGRATION.md section 3, from C: replicas 0 and 1 decoded straight into
 * HBM (records layout) and merged into the bucket layout; that result becomes fold position 0 of a
 * second merge (cdb_dev_state_rows), replica 2 decoded into HBM and appended as position 1
 * (cdb_dev_input_append); the host view of the second result (bytes resolved through the first
 * result's host view and replica 2's batch) is dumped to `path` for the caller to compare with the
 * oracle's fold of replicas 0, 1, 2. */
static int device_chain(cdb_ctx* ctx, const cdb_gen_config* cfg, const char* path) {
  uint8_t* raw[3];
  size_t len[3];
  for (uint32_t r = 0; r < 3; ++r)
    if (cdb_gen_snapshot(cfg, r, &raw[r], &len[r]) != CDB_OK) return 20;
  cdb_batch* b1[2];
  cdb_batch* b2[1];
  cdb_dev_input d1, d2;
  uint32_t failed = 0;
  size_t off = 0;
  cdb_status st = cdb_decode_snapshots_device(ctx, (const uint8_t* const*)raw, len, 2, CDB_DECODE_ROWS_RECORDS, b1,
                                              &d1, &failed, &off, NULL, NULL);
  if (st != CDB_OK || d1.keys.stride != 6 || d1.nodes.stride != 5) return 21;
  st = cdb_decode_snapshots_device(ctx, (const uint8_t* const*)&raw[2], &len[2], 1, CDB_DECODE_ROWS_RECORDS, b2, &d2,
                                   &failed, &off, NULL, NULL);
  if (st != CDB_OK) return 22;
  cdb_merge_opts opts;
  memset(&opts, 0, sizeof opts);
  cdb_merge_stats s1, s2;
  cdb_dev_output o1;
  memset(&o1, 0, sizeof o1);
  o1.compact = 0; /* the bucket layout */
  if ((st = cdb_merge_device(ctx, &d1, &opts, &o1, &s1, NULL)) != CDB_OK) {
    fprintf(stderr, "merge 1: %d %s\n", (int)st, cdb_last_error(ctx));
    return 23;
  }
  if (o1.keys.stride != 8 || o1.buckets.nb == 0 || o1.keys.n != s1.key_rows_out) return 24;
  cdb_merged* h1 = NULL;
  if (cdb_merged_from_device(ctx, NULL, b1, 2, &o1, &h1) != CDB_OK) return 25;
  /* position 0: merge 1's result (one run); position 1: replica 2 */
  cdb_dev_input in;
  memset(&in, 0, sizeof in);
  if (cdb_dev_rows_alloc_records(ctx, &in.keys, o1.keys.n + d2.keys.n, 7) != CDB_OK ||
      cdb_dev_rows_alloc_records(ctx, &in.nodes, o1.nodes.n + d2.nodes.n, 6) != CDB_OK ||
      cdb_dev_rows_alloc_records(ctx, &in.members, o1.members.n + d2.members.n, 6) != CDB_OK)
    return 26;
  if (cdb_dev_state_rows(ctx, &o1, &in.keys, &in.nodes, &in.members, NULL) != CDB_OK) return 27;
  in.n_pos = 1;
  in.n_runs = 1;
  in.run_start[0][1] = in.keys.n;
  in.run_start[1][1] = in.nodes.n;
  in.run_start[2][1] = in.members.n;
  if (cdb_dev_input_append(ctx, &in, &d2, 1, NULL) != CDB_OK || in.n_pos != 2) return 28;
  cdb_dev_output o2;
  memset(&o2, 0, sizeof o2);
  if ((st = cdb_merge_device(ctx, &in, &opts, &o2, &s2, NULL)) != CDB_OK) {
    fprintf(stderr, "merge 2: %d %s\n", (int)st, cdb_last_error(ctx));
    return 29;
  }
  cdb_merged* h2 = NULL;
  if (cdb_merged_from_device(ctx, h1, b2, 1, &o2, &h2) != CDB_OK) return 30;
  if (write_dump(ctx, h2, path)) return 31;
  printf("device chain: %llu + %llu key rows -> %llu (sorted runs %llu)\n", (unsigned long long)s1.key_rows_in,
         (unsigned long long)d2.keys.n, (unsigned long long)s2.key_rows_out, (unsigned long long)s2.sorted_runs);
  cdb_merged_free(h2);
  cdb_merged_free(h1);
  release_input(ctx, &in);
  release_input(ctx, &d1);
  release_input(ctx, &d2);
  cdb_batch_free(b1[0]);
  cdb_batch_free(b1[1]);
  cdb_batch_free(b2[0]);
  for (int r = 0; r < 3; ++r) cdb_free(raw[r]);
  return 0;
}

/* The multi-device context of INTEGRATION.md section 5 with two slots on device 0: replicas 0 and 1
 * on slot 0 (positions 0, 1), replica 2 on slot 1 (decoded at position 0, appended at position 2 so
 * that positions stay global across slots); one cdb_merge_sharded; slot d's host view dumped to
 * `prefix`.d (the caller merges the slots' dumps and compares with the oracle). */
static int sharded(const cdb_gen_config* cfg, const char* prefix) {
  const int devs[2] = {0, 0};
  cdb_ctx* ctx = NULL;
  if (cdb_ctx_create_multi(&ctx, 2, devs) != CDB_OK || cdb_ctx_device_count(ctx) != 2) return 40;
  cdb_ctx* c1 = cdb_ctx_shard(ctx, 1);
  uint8_t* raw[3];
  size_t len[3];
  for (uint32_t r = 0; r < 3; ++r)
    if (cdb_gen_snapshot(cfg, r, &raw[r], &len[r]) != CDB_OK) return 41;
  cdb_batch* bs[3];
  cdb_dev_input in[2], tmp;
  uint32_t failed = 0;
  size_t off = 0;
  if (cdb_decode_snapshots_device(ctx, (const uint8_t* const*)raw, len, 2, CDB_DECODE_ROWS_RECORDS, bs, &in[0], &failed,
                                  &off, NULL, NULL) != CDB_OK)
    return 42;
  if (cdb_decode_snapshots_device(c1, (const uint8_t* const*)&raw[2], &len[2], 1, CDB_DECODE_ROWS_RECORDS, &bs[2],
                                  &tmp, &failed, &off, NULL, NULL) != CDB_OK)
    return 43;
  memset(&in[1], 0, sizeof in[1]);
  if (cdb_dev_rows_alloc_records(c1, &in[1].keys, tmp.keys.n, 7) != CDB_OK ||
      cdb_dev_rows_alloc_records(c1, &in[1].nodes, tmp.nodes.n, 6) != CDB_OK ||
      cdb_dev_rows_alloc_records(c1, &in[1].members, tmp.members.n, 6) != CDB_OK)
    return 44;
  in[1].keys.n = in[1].nodes.n = in[1].members.n = 0;
  if (cdb_dev_input_append(c1, &in[1], &tmp, 2, NULL) != CDB_OK || in[1].n_pos != 3) return 45;
  cdb_merge_opts opts;
  memset(&opts, 0, sizeof opts);
  cdb_dev_output out[2];
  cdb_merge_stats st[2];
  cdb_exchange_stats xs;
  cdb_status s = cdb_merge_sharded(ctx, in, &opts, out, st, &xs);
  if (s != CDB_OK) {
    fprintf(stderr, "sharded: %d %s\n", (int)s, cdb_last_error(ctx));
    return 46;
  }
  if (xs.n_devices != 2 || xs.transport != 2) return 47;
  /* passing a slot's output back as an input is refused (it lives in the exchange workspace) */
  cdb_dev_input again[2];
  memcpy(again, in, sizeof again);
  again[0].keys = out[0].keys;
  again[0].keys.n = out[0].keys.n;
  again[0].n_runs = 0;
  if (cdb_merge_sharded(ctx, again, &opts, out, st, &xs) != CDB_BAD_ARGUMENT) return 48;
  if (cdb_merge_sharded(ctx, in, &opts, out, st, &xs) != CDB_OK) return 49;
  for (int d = 0; d < 2; ++d) {
    cdb_merged* h = NULL;
    if (cdb_merged_from_device(cdb_ctx_shard(ctx, d), NULL, bs, 3, &out[d], &h) != CDB_OK) return 50;
    char path[4096];
    snprintf(path, sizeof path, "%s.%d", prefix, d);
    if (write_dump(ctx, h, path)) return 51;
    cdb_merged_free(h);
  }
  printf("sharded: %llu + %llu key rows out, %llu transfers\n", (unsigned long long)st[0].key_rows_out,
         (unsigned long long)st[1].key_rows_out, (unsigned long long)xs.transfers);
  release_input(ctx, &in[0]);
  release_input(c1, &in[1]);
  release_input(c1, &tmp);
  for (int r = 0; r < 3; ++r) {
    cdb_batch_free(bs[r]);
    cdb_free(raw[r]);
  }
  cdb_ctx_destroy(ctx);
  return 0;
}

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
  int rc = 0;
  if (argc > 2 && (rc = device_chain(ctx, &cfg, argv[2])) != 0) return rc;
  cdb_ctx_destroy(ctx);
  if (argc > 3 && (rc = sharded(&cfg, argv[3])) != 0) return rc;
  return 0;
}
