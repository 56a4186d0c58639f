"""constdb_amd — MI355X-native batched CRDT merge engine for ConstDB's replica-sync path.

Thin ctypes mirror of the C ABI in ``include/cdb_merge.h`` (libcdbmerge.so: HIP kernels
for gfx950 + host C++). The product path is the HIP library: there is no CPU fallback —
merging without a visible gfx950 device raises ``NoDevice``.

Reference interface mirrored (fxsjy/ConstDB):
  * ``decode_snapshot``  ~ ``SnapshotLoader::next`` loop      (src/snapshot.rs:120-220)
  * ``DB.merge_snapshots`` ~ ``Puller::merge_replicates_in_main`` applying
    ``DB::merge_entry`` / ``DB::delete`` / ``DB::expire_at``    (src/replica/pull.rs:116-159)
  * errors ~ ``CstError`` (src/lib.rs:146-175)
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("CDB_LIB", os.path.join(_HERE, "libcdbmerge.so"))  # CDB_LIB: profiling builds

# ----------------------------------------------------------------- errors (lib.rs:146-175)
OK = 0
INVALID_SNAPSHOT = 1
INVALID_SNAPSHOT_CHECKSUM = 2
INVALID_TYPE = 3
IO_ERROR = 4
DICT_MERGE_UNIMPLEMENTED = 5
BAD_ARGUMENT = 6
DEVICE_ERROR = 7
OUT_OF_MEMORY = 8
NO_DEVICE = 9
INVALID_REQUEST_MSG = 10
NEED_MORE_MSG = 11

DECODE_REFERENCE_CHECKSUM = 1
MERGE_STRICT_DICT_PANIC = 1
MERGE_GC_DELETES = 2
MERGE_GC_MEMBERS = 4

GEN_NODE_PER_REPLICA = 1
GEN_OPS_ZIPF_MEMBERS = 2
GEN_OPS_TAGS_ONLY = 4
GEN_ROWS_RECORDS = 8
DECODE_ROWS_RECORDS = 2
DECODE_STREAM_ORDER = 4
DECODE_KEEP_BYTES = 8


class CstError(Exception):
    status = -1


class InvalidSnapshot(CstError):
    status = INVALID_SNAPSHOT

    def __init__(self, offset: int):
        super().__init__(f"invalid data in snapshot at offset {offset}")
        self.offset = offset


class InvalidSnapshotChecksum(CstError):
    status = INVALID_SNAPSHOT_CHECKSUM


class InvalidType(CstError):
    status = INVALID_TYPE


class IoError(CstError):
    status = IO_ERROR


class DictMergeUnimplemented(CstError):
    status = DICT_MERGE_UNIMPLEMENTED


class InvalidRequestMsg(CstError):
    status = INVALID_REQUEST_MSG

    def __init__(self, offset: int):
        super().__init__(f"malformed RESP message at offset {offset}")
        self.offset = offset


class NeedMoreMsg(CstError):
    status = NEED_MORE_MSG


class NoDevice(CstError):
    status = NO_DEVICE


class DeviceError(CstError):
    status = DEVICE_ERROR


_ERRORS = {INVALID_SNAPSHOT_CHECKSUM: InvalidSnapshotChecksum, INVALID_TYPE: InvalidType,
           IO_ERROR: IoError, DICT_MERGE_UNIMPLEMENTED: DictMergeUnimplemented, NO_DEVICE: NoDevice,
           DEVICE_ERROR: DeviceError, OUT_OF_MEMORY: DeviceError, BAD_ARGUMENT: ValueError,
           NEED_MORE_MSG: NeedMoreMsg}


def _raise(st: int, msg: str = "", offset: int = 0):
    if st == INVALID_SNAPSHOT:
        raise InvalidSnapshot(offset)
    if st == INVALID_REQUEST_MSG:
        raise InvalidRequestMsg(offset)
    cls = _ERRORS.get(st, CstError)
    raise cls(msg or f"cdb status {st}")


# ----------------------------------------------------------------- ctypes structs
class BatchInfo(ctypes.Structure):
    _fields_ = [("n_data", ctypes.c_uint64), ("n_expires", ctypes.c_uint64), ("n_deletes", ctypes.c_uint64),
                ("n_nodes", ctypes.c_uint64), ("n_members", ctypes.c_uint64), ("node_id", ctypes.c_uint64),
                ("uuid_he_sent", ctypes.c_uint64), ("n_replica_add", ctypes.c_uint32),
                ("n_replica_del", ctypes.c_uint32), ("version", ctypes.c_char * 16)]


class MergeOpts(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32), ("force_tier", ctypes.c_uint32), ("gc_watermark", ctypes.c_uint64),
                ("key_shift", ctypes.c_uint32), ("pipe_ranges", ctypes.c_uint32)]


class MergeStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "key_rows_in", "node_rows_in", "member_rows_in", "key_rows_out", "node_rows_out", "member_rows_out",
        "type_conflicts", "dict_merges", "deletes_gced", "members_gced", "duplicate_rows", "orphan_children",
        "hot_buckets", "wide_buckets", "mid_buckets")] + [(n, ctypes.c_double) for n in (
        "device_ms", "partition_ms", "bucket_ms", "finish_ms")] + [("sorted_runs", ctypes.c_uint64),
                                                                  ("hot_slow_runs", ctypes.c_uint64),
                                                                  ("hot_merged_children", ctypes.c_uint64),
                                                                  ("wave_pipe_buckets", ctypes.c_uint64),
                                                                  ("wave_pipe_units", ctypes.c_uint64)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class ReplicaEntry(ctypes.Structure):
    _fields_ = [("addr", ctypes.c_char_p), ("alias", ctypes.c_char_p), ("node_id", ctypes.c_uint64),
                ("uuid_he_sent", ctypes.c_uint64), ("add_time", ctypes.c_uint64), ("del_time", ctypes.c_uint64),
                ("has_add", ctypes.c_uint32), ("has_del", ctypes.c_uint32)]


class EncodeHeader(ctypes.Structure):
    _fields_ = [("node_id", ctypes.c_uint64), ("alias", ctypes.c_char_p), ("alias_len", ctypes.c_size_t),
                ("addr", ctypes.c_char_p), ("addr_len", ctypes.c_size_t), ("last_uuid", ctypes.c_uint64),
                ("replicas", ctypes.POINTER(ReplicaEntry)), ("n_replicas", ctypes.c_size_t)]


class EncodeStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("bytes", "data_entries", "expires", "deletes", "checksum")] + \
               [(n, ctypes.c_double) for n in ("upload_ms", "device_ms", "crc_ms", "download_ms")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class OpsInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "n_messages", "n_ops", "n_node_args", "n_member_args", "applied", "duplicates", "lost", "unknown",
        "unsupported", "cmd_errors", "replacks", "uuid_he_sent", "uuid_he_acked")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class ApplyStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "ops_in", "node_args_in", "member_args_in", "key_rows_in", "key_rows_out", "node_rows_out",
        "member_rows_out", "type_errors", "expired_on_query")] + [("device_ms", ctypes.c_double)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class DevRows(ctypes.Structure):
    """cdb_dev_rows: plain columns (stride 0), the records layout (col[0] the hash column, fields
    1.. one record of `stride` words per row), or a merge's bucket-layout rows (stride0 = stride)."""
    _fields_ = [("col", ctypes.c_void_p * 8), ("n", ctypes.c_uint64), ("stride", ctypes.c_uint32),
                ("stride0", ctypes.c_uint32)]


class DevBuckets(ctypes.Structure):
    """cdb_dev_buckets: a bucket-layout result's directory (library-owned)."""
    _fields_ = [("nb", ctypes.c_uint64), ("first", ctypes.c_void_p * 3), ("count", ctypes.c_void_p * 3),
                ("dense", ctypes.c_void_p * 3)]


MAX_RUNS = 64


class DevInput(ctypes.Structure):
    _fields_ = [("keys", DevRows), ("nodes", DevRows), ("members", DevRows), ("n_pos", ctypes.c_uint32),
                ("n_runs", ctypes.c_uint32), ("run_start", (ctypes.c_uint64 * (MAX_RUNS + 1)) * 3)]


class DevOutput(ctypes.Structure):
    _fields_ = [("keys", DevRows), ("nodes", DevRows), ("members", DevRows), ("compact", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("buckets", DevBuckets)]


class ExchangeStats(ctypes.Structure):
    """cdb_exchange_stats: the sharded merge's split / exchange / merge figures."""
    _fields_ = [("n_devices", ctypes.c_uint32), ("transport", ctypes.c_uint32), ("packed", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)] + [(n, ctypes.c_double) for n in (
                    "split_ms", "exchange_ms", "merge_ms", "total_ms")] + [(n, ctypes.c_uint64) for n in (
                    "bytes_moved", "bytes_local", "transfers")] + [("link_bytes", (ctypes.c_uint64 * 8) * 8)]

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_ if n not in ("link_bytes", "reserved")}
        k = self.n_devices
        d["link_bytes"] = [[self.link_bytes[i][j] for j in range(k)] for i in range(k)]
        return d


class GenConfig(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("universe", ctypes.c_uint64)] + [(n, ctypes.c_uint32) for n in (
        "n_replicas", "key_permille", "mix_bytes", "mix_counter", "mix_set", "mix_dict", "conflict_ppm",
        "tie_permille", "max_nodes", "mean_members", "member_universe", "del_permille", "side_permille",
        "value_min", "value_max", "shard", "n_shards", "replica_lo", "replica_hi", "flags", "hot_zipf_milli",
        "stream")] + [("hot_events", ctypes.c_uint64)]


# exported C-ABI function names (tests check the .so exports every one of them)
ABI_FUNCTIONS = (
    "cdb_ctx_create", "cdb_ctx_destroy", "cdb_last_error", "cdb_decode_snapshot", "cdb_decode_snapshot_gpu",
    "cdb_batch_info_get",
    "cdb_batch_column", "cdb_batch_free", "cdb_merge", "cdb_merged_canonical_dump", "cdb_merged_replicas",
    "cdb_merged_free", "cdb_free",
    "cdb_dev_rows_alloc", "cdb_dev_rows_release", "cdb_merge_device", "cdb_partition_owner", "cdb_gen_default",
    "cdb_gen_snapshot", "cdb_gen_device", "cdb_decode_ops", "cdb_ops_info_get", "cdb_ops_free", "cdb_apply_ops", "cdb_gen_ops",
    "cdb_encode_snapshot", "cdb_encode_device", "cdb_crc64_gpu", "cdb_upload_batches", "cdb_decode_snapshots_device",
    "cdb_decode_ops_gpu", "cdb_ops_column", "cdb_snapshot_index_selftest", "cdb_merge_into",
    "cdb_merged_from_device", "cdb_dev_state_rows", "cdb_ctx_create_multi", "cdb_ctx_device_count",
    "cdb_ctx_shard", "cdb_merge_sharded", "cdb_dev_rows_alloc_records", "cdb_dev_output_compact",
    "cdb_dev_input_append", "cdb_shard_splits", "cdb_shard_recv_plan", "cdb_merged_gc", "cdb_merged_garbage_count")

_lib = None


def _take(addr: int, n: int) -> bytes:
    """n bytes at addr as a bytes object (ctypes.string_at takes a C int size: at most 2 GiB)."""
    return bytes((ctypes.c_char * n).from_address(addr)) if n else b""


def lib_path() -> str:
    return _LIB_PATH


def lib():
    """Loads libcdbmerge.so. Raises OSError when it was not built (see __graft_entry__.build)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise OSError(f"{_LIB_PATH} missing: build it with `python constdb_amd/build.py`")
    # NOTE: torch bundles its own libamdhip64.so.7 / libhsa-runtime64.so.1. A process that
    # uses torch's GPU runtime AND this library must import torch first, so that our
    # DT_NEEDED (soname libamdhip64.so.7) binds to the runtime torch already mapped; two
    # HSA runtimes in one process do not share the GPU (see constdb_amd/dist.py, tests).
    L = ctypes.CDLL(_LIB_PATH)
    vp, c_st = ctypes.c_void_p, ctypes.c_int
    P = ctypes.POINTER
    sig = {
        "cdb_ctx_create": (c_st, [P(vp), ctypes.c_int]),
        "cdb_ctx_create_multi": (c_st, [P(vp), ctypes.c_int, P(ctypes.c_int)]),
        "cdb_ctx_device_count": (ctypes.c_int, [vp]),
        "cdb_ctx_shard": (vp, [vp, ctypes.c_int]),
        "cdb_merge_sharded": (c_st, [vp, P(DevInput), P(MergeOpts), P(DevOutput), P(MergeStats), P(ExchangeStats)]),
        "cdb_ctx_destroy": (None, [vp]),
        "cdb_last_error": (ctypes.c_char_p, [vp]),
        "cdb_decode_snapshot": (c_st, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, P(vp),
                                       P(ctypes.c_size_t)]),
        "cdb_decode_snapshot_gpu": (c_st, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, P(vp),
                                           P(ctypes.c_size_t), P(ctypes.c_double), P(ctypes.c_double)]),
        "cdb_batch_info_get": (c_st, [vp, P(BatchInfo)]),
        "cdb_batch_column": (c_st, [vp, ctypes.c_int, ctypes.c_int, P(P(ctypes.c_uint64)), P(ctypes.c_uint64)]),
        "cdb_batch_free": (None, [vp]),
        "cdb_merge": (c_st, [vp, P(vp), ctypes.c_uint32, P(MergeOpts), P(vp), P(MergeStats)]),
        "cdb_merged_canonical_dump": (c_st, [vp, vp, P(vp), P(ctypes.c_size_t)]),
        "cdb_merge_into": (c_st, [vp, vp, P(vp), ctypes.c_uint32, P(MergeOpts), P(vp), P(MergeStats)]),
        "cdb_merged_from_device": (c_st, [vp, vp, P(vp), ctypes.c_uint32, P(DevOutput), P(vp)]),
        "cdb_merged_gc": (c_st, [vp, vp, ctypes.c_uint64, P(ctypes.c_uint64)]),
        "cdb_merged_garbage_count": (ctypes.c_uint64, [vp]),
        "cdb_dev_state_rows": (c_st, [vp, P(DevOutput), P(DevRows), P(DevRows), P(DevRows), vp]),
        "cdb_merged_replicas": (c_st, [vp, P(P(ReplicaEntry)), P(ctypes.c_size_t)]),
        "cdb_merged_free": (None, [vp]),
        "cdb_free": (None, [vp]),
        "cdb_dev_rows_alloc": (c_st, [vp, P(DevRows), ctypes.c_uint64, ctypes.c_int]),
        "cdb_dev_rows_alloc_records": (c_st, [vp, P(DevRows), ctypes.c_uint64, ctypes.c_int]),
        "cdb_dev_output_compact": (c_st, [vp, P(DevOutput), P(DevOutput), vp]),
        "cdb_dev_input_append": (c_st, [vp, P(DevInput), P(DevInput), ctypes.c_uint32, vp]),
        "cdb_shard_splits": (c_st, [P(ctypes.c_uint64), P(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_uint32,
                                    P(ctypes.c_uint64)]),
        "cdb_shard_recv_plan": (c_st, [ctypes.c_uint32, P(ctypes.c_uint32), P(ctypes.c_uint64), ctypes.c_uint32,
                                       P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32),
                                       P(ctypes.c_uint64), P(ctypes.c_uint64)]),
        "cdb_dev_rows_release": (None, [vp, P(DevRows)]),
        "cdb_merge_device": (c_st, [vp, P(DevInput), P(MergeOpts), P(DevOutput), P(MergeStats), vp]),
        "cdb_partition_owner": (c_st, [vp, P(DevRows), ctypes.c_int, ctypes.c_int, P(DevRows), P(ctypes.c_uint64), vp]),
        "cdb_gen_default": (None, [P(GenConfig)]),
        "cdb_gen_snapshot": (c_st, [P(GenConfig), ctypes.c_uint32, P(vp), P(ctypes.c_size_t)]),
        "cdb_gen_device": (c_st, [vp, P(GenConfig), P(DevInput)]),
        "cdb_decode_ops": (c_st, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, P(vp), P(ctypes.c_size_t)]),
        "cdb_ops_info_get": (c_st, [vp, P(OpsInfo)]),
        "cdb_decode_ops_gpu": (c_st, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, P(vp),
                                      P(ctypes.c_size_t), P(ctypes.c_double), P(ctypes.c_double),
                                      P(ctypes.c_uint32)]),
        "cdb_ops_column": (c_st, [vp, ctypes.c_int, ctypes.c_int, P(P(ctypes.c_uint64)), P(ctypes.c_uint64)]),
        "cdb_snapshot_index_selftest": (c_st, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                               P(ctypes.c_uint64)]),
        "cdb_ops_free": (None, [vp]),
        "cdb_gen_ops": (c_st, [P(GenConfig), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, P(vp),
                               P(ctypes.c_size_t)]),
        "cdb_apply_ops": (c_st, [vp, vp, vp, P(vp), P(ApplyStats)]),
        "cdb_encode_snapshot": (c_st, [vp, vp, P(EncodeHeader), P(vp), P(ctypes.c_size_t), P(EncodeStats)]),
        "cdb_encode_device": (c_st, [vp, P(DevOutput), P(vp), ctypes.c_uint32, P(EncodeHeader), P(vp),
                                     P(ctypes.c_size_t), P(EncodeStats)]),
        "cdb_crc64_gpu": (c_st, [vp, ctypes.c_char_p, ctypes.c_size_t, P(ctypes.c_uint64)]),
        "cdb_upload_batches": (c_st, [vp, P(vp), ctypes.c_uint32, P(DevInput)]),
        "cdb_decode_snapshots_device": (c_st, [vp, P(ctypes.c_char_p), P(ctypes.c_size_t), ctypes.c_uint32,
                                               ctypes.c_uint32, P(vp), P(DevInput), P(ctypes.c_uint32),
                                               P(ctypes.c_size_t), P(ctypes.c_double), P(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def crc64_gpu(ctx: "Context", data: bytes) -> int:
    """CRC-64/Jones of `data` computed by the GPU checksum kernels (cdb_crc64_gpu)."""
    c = ctypes.c_uint64()
    ctx.check(lib().cdb_crc64_gpu(ctx.handle, data, len(data), ctypes.byref(c)))
    return c.value


# ----------------------------------------------------------------- context
class Context:
    """A device context (cdb_ctx). Needs a visible gfx950 GPU; raises NoDevice otherwise.
    Context(devices=[...]) is a multi-device context (cdb_ctx_create_multi): one engine context per
    device slot, RCCL between distinct devices; shard(i) is slot i's context."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None, _borrowed=None):
        self._ctx = ctypes.c_void_p()
        self._owner = None
        if _borrowed is not None:  # a slot of a multi-device context (owned by it)
            self._ctx, self._owner = ctypes.c_void_p(_borrowed[0]), _borrowed[1]
            self.device = device
            return
        if devices is None:
            st = lib().cdb_ctx_create(ctypes.byref(self._ctx), device)
            self.device = device
        else:
            arr = (ctypes.c_int * len(devices))(*devices)
            st = lib().cdb_ctx_create_multi(ctypes.byref(self._ctx), len(devices), arr)
            self.device = devices[0]
        if st != OK:
            why = lib().cdb_last_error(None).decode(errors="replace") if devices is not None else ""
            _raise(st, why or ("no HIP device" if st == NO_DEVICE else "cdb_ctx_create failed"))

    @property
    def n_devices(self) -> int:
        return lib().cdb_ctx_device_count(self._ctx)

    def shard(self, i: int) -> "Context":
        h = lib().cdb_ctx_shard(self._ctx, i)
        if not h:
            raise IndexError(i)
        return Context(device=-1, _borrowed=(h, self))

    @property
    def handle(self):
        return self._ctx

    def last_error(self) -> str:
        return (lib().cdb_last_error(self._ctx) or b"").decode()

    def check(self, st: int):
        if st != OK:
            _raise(st, self.last_error())

    def close(self):
        if self._ctx and self._owner is None:
            lib().cdb_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ----------------------------------------------------------------- decode
class Batch:
    """A decoded snapshot (cdb_batch): columnar rows + byte arena, host resident."""

    def __init__(self, handle, checksum_ok: bool = True):
        self._h = handle
        self.checksum_ok = checksum_ok

    @property
    def handle(self):
        return self._h

    def info(self) -> BatchInfo:
        bi = BatchInfo()
        lib().cdb_batch_info_get(self._h, ctypes.byref(bi))
        return bi

    def column(self, family: int, col: int):
        """(numpy-free) list of the u64 values of one decoded column."""
        ptr = ctypes.POINTER(ctypes.c_uint64)()
        n = ctypes.c_uint64()
        st = lib().cdb_batch_column(self._h, family, col, ctypes.byref(ptr), ctypes.byref(n))
        if st != OK:
            _raise(st)
        return [ptr[i] for i in range(n.value)]

    def column_array(self, family: int, col: int):
        import numpy as np
        ptr = ctypes.POINTER(ctypes.c_uint64)()
        n = ctypes.c_uint64()
        st = lib().cdb_batch_column(self._h, family, col, ctypes.byref(ptr), ctypes.byref(n))
        if st != OK:
            _raise(st)
        if n.value == 0:
            return np.zeros(0, dtype=np.uint64)
        return np.ctypeslib.as_array(ptr, shape=(n.value,)).copy()

    def __del__(self):
        try:
            if self._h:
                lib().cdb_batch_free(self._h)
                self._h = None
        except Exception:
            pass


def decode_snapshot(data: bytes, reference_checksum: bool = False, allow_bad_checksum: bool = False) -> Batch:
    """Decodes one snapshot (writer layout, server.rs:183-215). Mirrors the loader's errors:
    InvalidSnapshot(offset) / InvalidSnapshotChecksum / InvalidType / IoError."""
    h = ctypes.c_void_p()
    off = ctypes.c_size_t()
    flags = DECODE_REFERENCE_CHECKSUM if reference_checksum else 0
    st = lib().cdb_decode_snapshot(None, bytes(data), len(data), flags, ctypes.byref(h), ctypes.byref(off))
    if st == INVALID_SNAPSHOT_CHECKSUM and allow_bad_checksum and h:
        return Batch(h, checksum_ok=False)
    if st != OK:
        if h:
            lib().cdb_batch_free(h)
        _raise(st, offset=off.value)
    return Batch(h)


def decode_snapshot_gpu(ctx: "Context", data: bytes, reference_checksum: bool = False,
                        allow_bad_checksum: bool = False, timing: Optional[dict] = None) -> Batch:
    """decode_snapshot with the per-entry work on the GPU (cdb_decode_snapshot_gpu, SURVEY
    §8f.1): same batch, same errors. `timing` (a dict) receives index_ms / device_ms."""
    h = ctypes.c_void_p()
    off = ctypes.c_size_t()
    ims, dms = ctypes.c_double(), ctypes.c_double()
    flags = DECODE_REFERENCE_CHECKSUM if reference_checksum else 0
    st = lib().cdb_decode_snapshot_gpu(ctx.handle, bytes(data), len(data), flags, ctypes.byref(h), ctypes.byref(off),
                                       ctypes.byref(ims), ctypes.byref(dms))
    if timing is not None:
        timing.update(index_ms=ims.value, device_ms=dms.value)
    if st == INVALID_SNAPSHOT_CHECKSUM and allow_bad_checksum and h:
        return Batch(h, checksum_ok=False)
    if st != OK:
        if h:
            lib().cdb_batch_free(h)
        _raise(st, ctx.last_error(), offset=off.value)
    return Batch(h)


def decode_snapshots_device(ctx: "Context", snaps, reference_checksum: bool = False,
                            timing: Optional[dict] = None, records: bool = False, stream_order: bool = False,
                            keep_bytes: bool = False):
    """GPU decode of several snapshots straight into HBM (cdb_decode_snapshots_device):
    returns (batches, DevInput) -- the rows of snapshot i at fold position i in one set of
    device columns (release each family with cdb_dev_rows_release), each batch holding the
    host side (bytes, references, header). Errors are raised for the failing snapshot. records: the rows
    in the records layout (cdb_dev_rows.stride) instead of columns; keep_bytes: the snapshot bytes
    stay in HBM with the batches (cdb_encode_device). A snapshot may also be a CPU uint8 tensor
    (for instance page-locked memory): its bytes are passed in place."""
    n = len(snaps)
    for x in snaps:
        if hasattr(x, "data_ptr") and not (getattr(x, "device", None) is not None and x.device.type == "cpu"
                                           and str(x.dtype) == "torch.uint8" and x.is_contiguous()):
            raise TypeError("a snapshot tensor must be a contiguous CPU uint8 tensor (its bytes are read on the host)")
    datas = [x if hasattr(x, "data_ptr") else bytes(x) for x in snaps]
    bufs = (ctypes.c_char_p * max(n, 1))(*[ctypes.cast(x.data_ptr(), ctypes.c_char_p) if hasattr(x, "data_ptr")
                                           else x for x in datas])
    lens = (ctypes.c_size_t * max(n, 1))(*[x.numel() if hasattr(x, "data_ptr") else len(x) for x in datas])
    hs = (ctypes.c_void_p * max(n, 1))()
    din = DevInput()
    failed = ctypes.c_uint32()
    off = ctypes.c_size_t()
    ims, dms = ctypes.c_double(), ctypes.c_double()
    flags = ((DECODE_REFERENCE_CHECKSUM if reference_checksum else 0) | (DECODE_ROWS_RECORDS if records else 0)
             | (DECODE_STREAM_ORDER if stream_order else 0) | (DECODE_KEEP_BYTES if keep_bytes else 0))
    st = lib().cdb_decode_snapshots_device(ctx.handle, bufs, lens, n, flags, hs, ctypes.byref(din),
                                           ctypes.byref(failed), ctypes.byref(off), ctypes.byref(ims),
                                           ctypes.byref(dms))
    if timing is not None:
        timing.update(index_ms=ims.value, device_ms=dms.value, failed=failed.value)
    batches = [Batch(hs[i], checksum_ok=not (st == INVALID_SNAPSHOT_CHECKSUM and i == failed.value))
               for i in range(n) if hs[i]]
    if st not in (OK, INVALID_SNAPSHOT_CHECKSUM):
        _raise(st, ctx.last_error(), offset=off.value)
    return batches, din


def _encode_header(node_id, alias, addr, last_uuid, replicas, keep, rep=None):
    """A cdb_encode_header; `replicas` None or a list of dicts in the shape Merged.replicas()
    returns, or `rep` = (ReplicaEntry pointer, count) as cdb_merged_replicas gives. `keep` holds the
    buffers the header points into."""
    if rep is None:
        if not replicas:
            rep = (ctypes.POINTER(ReplicaEntry)(), 0)
        else:
            arr = (ReplicaEntry * len(replicas))()
            for i, d in enumerate(replicas):
                e = arr[i]
                a = d["addr"].encode()
                keep.append(a)
                e.addr = a
                if "add" in d:
                    t, nid, al, uuid = d["add"]
                    al = al.encode()
                    keep.append(al)
                    e.has_add, e.add_time, e.node_id, e.alias, e.uuid_he_sent = 1, t, nid, al, uuid
                else:
                    e.alias = b""
                if "del" in d:
                    e.has_del, e.del_time = 1, d["del"]
            keep.append(arr)
            rep = (ctypes.cast(arr, ctypes.POINTER(ReplicaEntry)), len(replicas))
    a, ad = alias.encode(), addr.encode()
    keep += [a, ad]
    return EncodeHeader(node_id, a, len(a), ad, len(ad), last_uuid, rep[0], rep[1])


def _take_bytes(out, n):
    try:
        return _take(out.value, n.value)
    finally:
        lib().cdb_free(out)


def encode_device(ctx: "Context", out: "DevOutput", batches, node_id: int = 1, alias: str = "n1",
                  addr: str = "127.0.0.1:9001", last_uuid: int = 0, replicas=None):
    """cdb_encode_device: a cdb_merge_device result (either output layout) written as a snapshot
    from HBM, fold position i resolving through batches[i]. Returns (bytes, EncodeStats)."""
    keep = []
    hdr = _encode_header(node_id, alias, addr, last_uuid, replicas, keep)
    hs = (ctypes.c_void_p * max(len(batches), 1))(*[b.handle for b in batches])
    o = ctypes.c_void_p()
    n = ctypes.c_size_t()
    st = EncodeStats()
    ctx.check(lib().cdb_encode_device(ctx.handle, ctypes.byref(out), hs, len(batches), ctypes.byref(hdr),
                                      ctypes.byref(o), ctypes.byref(n), ctypes.byref(st)))
    return _take_bytes(o, n), st


# ----------------------------------------------------------------- op stream
class Ops:
    """A decoded replicate stream (cdb_ops): op rows in stream order + the stream bytes."""

    def __init__(self, handle, complete: bool = True, consumed: int = 0):
        self._h = handle
        self.complete = complete
        self.consumed = consumed

    @property
    def handle(self):
        return self._h

    def info(self) -> OpsInfo:
        i = OpsInfo()
        lib().cdb_ops_info_get(self._h, ctypes.byref(i))
        return i

    def column(self, family: int, col: int):
        """A copy of one column as a numpy uint64 array (cdb_ops_column: byte references come as
        (offset, length) pairs)."""
        import numpy as np
        data = ctypes.POINTER(ctypes.c_uint64)()
        n = ctypes.c_uint64()
        st = lib().cdb_ops_column(self._h, family, col, ctypes.byref(data), ctypes.byref(n))
        if st != OK:
            _raise(st)
        if n.value == 0:
            return np.zeros(0, dtype=np.uint64)
        return np.ctypeslib.as_array(data, shape=(n.value,)).copy()

    def __del__(self):
        try:
            if self._h:
                lib().cdb_ops_free(self._h)
                self._h = None
        except Exception:
            pass


def decode_ops(data: bytes, uuid_he_sent: int, allow_partial: bool = False) -> Ops:
    """cdb_decode_ops (replica/pull.rs:184-235 up to the handlers): RESP framing, the uuid gate
    and argument parsing. Raises InvalidRequestMsg(offset) on malformed RESP; a stream that ends
    inside a message raises NeedMoreMsg unless allow_partial (then .complete is False and
    .consumed the bytes used)."""
    h = ctypes.c_void_p()
    off = ctypes.c_size_t()
    st = lib().cdb_decode_ops(None, bytes(data), len(data), uuid_he_sent, ctypes.byref(h), ctypes.byref(off))
    if st == NEED_MORE_MSG and allow_partial and h:
        return Ops(h, complete=False, consumed=off.value)
    if st != OK:
        if h:
            lib().cdb_ops_free(h)
        _raise(st, offset=off.value)
    return Ops(h, consumed=len(data))


def decode_ops_gpu(ctx: "Context", data: bytes, uuid_he_sent: int, allow_partial: bool = False,
                   timing: Optional[dict] = None) -> Ops:
    """cdb_decode_ops_gpu: the same decode with the per-message work on the GPU. timing (a dict)
    receives host_ms, device_ms and used_gpu."""
    h = ctypes.c_void_p()
    off = ctypes.c_size_t()
    hm, dm, ug = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint32()
    st = lib().cdb_decode_ops_gpu(ctx.handle, bytes(data), len(data), uuid_he_sent, ctypes.byref(h), ctypes.byref(off),
                                  ctypes.byref(hm), ctypes.byref(dm), ctypes.byref(ug))
    if timing is not None:
        timing.update(host_ms=hm.value, device_ms=dm.value, used_gpu=bool(ug.value))
    if st == NEED_MORE_MSG and allow_partial and h:
        return Ops(h, complete=False, consumed=off.value)
    if st != OK:
        if h:
            lib().cdb_ops_free(h)
        _raise(st, offset=off.value)
    return Ops(h, consumed=len(data))


# ----------------------------------------------------------------- merge
class Merged:
    """A merge result (cdb_merged)."""

    def __init__(self, ctx: Context, handle, stats: MergeStats, inputs: Sequence[Batch]):
        self._ctx = ctx
        self._h = handle
        self.stats = stats
        self._inputs = list(inputs)   # keep the byte arenas alive

    @property
    def handle(self):
        return self._h

    def canonical_dump(self) -> bytes:
        out = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._ctx.check(lib().cdb_merged_canonical_dump(self._ctx.handle, self._h, ctypes.byref(out),
                                                        ctypes.byref(n)))
        try:
            return _take(out.value, n.value) if n.value else b""
        finally:
            lib().cdb_free(out)

    def replicas(self):
        """The merged replica table (cdb_merged_replicas, replica/pull.rs:131-156): one dict per
        addr, sorted by addr, with the LWWHash add tag (node_id, alias, uuid_he_sent,
        add_time) and/or del tag (del_time)."""
        ptr = ctypes.POINTER(ReplicaEntry)()
        n = ctypes.c_size_t()
        self._ctx.check(lib().cdb_merged_replicas(self._h, ctypes.byref(ptr), ctypes.byref(n)))
        out = []
        for i in range(n.value):
            e = ptr[i]
            d = {"addr": e.addr.decode()}
            if e.has_add:
                d["add"] = (e.add_time, e.node_id, e.alias.decode(), e.uuid_he_sent)
            if e.has_del:
                d["del"] = e.del_time
            out.append(d)
        return out

    def encode_snapshot(self, node_id: int = 1, alias: str = "n1", addr: str = "127.0.0.1:9001",
                        last_uuid: int = 0, replicas="merged"):
        """cdb_encode_snapshot: this result in the reference's snapshot wire format
        (Server::dump_all, server.rs:183-215), laid out and checksummed on the GPU. `replicas`:
        "merged" (this result's replica table, cdb_merged_replicas), None, or a list of dicts in
        the shape replicas() returns. Returns (bytes, EncodeStats)."""
        keep = []
        if replicas == "merged":
            ptr = ctypes.POINTER(ReplicaEntry)()
            n = ctypes.c_size_t()
            self._ctx.check(lib().cdb_merged_replicas(self._h, ctypes.byref(ptr), ctypes.byref(n)))
            hdr = _encode_header(node_id, alias, addr, last_uuid, None, keep, rep=(ptr, n.value))
        else:
            hdr = _encode_header(node_id, alias, addr, last_uuid, replicas, keep)
        out = ctypes.c_void_p()
        n = ctypes.c_size_t()
        st = EncodeStats()
        self._ctx.check(lib().cdb_encode_snapshot(self._ctx.handle, self._h, ctypes.byref(hdr), ctypes.byref(out),
                                                  ctypes.byref(n), ctypes.byref(st)))
        return _take_bytes(out, n), st

    def gc(self, tombstone: int) -> int:
        """cdb_merged_gc: DB::gc(tombstone) (db.rs:82-119) on this result, in place, over the garbage
        list it keeps (DB::garbages across merge_into chains). Returns the Deletes rows removed."""
        removed = ctypes.c_uint64()
        self._ctx.check(lib().cdb_merged_gc(self._ctx.handle, self._h, tombstone, ctypes.byref(removed)))
        return removed.value

    @property
    def garbage_count(self) -> int:
        return lib().cdb_merged_garbage_count(self._h)

    def apply_ops(self, ops: "Ops") -> "Merged":
        """cdb_apply_ops: the op stream applied on the device on top of this result (SURVEY
        §8f.2). Returns a new result; this one is unchanged."""
        st = ApplyStats()
        h = ctypes.c_void_p()
        self._ctx.check(lib().cdb_apply_ops(self._ctx.handle, self._h, ops.handle, ctypes.byref(h), ctypes.byref(st)))
        m = Merged(self._ctx, h, self.stats, self._inputs + [ops])
        m.apply_stats = st
        return m

    def __del__(self):
        try:
            if self._h:
                lib().cdb_merged_free(self._h)
                self._h = None
        except Exception:
            pass


class DB:
    """Batched stand-in for the reference DB's replica-sync entry point.

    ``merge_snapshots([local, remote1, ...])`` has the effect of folding each snapshot, in
    order, through DB::merge_entry / DB::delete / DB::expire_at (replica/pull.rs:120-158),
    optionally followed by DB::gc(watermark) (db.rs:82-119)."""

    def __init__(self, ctx: Optional[Context] = None, device: int = 0):
        self.ctx = ctx or Context(device)

    def merge_batches(self, batches: Sequence[Batch], strict_dict_panic: bool = False,
                      gc_watermark: Optional[int] = None, gc_members: bool = False,
                      force_tier: int = 0, pipe_ranges: int = 0) -> Merged:
        n = len(batches)
        arr = (ctypes.c_void_p * max(n, 1))(*[b.handle for b in batches])
        opts = merge_opts(strict_dict_panic, gc_watermark, gc_members, force_tier, pipe_ranges)
        st = MergeStats()
        h = ctypes.c_void_p()
        rc = lib().cdb_merge(self.ctx.handle, arr, n, ctypes.byref(opts), ctypes.byref(h), ctypes.byref(st))
        if rc not in (OK, DICT_MERGE_UNIMPLEMENTED):
            _raise(rc, self.ctx.last_error())
        m = Merged(self.ctx, h, st, batches)
        if rc == DICT_MERGE_UNIMPLEMENTED:
            raise DictMergeUnimplemented(self.ctx.last_error())
        return m

    def merge_snapshots(self, snapshots: Sequence[bytes], **kw) -> Merged:
        return self.merge_batches([decode_snapshot(s) for s in snapshots], **kw)

    def merge_into(self, state: Merged, batches: Sequence[Batch], strict_dict_panic: bool = False,
                   gc_watermark: Optional[int] = None, gc_members: bool = False, force_tier: int = 0,
                   pipe_ranges: int = 0) -> Merged:
        """cdb_merge_into: `batches` merged into the existing result `state` (fold position 0),
        as the reference merges peer snapshots into its live DB (replica/pull.rs:120-128)."""
        n = len(batches)
        arr = (ctypes.c_void_p * max(n, 1))(*[b.handle for b in batches])
        opts = merge_opts(strict_dict_panic, gc_watermark, gc_members, force_tier, pipe_ranges)
        st = MergeStats()
        h = ctypes.c_void_p()
        rc = lib().cdb_merge_into(self.ctx.handle, state.handle, arr, n, ctypes.byref(opts), ctypes.byref(h),
                                  ctypes.byref(st))
        if rc not in (OK, DICT_MERGE_UNIMPLEMENTED):
            _raise(rc, self.ctx.last_error())
        m = Merged(self.ctx, h, st, state._inputs + list(batches))
        if rc == DICT_MERGE_UNIMPLEMENTED:
            raise DictMergeUnimplemented(self.ctx.last_error())
        return m


def merge_opts(strict_dict_panic: bool = False, gc_watermark: Optional[int] = None, gc_members: bool = False,
               force_tier: int = 0, pipe_ranges: int = 0) -> MergeOpts:
    opts = MergeOpts()
    opts.flags = (MERGE_STRICT_DICT_PANIC if strict_dict_panic else 0)
    opts.force_tier = force_tier
    opts.pipe_ranges = pipe_ranges
    if gc_watermark is not None:
        opts.flags |= MERGE_GC_DELETES | (MERGE_GC_MEMBERS if gc_members else 0)
        opts.gc_watermark = gc_watermark
    return opts


def merge_sharded(ctx: "Context", inputs: Sequence["DevInput"], **kw):
    """cdb_merge_sharded over every device slot of a multi-device context: inputs[i] are the rows
    on slot i. Returns (outputs: list of DevOutput (library-owned, valid until the next call),
    per-slot MergeStats, ExchangeStats)."""
    n = ctx.n_devices
    if len(inputs) != n:
        raise ValueError(f"{n} device slots, {len(inputs)} inputs")
    ins = (DevInput * n)(*inputs)
    outs = (DevOutput * n)()
    sts = (MergeStats * n)()
    xs = ExchangeStats()
    opts = merge_opts(**kw)
    ctx.check(lib().cdb_merge_sharded(ctx.handle, ins, ctypes.byref(opts), outs, sts, ctypes.byref(xs)))
    return list(outs), list(sts), xs


def merged_from_device(ctx: Context, dout: "DevOutput", inputs: Sequence[Batch], state: Optional[Merged] = None,
                       stats: Optional[MergeStats] = None) -> Merged:
    """cdb_merged_from_device: the host view of a cdb_merge_device result (rows downloaded, bytes
    resolved through `inputs`, and through `state` for fold position 0 when given)."""
    n = len(inputs)
    arr = (ctypes.c_void_p * max(n, 1))(*[b.handle for b in inputs])
    h = ctypes.c_void_p()
    ctx.check(lib().cdb_merged_from_device(ctx.handle, state.handle if state else None, arr, n, ctypes.byref(dout),
                                           ctypes.byref(h)))
    return Merged(ctx, h, stats if stats is not None else MergeStats(), (state._inputs if state else []) + list(inputs))


# ----------------------------------------------------------------- synthetic inputs
def gen_config(**overrides) -> GenConfig:
    c = GenConfig()
    lib().cdb_gen_default(ctypes.byref(c))
    for k, v in overrides.items():
        setattr(c, k, v)
    return c


def gen_ops(cfg: GenConfig, n_ops: int, uuid_he_sent: int = 0, zipf_milli: int = 0) -> bytes:
    """A seeded replicate stream over cfg's key universe (cdb_gen_ops)."""
    out = ctypes.c_void_p()
    n = ctypes.c_size_t()
    st = lib().cdb_gen_ops(ctypes.byref(cfg), n_ops, uuid_he_sent, zipf_milli, ctypes.byref(out), ctypes.byref(n))
    if st != OK:
        _raise(st)
    try:
        return _take(out.value, n.value)
    finally:
        lib().cdb_free(out)


def gen_snapshot(cfg: GenConfig, replica: int) -> bytes:
    out = ctypes.c_void_p()
    n = ctypes.c_size_t()
    st = lib().cdb_gen_snapshot(ctypes.byref(cfg), replica, ctypes.byref(out), ctypes.byref(n))
    if st != OK:
        _raise(st)
    try:
        return _take(out.value, n.value)
    finally:
        lib().cdb_free(out)
