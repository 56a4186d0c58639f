"""Snapshot encode straight from HBM (cdb_encode_device, SURVEY §8f.3 for a node whose state is a
cdb_merge_device result): byte for byte the stream cdb_encode_snapshot writes for the host view of
the same result (that encoder is pinned to the reference's writer by tests/test_encode_gpu.py), for
either result layout, for byte references still in HBM (device decode) or on the host (host decode,
or after a canonical dump pulled them down), for snapshot bytes kept in HBM (CDB_DECODE_KEEP_BYTES)
or uploaded, and with host-tier member references patched into the HBM tables. The stream decodes
back, through the oracle's loader, to the oracle's fold of the inputs (server.rs:183-215 ->
db.rs:122-136 then pull.rs:64-79)."""
import ctypes

import pytest
import torch  # noqa: F401  -- before libcdbmerge loads (one HIP runtime per process)

import cdb_oracle
import constdb_amd as cdb
import constdb_oracle as o
from snapgen import gen_replicas

pytestmark = pytest.mark.gpu

REPLICAS = [{"addr": "10.0.0.2:9001", "add": (7, 2, "n2", 99)}, {"addr": "10.0.0.3:9001", "del": 11}]


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _release(ctx, *sets):
    L = cdb.lib()
    for s in sets:
        for name in ("keys", "nodes", "members"):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(s, name)))


def _merge(ctx, din, compact):
    L = cdb.lib()
    dout = cdb.DevOutput()
    if compact:
        for name, nc in (("keys", 8), ("nodes", 6), ("members", 6)):
            r = cdb.DevRows()
            ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(din, name).n, nc))
            setattr(dout, name, r)
    dout.compact = 1 if compact else 0
    opts = cdb.merge_opts()
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(dout),
                                 ctypes.byref(st), None))
    return dout, st


def _roundtrip_vs_oracle(stream, snaps):
    """The encoded stream, loaded alone, holds the fold of the inputs (a merge result re-loaded is
    the same state: the oracle's canonical dumps agree)."""
    rc, want, _ = cdb_oracle.fold(snaps)
    assert rc == 0
    rc2, got, _ = cdb_oracle.fold([stream])
    assert rc2 == 0 and got == want


def _writer_check(stream):
    """The oracle's writer restatement (db.rs:122-136, object.rs:85-108, replica.rs:100-119) over the
    oracle's load of the stream reproduces it byte for byte (the order is the stream's)."""
    h = o.NodeHeader(node_id=5, alias="a5", addr="10.0.0.5:9001", last_uuid=1234)
    h.replicas_add = [(7, 2, "n2", "10.0.0.2:9001", 99)]
    h.replicas_del = [("10.0.0.3:9001", 11)]
    assert o.dump_all(o.fold_snapshots([stream]), h) == stream


def _case(ctx, snaps, records=True, compact=False, keep_bytes=True, host_refs_first=False, device_decode=True,
          writer=False):
    if device_decode:
        batches, din = cdb.decode_snapshots_device(ctx, snaps, records=records, keep_bytes=keep_bytes)
    else:
        batches = [cdb.decode_snapshot(s) for s in snaps]
        din = cdb.DevInput()
        arr = (ctypes.c_void_p * len(batches))(*[b.handle for b in batches])
        ctx.check(cdb.lib().cdb_upload_batches(ctx.handle, arr, len(batches), ctypes.byref(din)))
    dout = None
    try:
        dout, st = _merge(ctx, din, compact)
        if host_refs_first:  # the canonical dump pulls the byte references down first
            cdb.merged_from_device(ctx, dout, batches, stats=st).canonical_dump()
        got, est = cdb.encode_device(ctx, dout, batches, node_id=5, alias="a5", addr="10.0.0.5:9001",
                                     last_uuid=1234, replicas=REPLICAS)
        m = cdb.merged_from_device(ctx, dout, batches, stats=st)
        want, wst = m.encode_snapshot(node_id=5, alias="a5", addr="10.0.0.5:9001", last_uuid=1234,
                                      replicas=REPLICAS)
        assert got == want
        assert (est.bytes, est.checksum, est.data_entries, est.expires, est.deletes) == \
            (wst.bytes, wst.checksum, wst.data_entries, wst.expires, wst.deletes)
        _roundtrip_vs_oracle(got, snaps)
        if writer:
            _writer_check(got)
        return est
    finally:
        _release(ctx, din)
        if dout is not None and compact:
            _release(ctx, dout)


@pytest.mark.parametrize("records,compact,keep_bytes", [(True, False, True), (True, True, False),
                                                        (False, False, False), (False, True, True)])
@pytest.mark.parametrize("seed", range(3))
def test_encode_device_random(ctx, seed, records, compact, keep_bytes):
    snaps = gen_replicas(seed, n_replicas=2 + seed, n_keys=60 + 11 * seed, p_conflict=0.1, p_side=0.3)
    _case(ctx, snaps, records=records, compact=compact, keep_bytes=keep_bytes, writer=True)


def test_encode_device_after_refs_downloaded(ctx):
    """The byte references already pulled to the host by a canonical dump: uploaded again."""
    snaps = gen_replicas(7, n_replicas=3, n_keys=120, p_conflict=0.1, p_side=0.3)
    _case(ctx, snaps, host_refs_first=True)


def test_encode_device_host_batches(ctx):
    """Host-decoded batches (cdb_upload_batches): bytes and references all go up."""
    snaps = gen_replicas(8, n_replicas=3, n_keys=120, p_conflict=0.1, p_side=0.3)
    for compact in (False, True):
        _case(ctx, snaps, compact=compact, device_decode=False)


def test_encode_device_host_tier_patches(ctx):
    """Objects past the device decoder's dedup limits (3000 members): their member references come
    from the host decoder and are patched into the HBM tables before the emit."""
    big, d = o.Set(), o.Dict()
    for j in range(3100):
        big.set(b"m%d" % j, None, j % 17)
        d.set(b"f%d" % j, b"v%d" % (j * 7), j % 11)
    db = o.DB()
    db.data.update({b"big": o.Object(1, 0, 0, o.OBJECT_ENC_SET, big),
                    b"dict": o.Object(1, 0, 0, o.OBJECT_ENC_DICT, d)})
    snap = o.dump_all(db, o.NodeHeader())
    snaps = [gen_replicas(4, n_replicas=1)[0], snap, snap]
    for compact in (False, True):
        _case(ctx, snaps, compact=compact)


def test_encode_device_generator(ctx):
    """A 40K-key generator replica set (Set / Dict / Counter mix, deletes, expires), bucket layout."""
    cfg = cdb.gen_config(seed=11, universe=40_000, n_replicas=3, replica_hi=3, mix_set=20, mix_dict=20,
                         mean_members=5, del_permille=300, side_permille=200)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(3)]
    est = _case(ctx, snaps)
    assert est.data_entries > 30_000


def test_encode_device_empty(ctx):
    """No rows at all: the header, replica entries and checksum only."""
    snaps = [o.dump_all(o.DB(), o.NodeHeader())]
    _case(ctx, snaps)
    _case(ctx, snaps, compact=True, keep_bytes=False)


def test_encode_device_rejects_bad_arguments(ctx):
    L = cdb.lib()
    dout = cdb.DevOutput()
    hdr = cdb.EncodeHeader()
    o_ = ctypes.c_void_p()
    n = ctypes.c_size_t()
    assert L.cdb_encode_device(ctx.handle, None, None, 0, ctypes.byref(hdr), ctypes.byref(o_), ctypes.byref(n),
                               None) == cdb.BAD_ARGUMENT
    assert L.cdb_encode_device(ctx.handle, ctypes.byref(dout), None, 1, ctypes.byref(hdr), ctypes.byref(o_),
                               ctypes.byref(n), None) == cdb.BAD_ARGUMENT


def test_encode_device_c4_1m(ctx):
    """C4's shape (the bench's generator config) at 1M keys x 8 replicas: decoded into HBM with the
    bytes kept, merged into the bucket layout, encoded from HBM; equal to the host view's stream, and
    the C++ oracle's load + fold of that stream equals its fold of the eight snapshots."""
    from constdb_amd import configs
    cfg = configs.c4(cdb, 1_000_000)
    est = _case(ctx, [cdb.gen_snapshot(cfg, r) for r in range(8)])
    assert est.data_entries > 900_000
