"""GPU decode straight into HBM (cdb_decode_snapshots_device, SURVEY §8f.1 / pull.rs:64-79 ->
:120-128 without a host round trip): the device rows must equal, column for column, what
cdb_upload_batches leaves from the host decoder's batches (the host decoder is pinned to the
oracle's loader by tests/test_abi_decode.py, and that upload + merge to the oracle's fold by
tests/test_gpu_parity.py); the batches carry the same host side; errors name the snapshot
and the offset the host decoder reports; a bad checksum still returns every row."""
import ctypes

import numpy as np
import pytest
import torch  # noqa: F401  -- before libcdbmerge loads (one HIP runtime per process)

import constdb_amd as cdb
import constdb_oracle as o
from constdb_amd import configs
from snapgen import gen_replicas

pytestmark = pytest.mark.gpu

NCOLS = (7, 6, 6)


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _cols(din):
    """Every field of every family as numpy columns, from either input layout."""
    from constdb_amd.runs import wrap
    out = []
    for f, rows in enumerate((din.keys, din.nodes, din.members)):
        if not rows.n:
            out.append([np.zeros(0, np.uint64) for _ in range(NCOLS[f])])
            continue
        if rows.stride > 1:
            assert rows.stride == NCOLS[f] - 1
            rec = wrap(rows.col[1], rows.n * rows.stride).view(rows.n, rows.stride).cpu().numpy().view(np.uint64)
            out.append([wrap(rows.col[0], rows.n).cpu().numpy().view(np.uint64)] +
                       [rec[:, c - 1].copy() for c in range(1, NCOLS[f])])
        else:
            out.append([wrap(rows.col[c], rows.n).cpu().numpy().view(np.uint64) for c in range(NCOLS[f])])
    return out


def _release(din):
    L = cdb.lib()
    for fam in (din.keys, din.nodes, din.members):
        L.cdb_dev_rows_release(None, ctypes.byref(fam))


def _check(ctx, snaps, records=False):
    # stream order: the rows compare field for field with the host decoder's (a snapshot not in key-hash
    # order is otherwise sorted into a run: tests/test_records_gpu.py)
    batches, din = cdb.decode_snapshots_device(ctx, snaps, records=records, stream_order=True)
    if records:
        assert din.keys.stride == 6 and din.nodes.stride == 5 and din.members.stride == 5
    try:
        host = [cdb.decode_snapshot(s) for s in snaps]
        up = cdb.DevInput()
        arr = (ctypes.c_void_p * len(host))(*[b.handle for b in host])
        ctx.check(cdb.lib().cdb_upload_batches(ctx.handle, arr, len(host), ctypes.byref(up)))
        try:
            assert din.n_pos == len(snaps)
            for f, (x, y) in enumerate(zip(_cols(din), _cols(up))):
                if f == 0:  # key rows in (pos, src) order: a snapshot in key-hash order is placed as one run
                    x = [c[np.argsort(x[6] & np.uint64((1 << 56) - 1), kind="stable")] for c in x]
                for c in range(NCOLS[f]):
                    assert x[c].shape == y[c].shape and (x[c] == y[c]).all(), (f, c)
        finally:
            _release(up)
        for g, h in zip(batches, host):
            ig, ih = g.info(), h.info()
            for fld in ("n_data", "n_expires", "n_deletes", "n_nodes", "n_members", "node_id", "uuid_he_sent",
                        "n_replica_add", "n_replica_del", "version"):
                assert getattr(ig, fld) == getattr(ih, fld), fld
        return batches, din
    except BaseException:
        _release(din)
        raise


@pytest.mark.parametrize("records", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_device_decode_random(ctx, seed, records):
    snaps = gen_replicas(seed, n_replicas=1 + seed % 4, n_keys=40 + 7 * seed, p_conflict=0.1, p_side=0.3)
    _, din = _check(ctx, snaps, records)
    _release(din)


def test_device_decode_generator_and_merge(ctx):
    """A C4-shaped replica set (60K keys x 4): equal rows, and a merge of the device rows equals
    the merge of the uploaded host batches row for row."""
    cfg = cdb.gen_config(seed=3, universe=60_000, n_replicas=4, replica_hi=4, mix_set=20, mix_dict=20,
                         mean_members=6, del_permille=300)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(4)]
    _, din = _check(ctx, snaps)
    try:
        from test_gpu_parity import _dev_merge
        got, st = _dev_merge(ctx, din, torch)
        host = [cdb.decode_snapshot(s) for s in snaps]
        up = cdb.DevInput()
        arr = (ctypes.c_void_p * 4)(*[b.handle for b in host])
        ctx.check(cdb.lib().cdb_upload_batches(ctx.handle, arr, 4, ctypes.byref(up)))
        try:
            want, st2 = _dev_merge(ctx, up, torch)
        finally:
            _release(up)
        for x, y in zip(got, want):
            assert torch.equal(x, y)
        assert st.key_rows_out == st2.key_rows_out > 0
    finally:
        _release(din)


def test_device_decode_large_sections(ctx):
    """Snapshots whose DATAS sections exceed 2^17 entries (indexed on the device) decoded straight
    into HBM: rows equal the uploaded host batches."""
    cfg = cdb.gen_config(seed=9, universe=300_000, n_replicas=3, replica_hi=3, side_permille=100)
    _, din = _check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(3)])
    _release(din)


def test_device_decode_large_sections_with_huge_entries(ctx):
    """A device-indexed DATAS section holding Zipf-hot keys whose entries run to hundreds of KB
    (C5's generator at 300K keys): chunks that lie inside one entry find no sync point, or a
    spurious one in its member list, and the stitch rounds re-walk them from the true chain."""
    cfg = configs.c5(cdb, universe=300_000, events=3_000_000, replicas=2)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(2)]
    big = cdb.decode_snapshot(snaps[0]).info()
    assert big.n_data > (1 << 17)  # the section goes to the device index
    batches, din = _check(ctx, snaps)
    try:
        _dump_vs_oracle(ctx, snaps, batches, din)
    finally:
        _release(din)
    # damage inside the device-indexed section of the second snapshot: the same status and offset
    # as the host decoder, with the first snapshot indexed beside it
    for frac in (3, 2):
        bad = bytearray(snaps[1])
        at = len(bad) // frac
        bad[at:at + 8] = b"\xff" * 8
        want = None
        try:
            cdb.decode_snapshot(bytes(bad))
        except cdb.CstError as e:
            want = (type(e), getattr(e, "offset", None))
        if want is None:
            continue
        if want[0] is cdb.InvalidSnapshotChecksum:  # the entries still parse: rows returned, batch flagged
            batches, din = cdb.decode_snapshots_device(ctx, [snaps[0], bytes(bad)])
            _release(din)
            assert [b.checksum_ok for b in batches] == [True, False]
            continue
        tm = {}
        with pytest.raises(cdb.CstError) as ei:
            cdb.decode_snapshots_device(ctx, [snaps[0], bytes(bad)], timing=tm)
        assert (type(ei.value), getattr(ei.value, "offset", None)) == want and tm["failed"] == 1
    # a key's length byte broken at 1/8, 1/3 and 2/3 of the stream (entries start with the key
    # span, "key:<i>" here): the device walk fails on the true chain, the host pass reports it
    raw = snaps[1]
    for frac in (8, 3, 1.5):
        at = raw.index(b"key:", int(len(raw) / frac)) - 1
        bad = bytearray(raw)
        bad[at] = 0xFF
        with pytest.raises(cdb.CstError) as want:
            cdb.decode_snapshot(bytes(bad))
        assert type(want.value) is not cdb.InvalidSnapshotChecksum
        tm = {}
        with pytest.raises(cdb.CstError) as ei:
            cdb.decode_snapshots_device(ctx, [snaps[0], bytes(bad)], timing=tm)
        assert type(ei.value) is type(want.value) and tm["failed"] == 1
        assert getattr(ei.value, "offset", None) == getattr(want.value, "offset", None)


def test_device_decode_host_tier(ctx):
    """Objects past the per-thread dedup limits (3000 members, 1500 nodes) are decoded on the
    host and uploaded into their reserved rows at the snapshot's fold position; their member
    byte references (kept in HBM with the rest until the dump asks) resolve to the oracle's
    fold of the same snapshots."""
    big, d, c = o.Set(), o.Dict(), o.Counter()
    for j in range(3000):
        big.set(b"m%d" % j, None, j % 17)
        d.set(b"f%d" % j, b"v%d" % (j * 7), j % 11)
        if j % 5 == 0:
            big.dele[b"m%d" % j] = (j % 13) + 3
    for n in range(1500):
        c.data[n] = (n, n % 5)
    c.cal_sum()
    db = o.DB()
    db.data.update({b"big": o.Object(1, 0, 0, o.OBJECT_ENC_SET, big),
                    b"dict": o.Object(1, 0, 0, o.OBJECT_ENC_DICT, d),
                    b"cnt": o.Object(1, 0, 0, o.OBJECT_ENC_COUNTER, c)})
    snap = o.dump_all(db, o.NodeHeader())
    snaps = [gen_replicas(4, n_replicas=1)[0], snap, snap]
    for records in (False, True):  # (records: the host tier's rows go up as the hash column + records)
        batches, din = _check(ctx, snaps, records)
        try:
            _dump_vs_oracle(ctx, snaps, batches, din)
        finally:
            _release(din)


def _dump_vs_oracle(ctx, snaps, batches, din):
    """cdb_merge_device over the device-decoded rows, then the canonical dump (its first call
    downloads the batches' byte references) against the C++ oracle's fold."""
    import cdb_oracle
    from test_runs_oracle_gpu import _diff, _merge_device, _out_for
    dout = _out_for(ctx, din)
    try:
        st = _merge_device(ctx, din, dout)
        m = cdb.merged_from_device(ctx, dout, batches, stats=st)
        got = m.canonical_dump()
        assert m.canonical_dump() == got  # the references are on the host now
        rc, want, _ = cdb_oracle.fold(snaps)
        assert rc == 0
        assert got == want, _diff(got, want)
    finally:
        _release(dout)


def test_device_decode_c3_snapshots(ctx):
    """C3 replica states (op-stream apply results: ~300-member sets, mostly the host tier)."""
    snaps = configs.c3_snapshots(cdb, ctx, ops_per_replica=200_000)
    _, din = _check(ctx, snaps)
    _release(din)


def test_device_decode_errors(ctx):
    good = gen_replicas(7, n_replicas=2)
    bad = bytearray(good[1])
    cut = bytes(bad[: len(bad) // 2])
    want = None
    try:
        cdb.decode_snapshot(cut)
    except cdb.CstError as e:
        want = (type(e), getattr(e, "offset", None))
    tm = {}
    with pytest.raises(cdb.CstError) as ei:
        cdb.decode_snapshots_device(ctx, [good[0], cut], timing=tm)
    assert (type(ei.value), getattr(ei.value, "offset", None)) == want and tm["failed"] == 1
    # a checksum mismatch in snapshot 1: every row is still returned, that batch flagged
    bad[-1] ^= 0xFF
    batches, din = cdb.decode_snapshots_device(ctx, [good[0], bytes(bad)])
    try:
        assert [b.checksum_ok for b in batches] == [True, False]
        host = cdb.decode_snapshot(bytes(bad), allow_bad_checksum=True)
        assert din.keys.n == cdb.decode_snapshot(good[0]).info().n_data + cdb.decode_snapshot(good[0]).info().n_expires \
            + cdb.decode_snapshot(good[0]).info().n_deletes + host.info().n_data + host.info().n_expires \
            + host.info().n_deletes
    finally:
        _release(din)
    # rows in HBM: the host merge and the upload refuse such a batch
    with pytest.raises((cdb.CstError, ValueError)):
        cdb.DB(ctx).merge_batches(batches)
