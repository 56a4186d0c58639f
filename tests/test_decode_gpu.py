"""GPU snapshot decode against the host decoder (itself pinned to the oracle's
loader, tests/test_abi_decode.py): every column of every family, the batch info, and the
merge of GPU-decoded batches against the oracle; the same status and offset on bad input."""
import struct

import pytest
import torch  # noqa: F401  -- before libcdbmerge loads (one HIP runtime per process)

import cdb_oracle
import constdb_amd as cdb
import constdb_oracle as o
from snapgen import gen_replicas

pytestmark = pytest.mark.gpu

NCOLS = (7, 6, 6)


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _same_batch(a, b):
    ia, ib = a.info(), b.info()
    for f in ("n_data", "n_expires", "n_deletes", "n_nodes", "n_members", "node_id", "uuid_he_sent",
              "n_replica_add", "n_replica_del", "version"):
        assert getattr(ia, f) == getattr(ib, f), f
    for fam in range(3):
        for c in range(NCOLS[fam]):
            x, y = a.column_array(fam, c), b.column_array(fam, c)
            assert x.shape == y.shape and (x == y).all(), (fam, c)


def _check(ctx, snaps):
    gpu = []
    for s in snaps:
        g = cdb.decode_snapshot_gpu(ctx, s)
        _same_batch(cdb.decode_snapshot(s), g)
        gpu.append(g)
    rc, want, _ = cdb_oracle.fold(snaps)
    assert rc == 0
    # key/value/member byte references reach the canonical dump through the merge
    assert cdb.DB(ctx).merge_batches(gpu).canonical_dump() == want


@pytest.mark.parametrize("seed", range(12))
def test_decode_gpu_random(ctx, seed):
    _check(ctx, gen_replicas(seed, n_replicas=1 + seed % 4, n_keys=40 + 7 * seed, p_conflict=0.1, p_side=0.3))


@pytest.mark.parametrize("universe,replicas,seed", [(3000, 2, 1), (40000, 4, 3)])
def test_decode_gpu_generator(ctx, universe, replicas, seed):
    cfg = cdb.gen_config(seed=seed, universe=universe, n_replicas=replicas, replica_hi=replicas, mix_set=20,
                         mix_dict=20, mean_members=6, del_permille=300)
    _check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(replicas)])


def test_decode_gpu_host_tier_and_dedup(ctx):
    """Objects past the per-thread dedup limits (3000 members, 1500 nodes) take the host tier;
    members in both the add and the del map replay set/rem (lwwhash.rs:341-358)."""
    big, c = o.Set(), o.Counter()
    for j in range(3000):
        big.set(b"m%d" % j, None, j % 17)
        if j % 5 == 0:
            big.dele[b"m%d" % j] = (j % 13) + 3
    for n in range(1500):
        c.data[n] = (n, n % 5)
    c.cal_sum()
    s = o.Set()
    s.add[b"m"] = (5, None)
    s.dele[b"m"] = 7
    s.add[b"n"] = (9, None)
    s.dele[b"n"] = 3
    db = o.DB()
    db.data.update({b"big": o.Object(1, 0, 0, o.OBJECT_ENC_SET, big),
                    b"cnt": o.Object(1, 0, 0, o.OBJECT_ENC_COUNTER, c),
                    b"s": o.Object(2, 0, 0, o.OBJECT_ENC_SET, s)})
    db.deletes[b"gone"] = 4
    db.expires[b"s"] = 99
    _check(ctx, [o.dump_all(db, o.NodeHeader())])


def test_decode_gpu_duplicate_counter_node(ctx):
    """A node id repeated inside one counter: the last triple wins, the total counts both."""
    w = o.SnapshotWriter()
    w.write_bytes(b"CONSTDB")
    w.write_bytes(bytes([0, 1, 1, 1]))
    w.write_integer(1).write_integer(2).write_bytes(b"n1").write_integer(0).write_integer(0)
    w.write_byte(5).write_integer(1)
    w.write_integer(1).write_bytes(b"c").write_integer(1).write_integer(0).write_integer(0).write_byte(0)
    w.write_integer(3)
    for n, v, t in ((1, 5, 10), (2, 1, 1), (1, 7, 11)):
        w.write_integer(n).write_integer(v).write_integer(t)
    for f in (6, 7):
        w.write_byte(f).write_integer(0)
    w.write_byte(8)
    w.write_bytes(struct.pack("<Q", w.checksum()))
    raw = w.getvalue()
    g = cdb.decode_snapshot_gpu(ctx, raw)
    _same_batch(cdb.decode_snapshot(raw), g)
    assert g.column(1, 2) == [2, 1] and g.column(1, 3) == [1, 7] and g.column(0, 5) == [13]


def test_decode_gpu_errors_mirror_host(ctx):
    s = gen_replicas(3, n_replicas=1)[0]
    bad = bytearray(s)
    bad[-1] ^= 0xFF
    cases = [bytes(bad), s[:-15], b"CONST", s[: len(s) // 2]]
    db = o.DB()
    db.data[b"k"] = o.Object(5, 0, 0, o.OBJECT_ENC_BYTES, b"v")
    raw = bytearray(o.dump_all(db, o.NodeHeader()))
    raw[raw.index(b"\x01k") + 5] = 9  # unknown object tag
    cases.append(bytes(raw))
    for case in cases:
        want = got = None
        try:
            cdb.decode_snapshot(case)
        except cdb.CstError as e:
            want = (type(e), getattr(e, "offset", None))
        try:
            cdb.decode_snapshot_gpu(ctx, case)
        except cdb.CstError as e:
            got = (type(e), getattr(e, "offset", None))
        assert want is not None and got == want
    b = cdb.decode_snapshot_gpu(ctx, bytes(bad), allow_bad_checksum=True)
    _same_batch(cdb.decode_snapshot(bytes(bad), allow_bad_checksum=True), b)


def test_decode_gpu_checksum_modes_mirror_host(ctx):
    """The GPU path checks the stream CRC on the device (the index pass defers it): outcome and
    error offset equal the host decoder's in both checksum layouts, good and corrupted."""
    s = gen_replicas(5, n_replicas=1)[0]
    bad = bytearray(s)
    bad[len(bad) // 3] ^= 0x01  # inside an entry's bytes: parses, CRC differs
    for case in (s, bytes(bad)):
        for ref in (False, True):
            want = got = None
            try:
                cdb.decode_snapshot(case, reference_checksum=ref)
            except cdb.CstError as e:
                want = (type(e), getattr(e, "offset", None))
            try:
                cdb.decode_snapshot_gpu(ctx, case, reference_checksum=ref)
            except cdb.CstError as e:
                got = (type(e), getattr(e, "offset", None))
            assert got == want, (ref, case is s)


def test_decode_gpu_c4_replica_speed(ctx):
    """One C4-config replica snapshot of a 1M-key universe (~540K entries): identical batch;
    the host index pass and the device time are reported beside the host decoder's time."""
    import time
    cfg = cdb.gen_config(seed=4, universe=1_000_000, n_replicas=8, key_permille=500, mix_bytes=60, mix_counter=30,
                         mix_set=5, mix_dict=5, mean_members=4, member_universe=16, replica_hi=8)
    snap = cdb.gen_snapshot(cfg, 0)
    t0 = time.perf_counter()
    host = cdb.decode_snapshot(snap)
    t_host = (time.perf_counter() - t0) * 1e3
    cdb.decode_snapshot_gpu(ctx, snap)  # warm
    tm = {}
    t0 = time.perf_counter()
    g = cdb.decode_snapshot_gpu(ctx, snap, timing=tm)
    t_gpu = (time.perf_counter() - t0) * 1e3
    _same_batch(host, g)
    print(f"\ndecode {len(snap) / 1e6:.1f} MB: host {t_host:.1f} ms; gpu path {t_gpu:.1f} ms "
          f"(index {tm['index_ms']:.1f} ms, device {tm['device_ms']:.1f} ms)")


def test_decode_gpu_staging_ring_wraps(ctx):
    """A ~125 MB snapshot: the upload and the row download each span several 32 MB slots of the
    context's pinned staging ring, which wraps; the batch equals the host decoder's, twice in a
    row on one context (the ring continues across calls)."""
    cfg = cdb.gen_config(seed=11, universe=4_000_000, n_replicas=8, replica_hi=8)
    snap = cdb.gen_snapshot(cfg, 3)
    assert len(snap) > 4 * (32 << 20) // 2
    host = cdb.decode_snapshot(snap)
    for _ in range(2):
        _same_batch(host, cdb.decode_snapshot_gpu(ctx, snap))


def test_decode_gpu_device_index_mirrors_host(ctx):
    """A DATAS section of more than 2^17 entries is indexed on the device (speculative chains per
    8 KB chunk, stitched from the section start; the host pass resumes after it for EXPIRES,
    DELETES and the checksum). The batch equals the host decoder's, and on damaged streams --
    truncated inside the section or after it, bytes flipped inside it, a bad checksum -- the
    status and the error offset are the host decoder's (the device hands failures back to it)."""
    import random
    cfg = cdb.gen_config(seed=21, universe=400_000, n_replicas=2, replica_hi=2, side_permille=150, mix_set=10,
                         mix_dict=10)
    snap = cdb.gen_snapshot(cfg, 1)
    host = cdb.decode_snapshot(snap)
    assert host.info().n_data > (1 << 17) and host.info().n_expires > 0 and host.info().n_deletes > 0
    _same_batch(host, cdb.decode_snapshot_gpu(ctx, snap))
    rng = random.Random(5)
    cases = [snap[: len(snap) // 2], snap[: len(snap) * 9 // 10], snap[:-9], snap[:-3]]
    for _ in range(6):
        bad = bytearray(snap)
        at = rng.randrange(len(snap) // 10, len(snap) * 8 // 10)
        bad[at] ^= 1 << rng.randrange(8)
        cases.append(bytes(bad))
    bad = bytearray(snap)
    bad[-2] ^= 0x40
    cases.append(bytes(bad))
    for i, case in enumerate(cases):
        for ref in (False, True):
            want = got = None
            try:
                cdb.decode_snapshot(case, reference_checksum=ref)
            except cdb.CstError as e:
                want = (type(e), getattr(e, "offset", None))
            try:
                cdb.decode_snapshot_gpu(ctx, case, reference_checksum=ref)
            except cdb.CstError as e:
                got = (type(e), getattr(e, "offset", None))
            assert got == want, (i, ref)
