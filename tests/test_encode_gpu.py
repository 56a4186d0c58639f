"""GPU snapshot encode through the C ABI: cdb_encode_snapshot / cdb_crc64_gpu.

A merge result is written back in the reference's wire format (Server::dump_all,
server.rs:183-215) by the HIP kernels. Checks, per case:
  * the checksum: the oracle's CRC-64/Jones over the stream (crc64 2.0.0, pinned by the
    reference golden snapshot.rs:372) equals the 8 trailing LE bytes;
  * semantics: the oracle loads the stream (its loader restatement, snapshot.rs:120-220) and
    folds it into an empty DB; its canonical dump equals the merge result's;
  * bytes: the oracle's writer restatement (db.rs:122-136, object.rs:85-108,
    type_counter.rs:101-109, lwwhash.rs:189-205/325-339, replica.rs:100-119) applied to that
    DB, in the order the stream lists keys, nodes and members, reproduces the stream byte for
    byte (the reference's HashMap order is unspecified, so the order is the encoder's choice;
    every varint, length and section count is pinned);
  * the product's own decode + merge of the stream gives the same result again.
"""
import struct

import pytest
import torch  # noqa: F401  -- before libcdbmerge loads: one HIP runtime per process

import cdb_oracle
import constdb_amd as cdb
import constdb_oracle as o
from snapgen import gen_replicas

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def db():
    from constdb_amd import build
    build.build()
    return cdb.DB(cdb.Context(0))


def _hdr(m, **kw):
    reps = m.replicas()
    h = o.NodeHeader(node_id=kw.get("node_id", 1), alias=kw.get("alias", "n1"),
                     addr=kw.get("addr", "127.0.0.1:9001"), last_uuid=kw.get("last_uuid", 0))
    h.replicas_add = [(d["add"][0], d["add"][1], d["add"][2], d["addr"], d["add"][3]) for d in reps if "add" in d]
    h.replicas_del = [(d["addr"], d["del"]) for d in reps if "del" in d]
    return h


def _check_stream(m, enc, hdr, full=True):
    assert o.crc64(enc[:-8]) == struct.unpack("<Q", enc[-8:])[0]
    assert enc[-9] == o.SNAPSHOT_FLAG_CHECKSUM
    want = m.canonical_dump()
    if full:
        odb = o.fold_snapshots([enc])
        assert o.canonical_dump(odb) == want
        assert o.dump_all(odb, hdr) == enc
        assert o.fold_replicas([enc]) == m.replicas() or not m.replicas()
    else:
        rc, dump, _ = cdb_oracle.fold([enc])
        assert rc == 0 and dump == want


def _roundtrip(db, enc, want):
    m2 = db.merge_snapshots([enc])
    assert m2.canonical_dump() == want


@pytest.mark.parametrize("seed", range(12))
def test_encode_random(db, seed):
    snaps = gen_replicas(seed, n_replicas=1 + seed % 5, n_keys=30 + 7 * seed)
    m = db.merge_snapshots(snaps)
    kw = dict(node_id=3 + seed, alias="node-%d" % seed, addr="10.0.0.%d:7000" % seed, last_uuid=(1 << 40) + seed)
    enc, st = m.encode_snapshot(**kw)
    assert st.bytes == len(enc)
    assert st.checksum == struct.unpack("<Q", enc[-8:])[0]
    _check_stream(m, enc, _hdr(m, **kw))
    _roundtrip(db, enc, m.canonical_dump())


@pytest.mark.parametrize("gc", [0, 7, 1 << 62])
def test_encode_after_gc(db, gc):
    snaps = gen_replicas(40 + gc % 5, n_replicas=4, n_keys=80)
    m = db.merge_snapshots(snaps, gc_watermark=gc, gc_members=True)
    enc, _ = m.encode_snapshot()
    _check_stream(m, enc, _hdr(m))


@pytest.mark.parametrize("tier", [1, 2, 3])
def test_encode_forced_tiers(db, tier):
    snaps = gen_replicas(77, n_replicas=3, n_keys=60)
    m = db.merge_snapshots(snaps, force_tier=tier)
    enc, _ = m.encode_snapshot()
    _check_stream(m, enc, _hdr(m))


def test_encode_empty(db):
    empty = o.dump_all(o.DB(), o.NodeHeader())
    m = db.merge_snapshots([empty])
    enc, st = m.encode_snapshot(replicas=None)
    assert enc == o.dump_all(o.DB(), o.NodeHeader())
    assert (st.data_entries, st.expires, st.deletes) == (0, 0, 0)


def test_encode_varint_boundaries(db):
    """Every write_integer branch (snapshot.rs:25-37) in times, lengths, node ids and values:
    63/64, 2^14-1/2^14, 2^30-1/2^30, and a time >= 2^63 (negative as i64: one truncated byte)."""
    d = o.DB()
    edges = [0, 63, 64, (1 << 14) - 1, 1 << 14, (1 << 30) - 1, 1 << 30, (1 << 62) + 5]
    for i, t in enumerate(edges):
        c = o.Counter()
        c.data[t] = (edges[-1 - i], t)
        c.cal_sum()
        d.data[b"c%d" % i] = o.Object(t, t, t, o.OBJECT_ENC_COUNTER, c)
    d.data[b"v" * 64] = o.Object(1, 2, 3, o.OBJECT_ENC_BYTES, b"x" * (1 << 14))
    s = o.Set()
    for n in (63, 64, 200):
        s.set(b"m" * n, None, n)
    s.rem(b"gone", 1 << 30)
    d.data[b"s"] = o.Object(5, 0, 0, o.OBJECT_ENC_SET, s)
    dd = o.Dict()
    dd.set(b"f", b"y" * 70, 9)
    dd.rem(b"g", 10)
    d.data[b"d"] = o.Object(5, 0, 0, o.OBJECT_ENC_DICT, dd)
    d.expires[b"e" * 63] = 1 << 30
    d.deletes[b"r"] = (1 << 14) - 1
    snap = o.dump_all(d, o.NodeHeader())
    m = db.merge_snapshots([snap])
    enc, _ = m.encode_snapshot(replicas=None, last_uuid=1 << 30)
    _check_stream(m, enc, o.NodeHeader(last_uuid=1 << 30))


def test_encode_big_member_key(db):
    """A set with 3000 members (the global-scratch merge tier) and a counter with 200 nodes."""
    d = o.DB()
    s = o.Set()
    for i in range(3000):
        if i % 3:
            s.set(b"member-%d" % i, None, 100 + i)
        else:
            s.rem(b"member-%d" % i, 100 + i)
    d.data[b"big"] = o.Object(1, 0, 0, o.OBJECT_ENC_SET, s)
    c = o.Counter()
    for n in range(200):
        c.data[n + 1] = (n * 1000, 50 + n)
    c.cal_sum()
    d.data[b"ctr"] = o.Object(2, 0, 0, o.OBJECT_ENC_COUNTER, c)
    d2 = o.DB()
    s2 = o.Set()
    for i in range(0, 3000, 2):
        s2.set(b"member-%d" % i, None, 1000 + i)
    d2.data[b"big"] = o.Object(1, 0, 0, o.OBJECT_ENC_SET, s2)
    snaps = [o.dump_all(d, o.NodeHeader()), o.dump_all(d2, o.NodeHeader(node_id=2, addr="127.0.0.1:9002"))]
    m = db.merge_snapshots(snaps)
    enc, _ = m.encode_snapshot()
    _check_stream(m, enc, _hdr(m))


def test_encode_after_ops(db):
    """A result of cdb_apply_ops (its inputs include the op stream's byte arena)."""
    from opsgen import gen_stream
    snaps = gen_replicas(5, n_replicas=2, n_keys=50)
    m = db.merge_snapshots(snaps)
    keys = sorted({ln.split()[1] for ln in m.canonical_dump().decode().splitlines() if ln.startswith("K ")})
    stream = gen_stream(11, [bytes.fromhex(k) for k in keys], n_cmds=300, hazards=False)
    m2 = m.apply_ops(cdb.decode_ops(stream, 5))
    dump = m2.canonical_dump().decode()
    enc, _ = m2.encode_snapshot()
    if any(ln.startswith(" N ") and ln.split()[2].startswith("-") for ln in dump.splitlines()):
        # a negative counter value is truncated to one byte by write_integer (snapshot.rs:26-27)
        # and the stream no longer loads: only the checksum is checked
        assert o.crc64(enc[:-8]) == struct.unpack("<Q", enc[-8:])[0]
    else:
        _check_stream(m2, enc, _hdr(m2))


def test_encode_generator_medium(db):
    """C4-shaped generator input (20K-key universe x 8 replicas): the C++ oracle loads the
    stream (writer checksum verified) and its fold equals the merge result."""
    cfg = cdb.gen_config(seed=4, universe=20000, n_replicas=8, replica_hi=8)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    m = db.merge_snapshots(snaps)
    enc, st = m.encode_snapshot()
    assert st.bytes == len(enc) > 262144  # several CRC tiles
    _check_stream(m, enc, _hdr(m), full=False)
    _roundtrip(db, enc, m.canonical_dump())


@pytest.mark.parametrize("n", [1, 7, 8, 9, 1023, 1024, 1025, 262143, 262144, 262145, 3 * 262144 + 17])
def test_crc64_gpu_lengths(db, n):
    import random
    data = random.Random(n).randbytes(n)
    assert cdb.crc64_gpu(db.ctx, data) == o.crc64(data)


def test_crc64_gpu_reference_golden(db):
    """snapshot.rs:362-372: CRC-64 9519382692141102896 of the varint test stream, and the
    CRC-64/Jones check value of b"123456789"."""
    w = o.SnapshotWriter()
    w.write_bytes(b"CONST")
    w.write_bytes(b"DB")
    for i in [1, 2, 1 << 13, 1 << 20, 1 << 26, 1 << 30, 1 << 31]:
        w.write_integer(i)
    assert cdb.crc64_gpu(db.ctx, w.getvalue()) == 9519382692141102896
    assert cdb.crc64_gpu(db.ctx, b"123456789") == 0xE9C6D914C4B8D9CA
    assert cdb.crc64_gpu(db.ctx, b"") == 0
