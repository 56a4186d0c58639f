"""CPU tests of the product library: C-ABI exports, host decoder vs the oracle loader,
and the synthetic snapshot generator. No GPU needed (decode is host code)."""
import os
import re
import subprocess

import pytest

import constdb_amd as cdb
import constdb_oracle as o
from snapgen import gen_replicas

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="session", autouse=True)
def built():
    from constdb_amd import build
    build.build()


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "cdb_merge.h")).read()
    declared = set(re.findall(r"\b(cdb_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(cdb.ABI_FUNCTIONS)
    out = subprocess.check_output(["nm", "-D", "--defined-only", cdb.lib_path()]).decode()
    exported = set(re.findall(r" T (cdb_[a-z0-9_]+)$", out, re.M))
    assert declared <= exported, declared - exported
    L = cdb.lib()
    for name in declared:
        assert getattr(L, name)


def _oracle_entries(snap):
    return o.load_snapshot(snap)


@pytest.mark.parametrize("seed", range(12))
def test_decode_matches_oracle_loader(seed):
    snaps = gen_replicas(seed, n_replicas=2, big_times=bool(seed % 2))
    for snap in snaps:
        entries = _oracle_entries(snap)
        b = cdb.decode_snapshot(snap)
        info = b.info()
        data = [e for e in entries if e.kind == "Data"]
        assert info.n_data == len(data)
        assert info.n_expires == sum(e.kind == "Expires" for e in entries)
        assert info.n_deletes == sum(e.kind == "Deletes" for e in entries)
        node = [e for e in entries if e.kind == "Node"][0]
        assert info.node_id == node.args[0] and info.uuid_he_sent == node.args[3]
        assert info.version.decode() == "0.1.1.1"
        # per data row: times, tag, counter load sums
        ct, ut, dt = b.column(0, 2), b.column(0, 3), b.column(0, 4)
        aux, meta = b.column(0, 5), b.column(0, 6)
        nodes = members = 0
        for i, e in enumerate(data):
            _, obj = e.args
            assert (ct[i], ut[i], dt[i]) == (obj.create_time, obj.update_time, obj.delete_time)
            assert meta[i] >> 56 == obj.tag and meta[i] & ((1 << 48) - 1) == i
            if obj.tag == o.OBJECT_ENC_COUNTER:
                assert aux[i] == obj.enc.sum & ((1 << 64) - 1)
                nodes += len(obj.enc.data)
            elif obj.tag in (o.OBJECT_ENC_SET, o.OBJECT_ENC_DICT):
                members += len(obj.enc.add) + len(obj.enc.dele)
        assert info.n_nodes == nodes and info.n_members == members


def test_decode_member_reconstruction_matches_loader():
    """lwwhash.rs:341-358: a member present in both add and del sections keeps one tag."""
    s = o.Set()
    s.add[b"m"] = (5, None)
    s.dele[b"m"] = 7
    s.add[b"n"] = (9, None)
    s.dele[b"n"] = 3
    s.add[b"p"] = (4, None)
    db = o.DB()
    db.data[b"s"] = o.Object(1, 0, 0, o.OBJECT_ENC_SET, s)
    snap = o.dump_all(db, o.NodeHeader())
    b = cdb.decode_snapshot(snap)
    kinds = b.column(2, 5)
    ts = b.column(2, 4)
    got = sorted((t, k >> 56) for t, k in zip(ts, kinds))
    assert got == [(4, 0), (7, 1), (9, 0)]       # p add@4, m del@7, n add@9


def test_decode_duplicate_counter_node_keeps_last_and_total():
    """type_counter.rs:111-126: data.insert overwrites; total sums every value."""
    c = o.Counter()
    c.data[1] = (5, 10)
    db = o.DB()
    db.data[b"c"] = o.Object(1, 0, 0, o.OBJECT_ENC_COUNTER, c)
    snap = bytearray(o.dump_all(db, o.NodeHeader()))
    # rewrite "n=1, (1,5,10)" as "n=2, (1,5,10), (1,7,11)" by re-encoding the body
    w = o.SnapshotWriter()
    w.write_bytes(b"CONSTDB")
    w.write_bytes(bytes([0, 1, 1, 1]))
    w.write_integer(1).write_integer(2).write_bytes(b"n1").write_integer(0).write_integer(0)
    w.write_byte(5).write_integer(1)
    w.write_integer(1).write_bytes(b"c").write_integer(1).write_integer(0).write_integer(0).write_byte(0)
    w.write_integer(2)
    for n, v, t in ((1, 5, 10), (1, 7, 11)):
        w.write_integer(n).write_integer(v).write_integer(t)
    for f in (6, 7):
        w.write_byte(f).write_integer(0)
    w.write_byte(8)
    import struct
    w.write_bytes(struct.pack("<Q", w.checksum()))
    raw = w.getvalue()
    ent = o.load_snapshot(raw)[2].args[1]
    b = cdb.decode_snapshot(raw)
    assert b.column(1, 3) == [7] and b.column(1, 4) == [11]
    assert b.column(0, 5)[0] == ent.enc.sum == 12


def test_decode_errors_mirror_loader():
    snaps = gen_replicas(3, n_replicas=1)
    s = snaps[0]
    bad = bytearray(s)
    bad[-1] ^= 0xFF
    with pytest.raises(cdb.InvalidSnapshotChecksum):
        cdb.decode_snapshot(bytes(bad))
    b = cdb.decode_snapshot(bytes(bad), allow_bad_checksum=True)
    assert not b.checksum_ok and b.info().n_data > 0
    with pytest.raises(cdb.IoError):
        cdb.decode_snapshot(s[:-15])
    with pytest.raises(cdb.IoError):
        cdb.decode_snapshot(b"CONST")
    with pytest.raises((cdb.InvalidSnapshotChecksum, cdb.IoError)):
        cdb.decode_snapshot(s, reference_checksum=True)   # snapshot.rs:207-213 quirk
    db = o.DB()
    db.data[b"k"] = o.Object(5, 0, 0, o.OBJECT_ENC_BYTES, b"v")
    raw = bytearray(o.dump_all(db, o.NodeHeader()))
    i = raw.index(b"\x01k") + 2 + 3
    raw[i] = 9
    with pytest.raises(cdb.InvalidType):
        cdb.decode_snapshot(bytes(raw))
    empty = bytearray(o.dump_all(o.DB(), o.NodeHeader()))
    empty[len(empty) - 15] = 0x42
    with pytest.raises(cdb.InvalidSnapshot):
        cdb.decode_snapshot(bytes(empty))


def test_empty_snapshot_decodes():
    b = cdb.decode_snapshot(o.dump_all(o.DB(), o.NodeHeader()))
    i = b.info()
    assert (i.n_data, i.n_expires, i.n_deletes, i.n_nodes, i.n_members) == (0, 0, 0, 0, 0)


@pytest.mark.parametrize("seed", [1, 2])
def test_generator_snapshots_are_valid_reference_streams(seed):
    cfg = cdb.gen_config(seed=seed, universe=3000, n_replicas=3, replica_hi=3)
    for r in range(3):
        snap = cdb.gen_snapshot(cfg, r)
        entries = o.load_snapshot(snap)          # the oracle accepts it (CRC, layout)
        b = cdb.decode_snapshot(snap)
        assert b.info().n_data == sum(e.kind == "Data" for e in entries) > 0
