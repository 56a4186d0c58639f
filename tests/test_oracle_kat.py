"""Pin the oracle: the reference's own golden vectors + hand-derived merge KATs.

Every expectation below cites the reference line it is derived from. These tests
run on CPU only (no GPU, no product code).
"""
import struct

import pytest

import constdb_oracle as o


def _snap(objs=None, deletes=None, expires=None, node_id=1):
    """Build one snapshot (writer layout) from {key: Object}."""
    db = o.DB()
    for k, v in (objs or {}).items():
        db.data[k] = v
    for k, t in (deletes or {}).items():
        db.deletes[k] = t
    for k, t in (expires or {}).items():
        db.expires[k] = t
    return o.dump_all(db, o.NodeHeader(node_id=node_id, alias=f"n{node_id}"))


def _bytes(ct, v, ut=0, dt=0):
    return o.Object(ct, ut, dt, o.OBJECT_ENC_BYTES, v)


def _counter(nodes, ct=1, ut=0, dt=0):
    c = o.Counter()
    for n, (v, t) in nodes.items():
        c.data[n] = (v, t)
    c.cal_sum()
    return o.Object(ct, ut, dt, o.OBJECT_ENC_COUNTER, c)


def _set(adds, dels=None, ct=1, ut=0, dt=0):
    s = o.Set()
    for m, t in adds.items():
        s.set(m, None, t)
    for m, t in (dels or {}).items():
        s.rem(m, t)
    return o.Object(ct, ut, dt, o.OBJECT_ENC_SET, s)


def _dict(adds, dels=None, ct=1, ut=0, dt=0):
    d = o.Dict()
    for m, (t, v) in adds.items():
        d.set(m, v, t)
    for m, t in (dels or {}).items():
        d.rem(m, t)
    return o.Object(ct, ut, dt, o.OBJECT_ENC_DICT, d)


# ---------------------------------------------------------------- reference golden vectors
def test_reference_crc_golden():
    """snapshot.rs:362-372: the writer's CRC over this stream is 9519382692141102896."""
    w = o.SnapshotWriter()
    w.write_bytes(b"CONST")
    w.write_bytes(b"DB")
    for i in [1, 2, 1 << 13, 1 << 20, 1 << 26, 1 << 30, 1 << 31]:
        w.write_integer(i)
    assert w.checksum() == 9519382692141102896
    assert w.getvalue().hex() == (
        "434f4e53544442" "01" "02" "6000" "80100000" "84000000"
        "c00000000040000000" "c00000000080000000")


def test_reference_varint_roundtrip():
    """snapshot.rs:374-389: read back the same stream."""
    w = o.SnapshotWriter()
    w.write_bytes(b"CONST")
    w.write_bytes(b"DB")
    vals = [1, 2, 1 << 13, 1 << 20, 1 << 26, 1 << 30, 1 << 31]
    for i in vals:
        w.write_integer(i)
    r = o.SnapshotLoader(w.getvalue())
    assert r.read_bytes(5) == b"CONST"
    assert r.read_bytes(2) == b"DB"
    assert [r.read_integer() for _ in vals] == vals


def test_crc_check_value():
    """CRC-64/Jones (crc64 2.0.0) standard check value."""
    assert o.crc64(b"123456789") == 0xE9C6D914C4B8D9CA


@pytest.mark.parametrize("v,enc", [
    (0, "00"), (63, "3f"), (64, "4040"), (16383, "7fff"), (16384, "80004000"),
    ((1 << 30) - 1, "bfffffff"), (1 << 30, "c00000000040000000"),
    (-1, "ff"),                       # snapshot.rs:26-27: negatives take the 1-byte branch
])
def test_varint_boundaries(v, enc):
    w = o.SnapshotWriter()
    w.write_integer(v)
    assert w.getvalue().hex() == enc


def test_negative_varint_corrupts_stream():
    """R1: -1 is written as 0xFF, which the reader parses as the 9-byte form."""
    w = o.SnapshotWriter()
    w.write_integer(-1)
    with pytest.raises(o.IoError):
        o.SnapshotLoader(w.getvalue()).read_integer()


def test_reference_loader_checksum_quirk():
    """snapshot.rs:207-213 vs server.rs:205-207: the reference loader rejects a
    well-formed dump (reads the LE CRC as a varint and CRCs it too)."""
    s = _snap({b"k": _bytes(5, b"v")})
    assert len(o.load_snapshot(s, "writer")) == 3        # Version, Node, Data
    # the first LE CRC byte picks the varint form: a mismatch, or EOF for the 9-byte form
    with pytest.raises((o.InvalidSnapshotChecksum, o.IoError)):
        o.load_snapshot(s, "reference")
    bad = bytearray(s)
    bad[-1] ^= 1
    with pytest.raises(o.InvalidSnapshotChecksum):
        o.load_snapshot(bytes(bad), "writer")


def test_unknown_tag_is_invalid_type():
    """object.rs:121."""
    s = bytearray(_snap({b"k": _bytes(5, b"v")}))
    # patch the tag byte: ... klen k ct ut dt TAG
    i = s.index(b"\x01k") + 2 + 3
    assert s[i] == o.OBJECT_ENC_BYTES
    s[i] = 9
    with pytest.raises(o.InvalidType):
        o.load_snapshot(bytes(s))


def test_unknown_section_flag_is_invalid_snapshot():
    """snapshot.rs:236-238."""
    db = o.DB()
    s = bytearray(o.dump_all(db, o.NodeHeader()))
    i = len(s) - 9 - 6                  # DATAS flag: 05 00 06 00 07 00 08 <crc8>
    assert s[i] == o.SNAPSHOT_FLAG_DATAS
    s[i] = 0x42
    with pytest.raises(o.InvalidSnapshot):
        o.load_snapshot(bytes(s))


def test_truncated_is_io_error():
    s = _snap({b"k": _bytes(5, b"value")})
    with pytest.raises(o.IoError):
        o.load_snapshot(s[:-12])


# ---------------------------------------------------------------- merge KATs (§8a-T)
def _fold(*snaps, **kw):
    return o.fold_snapshots(list(snaps), **kw)


def test_bytes_ct_tie_keeps_earliest_value():
    """object.rs:71-73: strict `<` — a ct tie keeps the earlier pos's value."""
    db = _fold(_snap({b"k": _bytes(10, b"A", ut=3, dt=1)}),
               _snap({b"k": _bytes(10, b"B", ut=9, dt=0)}))
    x = db.data[b"k"]
    assert x.enc == b"A" and x.create_time == 10 and x.update_time == 9 and x.delete_time == 1


def test_bytes_max_ct_wins_times_independent():
    """object.rs:71-76: value from the max ct; ct, dt, ut each maxed independently."""
    db = _fold(_snap({b"k": _bytes(10, b"A", ut=50, dt=7)}),
               _snap({b"k": _bytes(12, b"B", ut=11, dt=3)}),
               _snap({b"k": _bytes(11, b"C", ut=12, dt=9)}))
    x = db.data[b"k"]
    assert (x.enc, x.create_time, x.update_time, x.delete_time) == (b"B", 12, 50, 9)


def test_counter_fold_is_order_dependent():
    """type_counter.rs:60-71: t of the (key,node) head is never updated."""
    a = _fold(_snap({b"c": _counter({1: (5, 10)})}), _snap({b"c": _counter({1: (7, 11)})}),
              _snap({b"c": _counter({1: (6, 12)})}))
    b = _fold(_snap({b"c": _counter({1: (5, 10)})}), _snap({b"c": _counter({1: (6, 12)})}),
              _snap({b"c": _counter({1: (7, 11)})}))
    assert a.data[b"c"].enc.data[1] == (6, 10)
    assert b.data[b"c"].enc.data[1] == (7, 10)
    assert a.data[b"c"].enc.sum == 6 and b.data[b"c"].enc.sum == 7


def test_counter_time_tie_takes_max_and_new_nodes_insert():
    """type_counter.rs:65-67 (tie -> max) and :81-83 (absent node -> insert)."""
    db = _fold(_snap({b"c": _counter({1: (5, 10), 2: (1, 3)})}),
               _snap({b"c": _counter({1: (3, 10), 3: (4, 8)})}),
               _snap({b"c": _counter({1: (9, 9), 3: (2, 9)})}))
    c = db.data[b"c"].enc
    assert c.data == {1: (5, 10), 2: (1, 3), 3: (2, 8)}
    assert c.sum == 8


def test_counter_unmerged_keeps_load_total():
    """type_counter.rs:111-126: an unmerged counter keeps its load-time total."""
    db = _fold(_snap({b"c": _counter({1: (5, 10), 2: (6, 1)})}))
    assert db.data[b"c"].enc.sum == 11


def test_non_bytes_object_times_are_head_times():
    """object.rs:68,78-79: Counter/Set/Dict merges do not touch ct/ut/dt."""
    db = _fold(_snap({b"c": _counter({1: (1, 1)}, ct=5, ut=6, dt=7)}),
               _snap({b"c": _counter({1: (1, 2)}, ct=50, ut=60, dt=70)}))
    x = db.data[b"c"]
    assert (x.create_time, x.update_time, x.delete_time) == (5, 6, 7)


def test_type_conflict_head_type_wins():
    """db.rs:36-40 + object.rs:80: mismatched types leave the local object untouched."""
    db = _fold(_snap({b"k": _counter({1: (1, 1)}, ct=5)}),
               _snap({b"k": _bytes(99, b"X")}),
               _snap({b"k": _counter({1: (4, 2)}, ct=6)}))
    x = db.data[b"k"]
    assert x.tag == o.OBJECT_ENC_COUNTER and x.enc.data == {1: (4, 1)}
    assert db.type_conflicts == 1


def test_set_ties_go_to_later_pos_and_remote_dels_ignored():
    """lwwhash.rs:87-107 (`*v > t` rejects; ties accepted) + :319-323 (only live adds)."""
    db = _fold(_snap({b"s": _set({b"a": 5, b"b": 7}, {b"d": 10})}),
               _snap({b"s": _set({b"d": 10, b"e": 1}, {b"a": 9})}),
               _snap({b"s": _set({b"b": 6})}))
    s = db.data[b"s"].enc
    assert s.add == {b"a": (5, None), b"b": (7, None), b"d": (10, None), b"e": (1, None)}
    assert s.dele == {}


def test_set_local_del_beats_older_add():
    db = _fold(_snap({b"s": _set({}, {b"m": 10})}), _snap({b"s": _set({b"m": 9})}))
    s = db.data[b"s"].enc
    assert s.add == {} and s.dele == {b"m": 10}


def test_dict_value_follows_tag_winner():
    """lwwhash.rs:176-179 (pre-panic loop): value of the winning add; ties -> later pos."""
    db = _fold(_snap({b"h": _dict({b"f": (5, b"x"), b"g": (9, b"y")})}),
               _snap({b"h": _dict({b"f": (5, b"z"), b"g": (8, b"w")})}))
    d = db.data[b"h"].enc
    assert d.add == {b"f": (5, b"z"), b"g": (9, b"y")}
    assert db.dict_merges == 1
    with pytest.raises(o.DictMergePanic):
        _fold(_snap({b"h": _dict({b"f": (5, b"x")})}), _snap({b"h": _dict({b"f": (6, b"z")})}),
              dict_panic=True)


def test_load_time_single_tag_invariant():
    """lwwhash.rs:341-358: a loaded member keeps exactly one tag (set then rem)."""
    s = o.Set()
    s.add[b"m"] = (5, None)
    s.dele[b"m"] = 7            # malformed on purpose: both tags
    s.add[b"n"] = (9, None)
    s.dele[b"n"] = 3
    obj = o.Object(1, 0, 0, o.OBJECT_ENC_SET, s)
    snap = _snap({b"s": obj})
    x = o.load_snapshot(snap)[2].args[1]
    assert x.enc.add == {b"n": (9, None)} and x.enc.dele == {b"m": 7}


def test_deletes_and_expires_last_pos_wins():
    """pull.rs:129-130 -> db.rs:68-76: plain overwrite, no time comparison."""
    db = _fold(_snap(deletes={b"a": 50, b"b": 1}, expires={b"x": 9}),
               _snap(deletes={b"a": 20}, expires={b"x": 3}))
    assert db.deletes == {b"a": 20, b"b": 1} and db.expires == {b"x": 3}


def test_gc_is_lifo_and_stops_at_first_newer():
    """db.rs:82-95: pops the most recent garbage first; stops at the first t > wm."""
    db = o.DB()
    db.delete(b"a", 5)
    db.delete(b"b", 50)
    db.delete(b"c", 6)
    db.gc(10)                   # pops c (6 <= 10, removed), then b (50 > 10) -> stop
    assert db.deletes == {b"a": 5, b"b": 50}
    db2 = o.DB()
    db2.delete(b"a", 5)
    db2.delete(b"a", 8)        # a -> 8; the earlier garbage (a,5) no longer matches
    db2.gc(100)
    assert db2.deletes == {}


def test_meet_scenario_from_bin_test():
    """bin/test.rs:85-106: r3 MEETs r2 and must read k3 == 2, k4 == 4."""
    t = 1 << 22
    r2 = _snap({b"k1": _counter({1: (1, 1 * t)}), b"k2": _counter({2: (2, 3 * t)}),
                b"k3": _counter({1: (1, 8 * t), 2: (1, 9 * t)}),
                b"k4": _counter({2: (4, 7 * t)})}, node_id=2)
    db = _fold(_snap({}, node_id=3), r2)
    assert db.data[b"k3"].enc.sum == 2 and db.data[b"k4"].enc.sum == 4
    assert db.data[b"k1"].enc.sum == 1 and db.data[b"k2"].enc.sum == 2


def test_canonical_dump_is_sorted_and_stable():
    db = _fold(_snap({b"b": _bytes(1, b"\x00"), b"a": _set({b"z": 1, b"y": 2}, {b"q": 3})},
                     deletes={b"d": 4}, expires={b"e": 5}))
    assert o.canonical_dump(db).decode().splitlines() == [
        "K 61 5 1 0 0", " D 71 3", " A 79 2", " A 7a 1",
        "K 62 3 1 0 0", " V 00", "X 65 5", "R 64 4"]


# ---------------------------------------------------------------- replica metadata (§8f.4)
def test_kat_replica_metadata_merge():
    """ReplicaManager's LWWHash<addr, ReplicaMeta> through the fold (replica/pull.rs:131-156,
    replica/replica.rs:29-35, crdt/lwwhash.rs:87-128); expected values derived by hand."""
    import constdb_oracle as o
    empty = o.DB()
    local = o.NodeHeader(node_id=1, replicas_add=[(5, 2, "a", "A", 50), (7, 4, "c", "C", 70)],
                         replicas_del=[("B", 9)])
    r1 = o.NodeHeader(node_id=2, replicas_add=[
        (4, 2, "a-old", "A", 40),       # add older than A's add tag (5): rejected
        (10, 3, "b", "B", 100),         # newer than B's del tag (9): B comes back, del tag dropped
        (99, 1, "me", "SELF", 1)],      # names the local node: skipped (pull.rs:133-135)
        replicas_del=[("A", 5), ("C", 6)])  # A: tie with its add -> removed; C: older -> kept
    r2 = o.NodeHeader(node_id=3, replicas_add=[(5, 2, "a2", "A", 55)])  # tie with A's del: re-added
    snaps = [o.dump_all(empty, h) for h in (local, r1, r2)]
    got = o.fold_replicas(snaps)
    assert got == [
        {"addr": "A", "add": (5, 2, "a2", 55)},
        {"addr": "B", "add": (10, 3, "b", 100)},
        {"addr": "C", "add": (7, 4, "c", 70)},
    ]
    # local maps are installed verbatim, both tags kept
    both = o.NodeHeader(node_id=1, replicas_add=[(8, 5, "d", "D", 1)], replicas_del=[("D", 3)])
    assert o.fold_replicas([o.dump_all(empty, both)]) == [{"addr": "D", "add": (8, 5, "d", 1), "del": 3}]
