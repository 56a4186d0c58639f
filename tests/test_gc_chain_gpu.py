"""DB::gc across chained merges (db.rs:14,73-76,82-119; Server::gc server.rs:257-262).

The reference's DB keeps `garbages`, the Deletes entries in the order DB::delete applied them, across
every MEET; DB::gc pops it from the back, removes a key's Deletes entry when the popped time equals
its current one, and stops at the first entry newer than the tombstone -- popping and losing it. A
result of this engine keeps the same list (cdb_merged.garbage): cdb_merge starts it with the merged
snapshots' Deletes entries, cdb_merge_into appends the new ones to the state's, and cdb_merged_gc /
the GC flag pop it. Checked against the Python oracle's DB (oracle/constdb_oracle.py DB.gc, a line
restatement of db.rs:82-119) run through the same chain: merge 3 snapshots with gc(w1), merge 3 more
into the result with gc(w2), then 2 more and a standalone gc(w3) -- canonical dumps equal and the
garbage lists of equal length after every step. The watermarks stop the pops inside the lists, so
stale entries (keys deleted again later) and the entry lost at each stop both matter."""
import pytest

import constdb_amd as cdb
import constdb_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def db():
    from constdb_amd import build
    build.build()
    return cdb.DB(cdb.Context(0))


def _fold_into(odb, snaps):  # replica/pull.rs:116-159, as oracle.fold_snapshots, onto an existing DB
    for snap in snaps:
        for e in o.load_snapshot(snap):
            if e.kind == "Data":
                odb.merge_entry(*e.args)
            elif e.kind == "Deletes":
                odb.delete(*e.args)
            elif e.kind == "Expires":
                odb.expire_at(*e.args)


def _diff(got, want):
    gl, wl = got.split(b"\n"), want.split(b"\n")
    i = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b), min(len(gl), len(wl)))
    return f"first diff at line {i}: gpu {gl[i] if i < len(gl) else None!r} oracle {wl[i] if i < len(wl) else None!r}"


def _quantile_time(snaps, q):
    odb = o.DB()
    _fold_into(odb, snaps)
    ts = sorted(t for _, _, t in odb.garbages)
    return ts[int(q * (len(ts) - 1))]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gc_chain_vs_oracle(db, seed):
    cfg = cdb.gen_config(seed=700 + seed, universe=3000, n_replicas=8, replica_hi=8, conflict_ppm=20000,
                         tie_permille=100, side_permille=400, del_permille=300, mix_set=20, mix_dict=20)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    # (a snapshot lists its Deletes in hash order, so the pops stop after about 1 / (1 - q) entries)
    w1 = _quantile_time(snaps[:3], 0.95)
    w2 = _quantile_time(snaps, 0.97)
    w3 = _quantile_time(snaps, 0.99)
    odb = o.DB()
    _fold_into(odb, snaps[:3])
    odb.gc(w1)
    m1 = db.merge_snapshots(snaps[:3], gc_watermark=w1)
    assert m1.canonical_dump() == o.canonical_dump(odb), _diff(m1.canonical_dump(), o.canonical_dump(odb))
    assert m1.garbage_count == len(odb.garbages)
    _fold_into(odb, snaps[3:6])
    before = len(odb.deletes)
    odb.gc(w2)
    m2 = db.merge_into(m1, [cdb.decode_snapshot(s) for s in snaps[3:6]], gc_watermark=w2)
    want = o.canonical_dump(odb)
    assert m2.canonical_dump() == want, _diff(m2.canonical_dump(), want)
    assert m2.garbage_count == len(odb.garbages)
    assert m2.stats.deletes_gced == before - len(odb.deletes)
    _fold_into(odb, snaps[6:])
    m3 = db.merge_into(m2, [cdb.decode_snapshot(s) for s in snaps[6:]])
    assert m3.garbage_count == len(odb.garbages)
    before = len(odb.deletes)
    odb.gc(w3)
    assert m3.gc(w3) == before - len(odb.deletes)
    want = o.canonical_dump(odb)
    assert m3.canonical_dump() == want, _diff(m3.canonical_dump(), want)
    assert m3.garbage_count == len(odb.garbages)


def _snap(deletes):
    d = o.DB()
    d.deletes.update(deletes)
    return o.dump_all(d, o.NodeHeader())


def test_gc_chain_differs_from_one_merge(db):
    """Why the list is kept (the gc_lifo KAT carried over two MEETs): [A{a:5}, B{b:50}] merged with
    gc(10) pops b (50 > 10: popped and lost, the loop ends), so a stays in the list; merging C{c:6}
    into that with gc(10) pops c and then a -- deletes = {b}. The same three snapshots in one merge
    with gc(10) pop c, then stop at b: deletes = {a, b}. The oracle's DB agrees with the chain."""
    A, B, C = _snap({b"a": 5}), _snap({b"b": 50}), _snap({b"c": 6})
    odb = o.DB()
    _fold_into(odb, [A, B])
    odb.gc(10)
    assert [k for k, _, _ in odb.garbages] == [b"a"]
    _fold_into(odb, [C])
    odb.gc(10)
    assert odb.deletes == {b"b": 50} and odb.garbages == []
    m1 = db.merge_snapshots([A, B], gc_watermark=10)
    assert m1.garbage_count == 1
    chain = db.merge_into(m1, [cdb.decode_snapshot(C)], gc_watermark=10)
    assert chain.canonical_dump() == o.canonical_dump(odb) and chain.garbage_count == 0
    one = db.merge_snapshots([A, B, C], gc_watermark=10)
    assert one.canonical_dump() == f"R {b'a'.hex()} 5\nR {b'b'.hex()} 50\n".encode()
    assert one.canonical_dump() != chain.canonical_dump()
