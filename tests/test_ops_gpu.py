"""Op-stream apply on the GPU through the C ABI: cdb_decode_ops + cdb_apply_ops on
top of a GPU merge result, against the hand-derived answers and the oracle
(constdb_ops_oracle.apply_replicates on the oracle's fold), byte for byte on canonical dumps."""
import pytest
import torch  # noqa: F401  -- before libcdbmerge loads: one HIP runtime per process

import constdb_amd as cdb
import constdb_oracle as o
import constdb_ops_oracle as oo
from ops_kats import cases
from opsgen import gen_stream
from snapgen import gen_replicas

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def db():
    from constdb_amd import build
    build.build()
    return cdb.DB(cdb.Context(0))


def _diff(got: bytes, want: bytes):
    gl, wl = got.decode().splitlines(), want.decode().splitlines()
    for i, (a, b) in enumerate(zip(gl, wl)):
        if a != b:
            return f"first diff at line {i}:\n gpu   : {a}\n oracle: {b}"
    return f"length differs: gpu {len(gl)} lines, oracle {len(wl)} lines"


def _gpu_apply(db, snaps, stream, u0):
    m = db.merge_snapshots(snaps)
    before = m.canonical_dump()
    m2 = m.apply_ops(cdb.decode_ops(stream, u0))
    assert m.canonical_dump() == before  # the state result is left unchanged
    return m2


@pytest.mark.parametrize("case", cases(), ids=lambda c: c[0])
def test_kat_gpu(db, case):
    name, snap, stream, u0, want = case
    got = _gpu_apply(db, [snap], stream, u0).canonical_dump().decode()
    assert got == want


def _parity(db, snaps, stream, u0=5):
    odb = o.fold_snapshots(snaps)
    st = oo.apply_replicates(odb, stream, u0)
    want = o.canonical_dump(odb)
    ops = cdb.decode_ops(stream, u0)
    m2 = db.merge_snapshots(snaps).apply_ops(ops)
    got = m2.canonical_dump()
    assert got == want, _diff(got, want)
    assert ops.info().cmd_errors + m2.apply_stats.type_errors == st.cmd_errors
    return m2


@pytest.mark.parametrize("seed", range(60))
def test_random_parity(db, seed):
    snaps = gen_replicas(seed, n_replicas=1 + seed % 3)
    keys = list(o.fold_snapshots(snaps).data) + [b"x%d" % i for i in range(3)]
    _parity(db, snaps, gen_stream(seed, keys, n_cmds=60 + 7 * seed))


@pytest.mark.parametrize("seed", range(4))
def test_random_parity_large(db, seed):
    # more events than one sort tile (2048) in every family; skewed key choice
    snaps = gen_replicas(100 + seed, n_replicas=2, n_keys=1500, n_members=12, n_nodes=6)
    keys = list(o.fold_snapshots(snaps).data)
    _parity(db, snaps, gen_stream(100 + seed, keys[:300] * 5 + keys, n_cmds=6000, t_range=40))


def test_empty_inputs(db):
    snap = o.dump_all(o.DB(), o.NodeHeader())
    assert _gpu_apply(db, [snap], b"", 0).canonical_dump() == b""
    _parity(db, gen_replicas(7), b"")
    _parity(db, [snap], oo.StreamBuilder(1, 5).cmd(6, "incr", b"c").bytes())


def test_chained_applies(db):
    snaps = gen_replicas(11, n_replicas=2)
    keys = list(o.fold_snapshots(snaps).data)
    s1 = gen_stream(1, keys, n_cmds=120, hazards=False)
    st = oo.StreamBuilder(3, 0)
    odb = o.fold_snapshots(snaps)
    a = oo.apply_replicates(odb, s1, 5)
    s2 = gen_stream(2, keys, n_cmds=120, hazards=False, uuid_he_sent=a.uuid_he_sent)
    oo.apply_replicates(odb, s2, a.uuid_he_sent)
    m = db.merge_snapshots(snaps).apply_ops(cdb.decode_ops(s1, 5)).apply_ops(cdb.decode_ops(s2, a.uuid_he_sent))
    assert m.canonical_dump() == o.canonical_dump(odb)
    del st


def test_hot_key(db):
    # one key owns thousands of members and ops (a long segment in every fold)
    sb = oo.StreamBuilder(2, 5)
    for i in range(3000):
        sb.cmd(6 + i % 50, ["sadd", "srem", "delset"][i % 7 % 3], b"hot", b"m%d" % (i % 900))
    snap = o.dump_all(o.DB(), o.NodeHeader())
    _parity(db, [snap], sb.bytes())


@pytest.mark.parametrize("zipf", [0, 900])
def test_generated_stream_parity(db, zipf):
    # the bench's generator (cdb_gen_ops) on a small universe, against the oracle
    cfg = cdb.gen_config(seed=5 + zipf, universe=3000, n_replicas=2)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(2)]
    stream = cdb.gen_ops(cfg, 20000, 0, zipf)
    m2 = _parity(db, snaps, stream, 0)
    assert m2.apply_stats.ops_in == 20000
