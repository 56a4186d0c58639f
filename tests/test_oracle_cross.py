"""The C++ oracle (oracle/cdb_oracle.cpp) must agree with the Python restatement."""
import pytest

import cdb_oracle
import constdb_oracle as o
from snapgen import gen_replicas


def _py(snaps, gc=None, members=False):
    db = o.fold_snapshots(snaps)
    if gc is not None:
        db.gc(gc)
    if members:
        db.gc_member_tombstones(gc)
    return o.canonical_dump(db), db


@pytest.mark.parametrize("seed", range(40))
def test_cpp_oracle_matches_python(seed):
    snaps = gen_replicas(seed, n_replicas=1 + seed % 5, big_times=seed % 2 == 1)
    want, db = _py(snaps)
    rc, got, st = cdb_oracle.fold(snaps)
    assert rc == 0
    assert got == want
    assert st.type_conflicts == db.type_conflicts and st.dict_merges == db.dict_merges


@pytest.mark.parametrize("seed", range(10))
def test_cpp_oracle_gc_matches_python(seed):
    snaps = gen_replicas(100 + seed, n_replicas=4, p_side=0.4)
    wm = 4
    want, _ = _py(snaps, gc=wm, members=True)
    rc, got, _ = cdb_oracle.fold(snaps, flags=cdb_oracle.FLAG_GC | cdb_oracle.FLAG_GC_MEMBERS,
                                 gc_watermark=wm)
    assert rc == 0 and got == want


def test_cpp_oracle_errors():
    snaps = gen_replicas(7, n_replicas=2)
    bad = bytearray(snaps[1])
    bad[-3] ^= 0x10
    rc, _, st = cdb_oracle.fold([snaps[0], bytes(bad)])
    assert rc == 2 and st.err_snapshot == 1          # InvalidSnapshotChecksum
    rc, _, _ = cdb_oracle.fold([snaps[0][:-20]])
    assert rc == 4                                   # IoError (EOF)
    rc, _, _ = cdb_oracle.fold(snaps, flags=cdb_oracle.FLAG_REFERENCE_CHECKSUM)
    assert rc in (2, 4)                              # the reference loader's quirk
