"""The reference-asserted op streams of bin/test.rs:122-396 (tests/golden/bintest_*, see
tests/test_bintest.py) through the GPU: the replicate stream decoded (cdb_decode_ops) and applied on
the device (cdb_apply_ops) to the empty state must give the frozen dump and answer the
test's model (GET / SMEMBERS / HGETALL); and the three converged replicas, written back as snapshots
(cdb_encode_snapshot) and merged by the snapshot merge (every replica holds the same state after
bin/test.rs's sync: the merge must leave it as it is), answer the same model."""
import pytest
import torch  # noqa: F401  -- before libcdbmerge loads: one HIP runtime per process

import constdb_amd as cdb
from test_bintest import CASES, check_model, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def db():
    from constdb_amd import build
    build.build()
    return cdb.DB(cdb.Context(0))


@pytest.mark.parametrize("name", CASES)
def test_gpu_op_apply_and_merge_answer_the_reference_model(db, name):
    state, stream, want, meta = load(name)
    ops = cdb.decode_ops(stream, meta["uuid_he_sent"])
    m = db.merge_snapshots([state]).apply_ops(ops)
    got = m.canonical_dump()
    assert got == want
    check_model(got, meta["pinning"]["model"])
    snap, _ = m.encode_snapshot(replicas=None)
    merged = db.merge_snapshots([snap, snap, snap]).canonical_dump()
    assert merged == want
    check_model(merged, meta["pinning"]["model"])
