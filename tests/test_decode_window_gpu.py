"""Decode into HBM of snapshots in the 64-512 MB window (snapshot.rs:120-220 then the merge
of pull.rs:120-128), where the decoder page-locks the CALLER's buffer and starts its upload before the host
index pass (decode_gpu.hip GpuDecode::index). Every case merges the decoded rows on the sorted-run path and
compares the canonical dump with the C++ oracle's sequential fold of the same snapshots:
  * three C4-shaped snapshots of ~118 MB each (DATAS deferred to the device index);
  * the same buffer passed twice (its second page-lock fails: that snapshot falls back to the batch copy);
  * a snapshot already in page-locked memory (its page-lock fails the same way);
  * a ~100 MB snapshot whose DATAS section is too short to defer (large Bytes values): the early upload
    with the host index pass only."""
import pytest
import torch

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs
from test_decode_merge_full_gpu import _merge, _release

pytestmark = pytest.mark.gpu

MB = 1 << 20


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


@pytest.fixture(scope="module")
def c4_snaps():
    cfg = configs.c4(cdb, 4_000_000)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(3)]
    assert all(64 * MB <= len(s) <= 512 * MB for s in snaps)
    return snaps


def _decode_merge(ctx, snaps, want_snaps=None):
    rc, want, ost = cdb_oracle.fold([bytes(s.numpy()) if hasattr(s, "numpy") else s for s in (want_snaps or snaps)])
    assert rc == 0
    batches, din = cdb.decode_snapshots_device(ctx, snaps, records=True)
    try:
        out, st = _merge(ctx, din, compact=False)
        got = cdb.merged_from_device(ctx, out, batches, stats=st).canonical_dump()
    finally:
        _release(ctx, din)
    assert got == want
    assert st.type_conflicts == ost.type_conflicts
    return st


def test_decode_window_early_upload_vs_oracle(ctx, c4_snaps):
    st = _decode_merge(ctx, c4_snaps)
    assert st.sorted_runs == 1


def test_decode_window_same_buffer_twice_vs_oracle(ctx, c4_snaps):
    _decode_merge(ctx, [c4_snaps[0], c4_snaps[0], c4_snaps[1]])


def test_decode_window_page_locked_caller_buffer_vs_oracle(ctx, c4_snaps):
    pinned = torch.empty(len(c4_snaps[0]), dtype=torch.uint8, pin_memory=True)
    pinned.copy_(torch.frombuffer(bytearray(c4_snaps[0]), dtype=torch.uint8))
    _decode_merge(ctx, [pinned, c4_snaps[1], c4_snaps[2]], want_snaps=[c4_snaps[0], c4_snaps[1], c4_snaps[2]])


def test_decode_window_short_datas_not_deferred_vs_oracle(ctx):
    cfg = cdb.gen_config(seed=11, universe=100_000, n_replicas=2, key_permille=900, mix_bytes=1, mix_counter=0,
                         mix_set=0, mix_dict=0, value_min=900, value_max=1100, replica_lo=0, replica_hi=2)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(2)]
    assert all(64 * MB <= len(s) <= 512 * MB for s in snaps)
    _decode_merge(ctx, snaps)
