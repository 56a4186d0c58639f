"""The GPU decode's host index pass with a large DATAS section split over threads (speculative
sync points, stitched in order: constdb_amd/csrc/decode.cpp parallel_datas) must equal the
sequential pass entry for entry, status and offset included. CPU only (cdb_snapshot_index_selftest
needs no device)."""
import ctypes
import random

import pytest

import constdb_amd as cdb


def _check(snap, threads=8, flags=0):
    n = ctypes.c_uint64()
    st = cdb.lib().cdb_snapshot_index_selftest(bytes(snap), len(snap), flags, threads, ctypes.byref(n))
    assert st == cdb.OK, "parallel index differs from the sequential pass"
    return n.value


@pytest.mark.parametrize("seed,threads", [(1, 2), (2, 8), (3, 16), (4, 13)])
def test_generator_snapshots(seed, threads):
    cfg = cdb.gen_config(seed=seed, universe=300_000, n_replicas=2, replica_hi=2, mix_set=20, mix_dict=20,
                         mean_members=4, side_permille=300)
    n = _check(cdb.gen_snapshot(cfg, 0), threads)
    assert n > (1 << 17)


def test_big_objects_and_tiny_ranges():
    """Objects of thousands of members (an entry longer than a thread's range) and many threads."""
    cfg = cdb.gen_config(seed=9, universe=200_000, n_replicas=1, replica_hi=1, mix_set=30, mean_members=40)
    _check(cdb.gen_snapshot(cfg, 0), 64)


def test_truncated_and_corrupted():
    """Errors on the true chain hand the section back to the sequential pass: same status and
    offset; corruption elsewhere changes nothing."""
    cfg = cdb.gen_config(seed=5, universe=200_000, n_replicas=1, replica_hi=1)
    snap = cdb.gen_snapshot(cfg, 0)
    rng = random.Random(1)
    for cut in rng.sample(range(100, len(snap)), 6):
        _check(snap[:cut], 8)
    for pos in rng.sample(range(100, len(snap)), 12):
        bad = bytearray(snap)
        bad[pos] ^= 0xFF
        _check(bytes(bad), 8)


def test_small_snapshot_stays_sequential():
    cfg = cdb.gen_config(seed=6, universe=2000, n_replicas=1, replica_hi=1)
    _check(cdb.gen_snapshot(cfg, 0), 8)
