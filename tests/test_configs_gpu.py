"""BASELINE.json configs C1/C2, C3 and C5 on the GPU, bit-exact against the C++
oracle's sequential fold (oracle/cdb_oracle.cpp, restating db.rs:31-119, object.rs:63-83,
type_counter.rs:59-91, crdt/lwwhash.rs:87-128,319-323):
  * C1/C2 at full size (1M Bytes + 1M counters per node, 50 % overlap) through cdb_merge, the
    host-boundary FFI call a Rust puller would make (pull.rs:120-128);
  * C3 at full size: 4 replica states, each left by replaying 10M sadd/srem/hset/hdel through the
    device op apply, merged with DB::gc at the median member time;
  * C5 (Zipf hot keys) at sizes the oracle folds in seconds, whose hottest keys own 10^4-10^5
    children (the over-capacity bucket tiers).
The device generator (the bench's inputs) is checked row for row against the host writer
(the oracle's inputs) on every config."""
import ctypes

import numpy as np
import pytest
import torch  # noqa: F401  -- before libcdbmerge loads (one HIP runtime per process)

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs

pytestmark = pytest.mark.gpu

NCOLS = (7, 6, 6)


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _check(ctx, snaps, gc=None, tier=0, want=None):
    flags = cdb_oracle.FLAG_GC if gc is not None else 0
    if want is None:
        rc, want, ost = cdb_oracle.fold(snaps, flags=flags, gc_watermark=gc or 0)
        assert rc == 0
    else:
        want, ost = want
    m = cdb.DB(ctx).merge_snapshots(snaps, gc_watermark=gc, force_tier=tier)
    got = m.canonical_dump()
    if got != want:
        gl, wl = got.split(b"\n"), want.split(b"\n")
        i = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b), min(len(gl), len(wl)))
        raise AssertionError(f"first diff at line {i}: gpu {gl[i][:200] if i < len(gl) else None!r} "
                             f"oracle {wl[i][:200] if i < len(wl) else None!r} ({len(gl)} vs {len(wl)} lines)")
    assert m.stats.type_conflicts == ost.type_conflicts
    assert m.stats.dict_merges == ost.dict_merges
    return m


def _rows_multiset(cols, fam):
    """Rows of one family as a sorted structured array, src stripped from meta (the device
    generator's src are model coordinates, a decoded batch's are row indices)."""
    arr = np.stack(cols, axis=1).astype(np.uint64)
    meta = NCOLS[fam] - 1
    arr[:, meta] &= np.uint64(0xFFFF000000000000)
    v = arr.view([(f"c{i}", np.uint64) for i in range(arr.shape[1])]).ravel()
    return np.sort(v)


def _device_matches_host(ctx, cfg, replicas):
    L = cdb.lib()
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
    try:
        batches = [cdb.decode_snapshot(cdb.gen_snapshot(cfg, r)) for r in range(replicas)]
        for fam, rows in enumerate((din.keys, din.nodes, din.members)):
            dev = [(_wrap(rows.col[c], rows.n).cpu().numpy().view(np.uint64) if rows.n else np.zeros(0, np.uint64))
                   for c in range(NCOLS[fam])]
            host = []
            for c in range(NCOLS[fam]):
                parts = []
                for r, b in enumerate(batches):
                    col = b.column_array(fam, c)
                    if c == NCOLS[fam] - 1:  # the decoder leaves pos 0: the fold position is the batch index
                        col = (col & np.uint64(0xFF00FFFFFFFFFFFF)) | np.uint64(r << 48)
                    parts.append(col)
                host.append(np.concatenate(parts) if parts else np.zeros(0, np.uint64))
            assert len(dev[0]) == len(host[0]), (fam, len(dev[0]), len(host[0]))
            if len(dev[0]):
                assert (_rows_multiset(dev, fam) == _rows_multiset(host, fam)).all(), fam
    finally:
        for fam in (din.keys, din.nodes, din.members):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))


def _wrap(ptr, n):
    """A torch view of n int64 at device address ptr (owned by the library)."""
    class _Cai:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 2}
    return torch.as_tensor(_Cai(), device="cuda")


# ------------------------------------------------------------------ C1 / C2
def test_c1_device_generator_matches_host(ctx):
    _device_matches_host(ctx, configs.c1(cdb, per_node=20_000), 2)


def test_c1_full_size_bit_exact(ctx):
    """C1/C2: the 2-node MEET at its stated size through the host-boundary cdb_merge."""
    cfg = configs.c1(cdb)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(2)]
    m = _check(ctx, snaps)
    st = m.stats
    assert 3_900_000 < st.key_rows_in < 4_100_000          # 4M key rows in
    assert 2_900_000 < st.key_rows_out < 3_100_000         # 3M out (50 % overlap)
    assert 1_900_000 < st.node_rows_in < 2_100_000        # one node per counter


# ------------------------------------------------------------------ C3
def test_c3_full_size_bit_exact(ctx, c3_snaps):
    """C3: 4 replica states from 10M sadd/srem/hset/hdel each (device op apply on a synced state
    holding Expires and Deletes), merged with DB::gc at the median member time; bit-exact against
    the oracle's fold + gc. Every replica agrees on a key's type, and GC removes Deletes."""
    snaps = c3_snaps
    batches = [cdb.decode_snapshot(s) for s in snaps]
    wm = configs.median_member_time(cdb, batches)
    assert wm > 0
    assert sum(b.info().n_deletes for b in batches) > 0
    m = _check(ctx, snaps)
    assert m.stats.member_rows_in > 1_000_000
    assert m.stats.type_conflicts < 0.01 * m.stats.key_rows_in
    g = _check(ctx, snaps, gc=wm)
    assert g.stats.deletes_gced > 0


# ------------------------------------------------------------------ C5
def test_c5_device_generator_matches_host(ctx):
    _device_matches_host(ctx, configs.c5(cdb, universe=50_000, events=400_000), 8)


@pytest.mark.parametrize("universe,events", [(100_000, 800_000), (300_000, 3_000_000)])
def test_c5_scaled_bit_exact(ctx, universe, events):
    cfg = configs.c5(cdb, universe=universe, events=events)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    m = _check(ctx, snaps)
    assert m.stats.hot_buckets + m.stats.mid_buckets > 0


def test_c5_pipelined_ranges_bit_exact(ctx):
    """C5 with the bucket phase in 8 ranges (cdb_merge_opts.pipe_ranges; automatic only from 64M
    rows): bit-exact against the oracle although the workgroup tiers add outputs after the ranges."""
    cfg = configs.c5(cdb, universe=100_000, events=800_000)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    rc, want, ost = cdb_oracle.fold(snaps)
    assert rc == 0
    m = cdb.DB(ctx).merge_snapshots(snaps, pipe_ranges=8)
    assert m.canonical_dump() == want
    assert m.stats.hot_buckets + m.stats.mid_buckets > 0


def test_c3_chip_wide_child_path_repeatable(ctx):
    """Every bucket of a C3 merge through the over-capacity tier (force_tier=2: key table, tag
    sort, per-run fold): bit-exact three times over. The tag sort keeps rows of one (key,
    child) in input order, which varies from merge to merge, so the fold must not depend on it."""
    snaps = configs.c3_snapshots(cdb, ctx, ops_per_replica=200_000)
    rc, want, ost = cdb_oracle.fold(snaps)
    assert rc == 0
    for _ in range(3):
        _check(ctx, snaps, tier=2, want=(want, ost))


def test_c5_child_id_collisions(ctx, monkeypatch):
    """Tags with 6 child-id hash bits: most runs hold several exact ids, folded by successor
    selection instead of the one-id linear pass."""
    monkeypatch.setenv("CDB_HOT_ID_BITS", "6")
    cfg = configs.c5(cdb, universe=50_000, events=400_000)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    m = _check(ctx, snaps, tier=2)
    assert m.stats.hot_buckets > 0
    slow = m.stats.hot_slow_runs
    assert slow > 0
    monkeypatch.delenv("CDB_HOT_ID_BITS")
    m = _check(ctx, snaps, tier=2)  # sized id bits: about 1 run in 1000 takes the selection path
    assert m.stats.hot_slow_runs * 20 < slow
