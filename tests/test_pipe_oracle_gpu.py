"""The headline kernel against the oracle: bucket_wave_pipe_kernel (runs.hip.h), the persistent wave
tier that folds ~95 % of C4's buckets in the bench step.

It runs from kPipeMinBuckets (2^19) buckets on (engine.hip), so C4 at 1M keys (~108K buckets) would
take round 4's one-bucket-per-wave kernel. CDB_WAVE_PIPE=force runs it at any bucket count, and
stats.wave_pipe_buckets counts the buckets it folded, so every case below asserts that the kernel
under test is the one that folded. Compared byte for byte (canonical dump) with the C++ oracle's
sequential fold (oracle/cdb_oracle.cpp: db.rs:31-43, object.rs:63-83 -- the Bytes LWW arm, 60 % of
C4's keys -- type_counter.rs:59-91 with 1-8 nodes per counter, lwwhash.rs:87-128,319-323):
  * C4's shape at 1M keys x 8 replicas, forced, in both layouts the kernel is instantiated for
    (records: the bench's input; plain columns), as generator-order snapshots sorted into runs on the
    device, and as snapshots encoded from merge results (each replica merged alone and written back
    -- the state runs the bench times: children in child order);
  * the same with DB::gc of Deletes (db.rs:82-119);
  * C4 at a 5M-key universe (~530K buckets), where the kernel runs without the hook;
  * small random states (type conflicts, time ties, side maps, few buckets per XCD slab), forced.
Round 6: the kernel's unit is a group of consecutive buckets (runs.hip.h, pipe_units_kernel); every case
asserts that groups formed (stats.wave_pipe_units < wave_pipe_buckets), and CDB_GROUPS=0 (one bucket
per unit, round-5 bucket sizes) is pinned to the oracle as well."""
import ctypes

import pytest

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import sort_into_runs

pytestmark = pytest.mark.gpu

NAMES = ("keys", "nodes", "members")


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _release(ctx, *sets):
    for s in sets:
        for name in NAMES:
            cdb.lib().cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(s, name)))


def _diff(got, want):
    gl, wl = got.split(b"\n"), want.split(b"\n")
    i = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b), min(len(gl), len(wl)))
    return (f"first diff at line {i}: gpu {gl[i][:200] if i < len(gl) else None!r} "
            f"oracle {wl[i][:200] if i < len(wl) else None!r} ({len(gl)} vs {len(wl)} lines)")


def _merge_vs_oracle(ctx, snaps, records, gc=None, upload=False):
    """snaps decoded into HBM (GPU decoder, one run per snapshot; or host decode + upload as plain
    columns put in runs), merged into the bucket layout, dumped; returns the merge stats."""
    flags = cdb_oracle.FLAG_GC if gc is not None else 0
    rc, want, ost = cdb_oracle.fold(snaps, flags=flags, gc_watermark=gc or 0)
    assert rc == 0
    L = cdb.lib()
    if upload:
        batches = [cdb.decode_snapshot(s) for s in snaps]
        din = cdb.DevInput()
        arr = (ctypes.c_void_p * len(batches))(*[b.handle for b in batches])
        ctx.check(L.cdb_upload_batches(ctx.handle, arr, len(batches), ctypes.byref(din)))
        sort_into_runs(din)
    else:
        batches, din = cdb.decode_snapshots_device(ctx, snaps, records=records)
        if din.n_runs == 0:  # (a snapshot decoded on the host tier stays in stream order)
            sort_into_runs(din)
    assert (din.keys.stride == 6) == records
    out = cdb.DevOutput()
    out.compact = 0
    st = cdb.MergeStats()
    try:
        assert din.n_runs == len(snaps)
        ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.merge_opts(gc_watermark=gc)),
                                     ctypes.byref(out), ctypes.byref(st), None))
        got = cdb.merged_from_device(ctx, out, batches, stats=st).canonical_dump()
    finally:
        _release(ctx, din)
    assert st.sorted_runs == 1
    assert got == want, _diff(got, want)
    assert (st.type_conflicts, st.dict_merges) == (ost.type_conflicts, ost.dict_merges)
    return st


def _assert_pipe_folded_most(st, grouped=True):
    """The persistent kernel folded the bulk of the buckets (the rest: the wide tier, 65..128 key
    rows or 129..256 children, and the workgroup tiers), in groups of several buckets per unit."""
    assert st.wave_pipe_buckets > 0
    assert st.wave_pipe_buckets > 5 * (st.wide_buckets + st.mid_buckets + st.hot_buckets)
    if grouped:
        assert 0 < st.wave_pipe_units < 0.8 * st.wave_pipe_buckets
    else:
        assert st.wave_pipe_units == st.wave_pipe_buckets


@pytest.fixture(scope="module")
def c4_1m():
    cfg = configs.c4(cdb, 1_000_000)
    return [cdb.gen_snapshot(cfg, r) for r in range(8)]


@pytest.fixture(scope="module")
def c4_1m_states(ctx, c4_1m):
    """Each replica as this engine keeps it: merged alone and encoded (server.rs:183-215) -- DATAS,
    EXPIRES, DELETES in key-hash order, every key's children in child_order (common.h)."""
    db = cdb.DB(ctx)
    return [db.merge_snapshots([s]).encode_snapshot(replicas=None)[0] for s in c4_1m]


@pytest.mark.parametrize("records", [True, False])
def test_pipe_forced_c4_1m_vs_oracle(ctx, monkeypatch, c4_1m, records):
    monkeypatch.setenv("CDB_WAVE_PIPE", "force")
    st = _merge_vs_oracle(ctx, c4_1m, records)
    assert st.key_rows_in > 4_000_000
    _assert_pipe_folded_most(st)
    monkeypatch.setenv("CDB_WAVE_PIPE", "0")  # the hook really switches kernels
    assert _merge_vs_oracle(ctx, c4_1m, records).wave_pipe_buckets == 0


def test_pipe_forced_c4_1m_one_bucket_units_vs_oracle(ctx, monkeypatch, c4_1m):
    monkeypatch.setenv("CDB_WAVE_PIPE", "force")
    monkeypatch.setenv("CDB_GROUPS", "0")
    _assert_pipe_folded_most(_merge_vs_oracle(ctx, c4_1m, records=True), grouped=False)


def test_pipe_forced_c4_1m_plain_columns_upload_vs_oracle(ctx, monkeypatch, c4_1m):
    monkeypatch.setenv("CDB_WAVE_PIPE", "force")
    _assert_pipe_folded_most(_merge_vs_oracle(ctx, c4_1m, records=False, upload=True))


def test_pipe_forced_c4_1m_state_runs_vs_oracle(ctx, monkeypatch, c4_1m_states):
    monkeypatch.setenv("CDB_WAVE_PIPE", "force")
    st = _merge_vs_oracle(ctx, c4_1m_states, records=True)
    _assert_pipe_folded_most(st)


def test_pipe_forced_c4_1m_gc_vs_oracle(ctx, monkeypatch, c4_1m_states):
    monkeypatch.setenv("CDB_WAVE_PIPE", "force")
    # (a watermark after every time: DB::gc pops the whole garbage list -- with a mid watermark the
    # LIFO stop comes within a few entries of the end of a hash-ordered list)
    gc = (configs.T0_MS + (1 << 30)) << 22
    st = _merge_vs_oracle(ctx, c4_1m_states, records=True, gc=gc)
    _assert_pipe_folded_most(st)
    assert st.deletes_gced > 0
    _merge_vs_oracle(ctx, c4_1m_states, records=True, gc=(configs.T0_MS + (1 << 18)) << 22)


@pytest.mark.timeout(900)
def test_pipe_natural_c4_5m_vs_oracle(ctx, monkeypatch):
    """C4 at a 5M-key universe x 8 replicas (~21M key rows, > 2^19 buckets): the persistent kernel
    runs without the hook, on the state runs (encoded merge results) the bench times."""
    monkeypatch.delenv("CDB_WAVE_PIPE", raising=False)
    cfg = configs.c4(cdb, 5_000_000)
    db = cdb.DB(ctx)
    snaps = []
    for r in range(8):
        snaps.append(db.merge_snapshots([cdb.gen_snapshot(cfg, r)]).encode_snapshot(replicas=None)[0])
    st = _merge_vs_oracle(ctx, snaps, records=True)
    assert st.key_rows_in > 20_000_000
    _assert_pipe_folded_most(st)


@pytest.mark.parametrize("seed", range(6))
def test_pipe_forced_random_vs_oracle(ctx, monkeypatch, seed):
    """Small random states (a few hundred buckets: XCD slabs of a few buckets, empty chunks)."""
    monkeypatch.setenv("CDB_WAVE_PIPE", "force")
    cfg = cdb.gen_config(seed=600 + seed, universe=500 + 3000 * seed, n_replicas=1 + seed % 8,
                         replica_hi=1 + seed % 8, conflict_ppm=30000, tie_permille=150, side_permille=250,
                         mean_members=3 + seed, del_permille=300)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(cfg.n_replicas)]
    st = _merge_vs_oracle(ctx, snaps, records=bool(seed % 2))
    assert st.wave_pipe_buckets > 0
    assert st.wave_pipe_units < st.wave_pipe_buckets


def test_pipe_pipelined_ranges_dense_vs_oracle(ctx, monkeypatch, c4_1m):
    """Dense output with the bucket phase in 8 ranges (cdb_merge_opts.pipe_ranges): the unit bitmap
    starts a unit at every range start, so no group spans two ranges' compactions."""
    from test_runs_oracle_gpu import runs_merge
    monkeypatch.setenv("CDB_WAVE_PIPE", "force")
    rc, want, _ = cdb_oracle.fold(c4_1m)
    assert rc == 0
    m = runs_merge(ctx, c4_1m, pipe_ranges=8)
    assert m.canonical_dump() == want
    st = m.stats
    assert 0 < st.wave_pipe_units < 0.8 * st.wave_pipe_buckets
