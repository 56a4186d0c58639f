"""The records input layout and the bucket-layout result (cdb_merge.h: cdb_dev_rows.stride,
cdb_dev_output.compact = 0) against the oracle.

Records: the key-hash column plus one record of ncols - 1 words per row; on the sorted-run path the
wave kernel copies a bucket's record bytes into LDS with LDS-DMA (runs.hip.h load_runs_staged), the
other tiers and the partition path read them field by field. The bucket layout: the merge's own row
slots plus the bucket directory, read directly by cdb_dev_state_rows (the next merge's position 0)
and compacted on the way by cdb_merged_from_device / cdb_dev_output_compact. Every result is
compared byte for byte with the C++ oracle's sequential fold (oracle/cdb_oracle.cpp: db.rs:31-119,
object.rs:63-83, type_counter.rs:59-91, crdt/lwwhash.rs:87-128,319-323)."""
import ctypes

import pytest
import torch

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import sort_into_runs, to_records, wrap

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _arr(batches):
    return (ctypes.c_void_p * max(len(batches), 1))(*[b.handle for b in batches])


def _upload(ctx, batches, records):
    din = cdb.DevInput()
    ctx.check(cdb.lib().cdb_upload_batches(ctx.handle, _arr(batches), len(batches), ctypes.byref(din)))
    if records:
        to_records(cdb, ctx, din)
        assert din.keys.stride == 6 and din.nodes.stride == 5 and din.members.stride == 5
    return din


def _dense_out(ctx, din):
    L = cdb.lib()
    dout = cdb.DevOutput()
    for name, nc in (("keys", 8), ("nodes", 6), ("members", 6)):
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(din, name).n, nc))
        setattr(dout, name, r)
    dout.compact = 1
    return dout


def _release(ctx, *sets):
    L = cdb.lib()
    for s in sets:
        for name in ("keys", "nodes", "members"):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(s, name)))


def _merge(ctx, din, dout, **kw):
    opts = cdb.merge_opts(**kw)
    st = cdb.MergeStats()
    ctx.check(cdb.lib().cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(dout),
                                         ctypes.byref(st), None))
    return st


def _diff(got, want):
    gl, wl = got.split(b"\n"), want.split(b"\n")
    i = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b), min(len(gl), len(wl)))
    return (f"first diff at line {i}: gpu {gl[i][:200] if i < len(gl) else None!r} "
            f"oracle {wl[i][:200] if i < len(wl) else None!r} ({len(gl)} vs {len(wl)} lines)")


def merge_layout(ctx, snaps, records=True, buckets=True, runs=True, sections=False, **kw):
    """snaps decoded, uploaded in the given input layout (in runs or not), merged into the given
    result layout; returns (host view, stats)."""
    batches = [cdb.decode_snapshot(s) for s in snaps]
    din = _upload(ctx, batches, records)
    dense = None
    try:
        if runs:
            sort_into_runs(din, sections=sections)
        if buckets:
            dout = cdb.DevOutput()
            dout.compact = 0
        else:
            dout = dense = _dense_out(ctx, din)
        st = _merge(ctx, din, dout, **kw)
        assert st.sorted_runs == (1 if runs else 0)
        if buckets:
            assert dout.keys.stride == 8 and dout.keys.stride0 == 8 and dout.nodes.stride == 6
            assert dout.buckets.nb > 0 and dout.keys.n == st.key_rows_out
        return cdb.merged_from_device(ctx, dout, batches, stats=st), st
    finally:
        _release(ctx, din)
        if dense is not None:
            _release(ctx, dense)


def check(ctx, snaps, gc=None, gc_members=False, **kw):
    flags = (cdb_oracle.FLAG_GC if gc is not None else 0) | (cdb_oracle.FLAG_GC_MEMBERS if gc_members else 0)
    rc, want, ost = cdb_oracle.fold(snaps, flags=flags, gc_watermark=gc or 0)
    assert rc == 0
    m, st = merge_layout(ctx, snaps, gc_watermark=gc, gc_members=gc_members, **kw)
    got = m.canonical_dump()
    assert got == want, _diff(got, want)
    assert st.type_conflicts == ost.type_conflicts
    assert st.dict_merges == ost.dict_merges
    return st


def _small(seed, universe, replicas, **kw):
    base = dict(seed=seed, universe=universe, n_replicas=replicas, replica_hi=replicas)
    base.update(kw)
    return cdb.gen_config(**base)


@pytest.mark.parametrize("records,buckets", [(True, True), (True, False), (False, True)])
@pytest.mark.parametrize("seed", range(4))
def test_layouts_random_vs_oracle(ctx, seed, records, buckets):
    """Random states (type conflicts, ties, side maps, long member lists) in each input layout and
    result layout, on the sorted-run path."""
    cfg = _small(500 + seed, 3000 + 4000 * seed, 2 + 2 * seed, conflict_ppm=30000, tie_permille=150,
                 side_permille=250, mean_members=3 + 2 * seed, del_permille=300)
    check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(cfg.n_replicas)], records=records, buckets=buckets,
          sections=bool(seed % 2))


@pytest.mark.parametrize("tier", [1, 2, 3, 4])
def test_records_forced_tiers_vs_oracle(ctx, tier):
    """Every tier reading records: the workgroup tiers' materialisation, the chip-wide path's runs
    mode, the wide tier's field-by-field loads."""
    cfg = _small(540 + tier, 5000, 5, conflict_ppm=20000, side_permille=200, tie_permille=100, mean_members=6)
    check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(5)], force_tier=tier)


def test_records_partition_path_vs_oracle(ctx):
    """Records not in runs: the partition path reads them field by field (strided column sets)."""
    cfg = _small(551, 20000, 4, conflict_ppm=20000, side_permille=200, mean_members=4)
    check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(4)], runs=False)
    check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(4)], runs=False, buckets=False)


def test_records_gc_vs_oracle(ctx):
    cfg = _small(557, 20000, 4, mix_set=40, mix_dict=40, side_permille=300, del_permille=400)
    wm = (configs.T0_MS + (1 << 30)) << 22
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(4)]
    st = check(ctx, snaps, gc=wm, sections=True)
    assert st.deletes_gced > 0
    check(ctx, snaps, gc=wm, gc_members=True)


def test_records_c4_1m_vs_oracle(ctx):
    """C4's shape (the bench's generator config) at 1M keys x 8 replicas, records in, bucket layout out."""
    cfg = configs.c4(cdb, 1_000_000)
    st = check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(8)])
    assert st.key_rows_in > 4_000_000


def test_records_c5_300k_vs_oracle(ctx):
    """C5's hot keys from records: the chip-wide child path reads the children from the runs' records."""
    cfg = configs.c5(cdb, universe=300_000, events=3_000_000)
    st = check(ctx, [cdb.gen_snapshot(cfg, r) for r in range(8)])
    assert st.hot_buckets + st.mid_buckets > 0


def test_gen_device_records_equal_columns(ctx):
    """cdb_gen_device with CDB_GEN_ROWS_RECORDS writes the same rows as with columns."""
    L = cdb.lib()
    cfg = configs.c4(cdb, 200_000)
    a, b = cdb.DevInput(), cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(a)))
    cfg.flags |= cdb.GEN_ROWS_RECORDS
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(b)))
    try:
        for name, nc in (("keys", 7), ("nodes", 6), ("members", 6)):
            ra, rb = getattr(a, name), getattr(b, name)
            assert ra.n == rb.n and rb.stride == nc - 1
            assert torch.equal(wrap(ra.col[0], ra.n), wrap(rb.col[0], rb.n))
            rec = wrap(rb.col[1], rb.n * (nc - 1)).view(rb.n, nc - 1)
            for c in range(1, nc):
                assert torch.equal(wrap(ra.col[c], ra.n), rec[:, c - 1]), (name, c)
    finally:
        _release(ctx, a, b)


def test_bucket_layout_compacts_to_dense(ctx):
    """cdb_dev_output_compact of a bucket-layout result equals the compact = 1 merge of the same
    input, column for column (C4 shape, 500K keys)."""
    L = cdb.lib()
    cfg = configs.c4(cdb, 500_000)
    cfg.flags |= cdb.GEN_ROWS_RECORDS
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
    sort_into_runs(din)
    d1 = _dense_out(ctx, din)
    d2 = _dense_out(ctx, din)
    try:
        st1 = _merge(ctx, din, d1)
        b = cdb.DevOutput()
        b.compact = 0
        st2 = _merge(ctx, din, b)
        assert st1.key_rows_out == st2.key_rows_out == b.keys.n
        ctx.check(L.cdb_dev_output_compact(ctx.handle, ctypes.byref(b), ctypes.byref(d2), None))
        for name, nc in (("keys", 8), ("nodes", 6), ("members", 6)):
            r1, r2 = getattr(d1, name), getattr(d2, name)
            assert r1.n == r2.n
            for c in range(nc):
                assert torch.equal(wrap(r1.col[c], r1.n), wrap(r2.col[c], r2.n)), (name, c)
    finally:
        _release(ctx, din, d1, d2)


@pytest.mark.parametrize("records", [True, False])
def test_bucket_layout_state_chain_vs_oracle(ctx, records):
    """A result kept in HBM in the bucket layout becomes fold position 0 of the next merge through
    cdb_dev_state_rows (into records or columns, one run); the second merge, on the sorted-run path,
    equals the oracle's fold of every snapshot."""
    L = cdb.lib()
    cfg = _small(561, 40000, 5, conflict_ppm=20000, tie_permille=100, side_permille=150, mean_members=4)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(5)]
    b1 = [cdb.decode_snapshot(s) for s in snaps[:2]]
    b2 = [cdb.decode_snapshot(s) for s in snaps[2:]]
    din1 = _upload(ctx, b1, records)
    sort_into_runs(din1)
    out1 = cdb.DevOutput()
    out1.compact = 0
    st1 = _merge(ctx, din1, out1)
    state_host = cdb.merged_from_device(ctx, out1, b1, stats=st1)
    # position 0 = merge 1's result, then the new replicas at positions 1.., one input
    din2 = _upload(ctx, b2, False)
    K0, N0, M0 = out1.keys.n, out1.nodes.n, out1.members.n
    both = cdb.DevInput()
    alloc = L.cdb_dev_rows_alloc_records if records else L.cdb_dev_rows_alloc
    for f, (name, nc, n0) in enumerate((("keys", 7, K0), ("nodes", 6, N0), ("members", 6, M0))):
        r = cdb.DevRows()
        ctx.check(alloc(ctx.handle, ctypes.byref(r), n0 + getattr(din2, name).n, nc))
        setattr(both, name, r)
    ctx.check(L.cdb_dev_state_rows(ctx.handle, ctypes.byref(out1), ctypes.byref(both.keys), ctypes.byref(both.nodes),
                                   ctypes.byref(both.members), None))
    try:
        # append the new replicas' rows (pos + 1) behind the state rows, then runs by position
        for f, (name, nc, n0) in enumerate((("keys", 7, K0), ("nodes", 6, N0), ("members", 6, M0))):
            src, dst = getattr(din2, name), getattr(both, name)
            n = src.n
            dst.n = n0 + n
            if n:
                meta = wrap(src.col[nc - 1], n)
                meta.add_(1 << 48)
                wrap(dst.col[0], n0 + n)[n0:].copy_(wrap(src.col[0], n))
                if records:
                    rec = wrap(dst.col[1], (n0 + n) * (nc - 1)).view(n0 + n, nc - 1)
                    for c in range(1, nc):
                        rec[n0:, c - 1].copy_(wrap(src.col[c], n))
                else:
                    for c in range(1, nc):
                        # columns of a cdb_dev_rows_alloc block: stride n0 + n between columns
                        wrap(dst.col[c], n0 + n)[n0:].copy_(wrap(src.col[c], n))
            setattr(both, name, dst)
        torch.cuda.synchronize()
        both.n_pos = 1 + len(b2)
        sort_into_runs(both)
        out2 = cdb.DevOutput()
        out2.compact = 0
        st2 = _merge(ctx, both, out2)
        assert st2.sorted_runs == 1
        m = cdb.merged_from_device(ctx, out2, b2, state=state_host, stats=st2)
        rc, want, _ = cdb_oracle.fold(snaps)
        assert rc == 0
        got = m.canonical_dump()
        assert got == want, _diff(got, want)
    finally:
        _release(ctx, din1, din2, both)


@pytest.mark.parametrize("seed", [0, 1])
def test_decode_records_runs_vs_oracle(ctx, seed):
    """Snapshots this engine encoded (key-hash order) and the same replicas in generator order (the
    reference's HashMap order: no key order), decoded straight into HBM as records
    (CDB_DECODE_ROWS_RECORDS) -- the first placed as one run per snapshot by merging its sections, the
    second sorted into one run per snapshot on the device -- merged into the bucket layout on the
    sorted-run path through the staged loads: equal to the oracle. With CDB_DECODE_STREAM_ORDER the
    generator-order rows take the partition path from records."""
    cfg = _small(600 + seed, 30000, 4 + seed, conflict_ppm=20000, tie_permille=100, side_permille=300,
                 mix_set=20, mix_dict=20, del_permille=300)
    raw = [cdb.gen_snapshot(cfg, r) for r in range(cfg.n_replicas)]
    db = cdb.DB(ctx)
    encs = [db.merge_snapshots([x]).encode_snapshot(replicas=None)[0] for x in raw]
    for snaps, want_runs in ((encs, True), (raw, True), (raw, False)):
        rc, want, ost = cdb_oracle.fold(snaps)
        assert rc == 0
        batches, din = cdb.decode_snapshots_device(ctx, snaps, records=True, stream_order=not want_runs)
        try:
            assert din.keys.stride == 6 and (din.n_runs == len(snaps)) == want_runs
            out = cdb.DevOutput()
            out.compact = 0
            st = _merge(ctx, din, out)
            assert st.sorted_runs == (1 if want_runs else 0)
            got = cdb.merged_from_device(ctx, out, batches, stats=st).canonical_dump()
            assert got == want, _diff(got, want)
            assert st.type_conflicts == ost.type_conflicts
        finally:
            _release(ctx, din)


def _filtered(ctx, batches, key_lo, child_lo):
    """The batches uploaded as columns, keeping key rows with unsigned hash >= key_lo and child rows
    with unsigned parent hash >= child_lo (rows keep their meta, so bytes still resolve)."""
    L = cdb.lib()
    din = _upload(ctx, batches, False)
    out = cdb.DevInput()
    out.n_pos = din.n_pos
    keep = []
    for name, nc, lo in (("keys", 7, key_lo), ("nodes", 6, child_lo), ("members", 6, child_lo)):
        rows = getattr(din, name)
        cols = [wrap(rows.col[c], rows.n) for c in range(nc)] if rows.n else []
        sel = ((cols[0] ^ (-(1 << 63))) >= (lo - (1 << 63))) if rows.n else None
        r = cdb.DevRows()
        n = int(sel.sum()) if rows.n else 0
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), n, nc))
        for c in range(nc):
            if n:
                wrap(r.col[c], n).copy_(cols[c][sel])
        keep.append(r)
        setattr(out, name, r)
    torch.cuda.synchronize()
    _release(ctx, din)
    return out


def test_keyless_buckets_first_in_chip_wide_batches(ctx, monkeypatch):
    """buckets holding children but no key rows (orphans), placed first in chip-wide
    batches (every bucket chip-wide, small key-table batches): nothing is output for them, every
    child counts as an orphan, and the rest of the result equals the merge of the same input without
    those children (which the oracle tests pin)."""
    cfg = _small(611, 20000, 4, mix_set=40, mix_dict=30, mean_members=6, side_permille=100)
    batches = [cdb.decode_snapshot(cdb.gen_snapshot(cfg, r)) for r in range(4)]
    lo = 1 << 58  # the lowest 1/64 of the hash space: several buckets, no key rows left in them
    orphan_in = _filtered(ctx, batches, lo, 0)
    clean = _filtered(ctx, batches, lo, lo)
    try:
        n_orphans = (orphan_in.nodes.n - clean.nodes.n) + (orphan_in.members.n - clean.members.n)
        assert n_orphans > 0
        sort_into_runs(orphan_in)
        sort_into_runs(clean)
        monkeypatch.setenv("CDB_HOT_KEY_CAP", "1500")
        o1 = cdb.DevOutput()
        st1 = _merge(ctx, orphan_in, o1, force_tier=2)
        got = cdb.merged_from_device(ctx, o1, batches, stats=st1).canonical_dump()
        monkeypatch.delenv("CDB_HOT_KEY_CAP")
        o2 = cdb.DevOutput()
        st2 = _merge(ctx, clean, o2)
        want = cdb.merged_from_device(ctx, o2, batches, stats=st2).canonical_dump()
        assert got == want, _diff(got, want)
        assert st1.orphan_children == n_orphans and st2.orphan_children == 0
        assert st1.key_rows_out == st2.key_rows_out
    finally:
        _release(ctx, orphan_in, clean)


@pytest.mark.parametrize("records", [False, True])
def test_decode_reference_order_sorted_vs_oracle(ctx, records):
    """The reference's HashMap-order dumps (the Python oracle's writer iterates its dict in insertion
    order, not key order) with every kind of entry, expires and deletes, decoded into HBM: every
    snapshot becomes one run (sorted on the device), the merge takes the sorted-run path, and the
    result -- with DB::gc -- equals the oracle's fold; C4's shape at 200K keys too."""
    from snapgen import gen_replicas
    snaps = gen_replicas(31, n_replicas=5, n_keys=3000, p_conflict=0.05, p_side=0.3)
    cfg = configs.c4(cdb, 200_000)
    for group, wm in ((snaps, None), (snaps, (configs.T0_MS + (1 << 30)) << 22),
                      ([cdb.gen_snapshot(cfg, r) for r in range(8)], None)):
        flags = cdb_oracle.FLAG_GC if wm is not None else 0
        rc, want, ost = cdb_oracle.fold(group, flags=flags, gc_watermark=wm or 0)
        assert rc == 0
        batches, din = cdb.decode_snapshots_device(ctx, group, records=records)
        try:
            assert din.n_runs == len(group)
            out = cdb.DevOutput()
            st = _merge(ctx, din, out, gc_watermark=wm)
            assert st.sorted_runs == 1
            got = cdb.merged_from_device(ctx, out, batches, stats=st).canonical_dump()
            assert got == want, _diff(got, want)
            assert st.type_conflicts == ost.type_conflicts
        finally:
            _release(ctx, din)
