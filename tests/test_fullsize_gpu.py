"""What the bench lines time, checked at the size they time it.

* C5 at its bench size (10M keys, 80M Zipf-skewed child events, 8 replicas): the replicas' snapshots
  decoded into HBM as records, laid out as one key-hash-ordered run each, merged by cdb_merge_device into the
  bucket layout -- the chip-wide child path with its global sort for keys of 10^4..10^7 children --
  and the canonical dump compared byte for byte with the C++ oracle's sequential fold of the same
  snapshots (Counter::merge type_counter.rs:59-87, LWWHash::set / Set::merge lwwhash.rs:87-107,
  319-323).
* C4's shard in the bench's exact mode (records in, bucket layout out, one run per replica): the
  result, compacted, equals row for row the merge of the same rows as plain columns into dense
  columns, and holds the full-size invariants of test_runs_oracle_gpu.py (key-hash order, child
  ranges tiling the children, counter sums, a second merge bit-identical)."""
import ctypes
import hashlib

import pytest
import torch

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import SIGN, sort_into_runs, wrap

pytestmark = pytest.mark.gpu

NC = (("keys", 8), ("nodes", 6), ("members", 6))


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _release(ctx, *sets):
    for s in sets:
        for name, _ in NC:
            cdb.lib().cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(s, name)))


def _merge(ctx, din, dense):
    L = cdb.lib()
    out = cdb.DevOutput()
    if dense:
        for name, nc in NC:
            r = cdb.DevRows()
            ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(din, name).n, nc))
            setattr(out, name, r)
    out.compact = 1 if dense else 0
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.merge_opts()), ctypes.byref(out),
                                 ctypes.byref(st), None))
    return out, st


def _cols(out):
    return [torch.stack([wrap(getattr(out, name).col[c], getattr(out, name).n) for c in range(nc)]).clone()
            for name, nc in NC]


def _compacted(ctx, out):
    """A bucket-layout result as dense columns (cdb_dev_output_compact into fresh rows)."""
    L = cdb.lib()
    dense = cdb.DevOutput()
    for name, nc in NC:
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(out, name).n, nc))
        setattr(dense, name, r)
    dense.compact = 1
    ctx.check(L.cdb_dev_output_compact(ctx.handle, ctypes.byref(out), ctypes.byref(dense), None))
    cols = _cols(dense)
    _release(ctx, dense)
    return cols


def _first_diff(got, want):
    gl, wl = got.split(b"\n"), want.split(b"\n")
    i = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b), min(len(gl), len(wl)))
    return (f"first diff at line {i}: gpu {gl[i][:200] if i < len(gl) else None!r} "
            f"oracle {wl[i][:200] if i < len(wl) else None!r} ({len(gl)} vs {len(wl)} lines)")


@pytest.mark.timeout(1500)
def test_c5_bench_size_vs_oracle(ctx):
    cfg = configs.c5(cdb)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    rc, want, ost = cdb_oracle.fold(snaps)
    assert rc == 0
    batches, din = cdb.decode_snapshots_device(ctx, snaps, records=True)
    del snaps
    try:
        assert din.keys.stride == 6
        if din.n_runs == 0:
            # a key with more children than the decoder's per-thread limits is decoded on the host
            # tier, and such a snapshot is left in stream order (the partition path would merge it):
            # laid out as one run per replica here, as the bench's setup does with its rows
            sort_into_runs(din, 8)
        assert din.n_runs == 8
        out, st = _merge(ctx, din, dense=False)
        assert st.sorted_runs == 1
        assert st.node_rows_in + st.member_rows_in > 70_000_000 and st.key_rows_in > 35_000_000
        assert st.mid_buckets + st.hot_buckets > 0  # buckets beyond a wave: the workgroup and chip-wide tiers
        got = cdb.merged_from_device(ctx, out, batches, stats=st).canonical_dump()
    finally:
        _release(ctx, din)
    if got != want:
        pytest.fail(_first_diff(got, want))
    assert hashlib.sha256(got).digest() == hashlib.sha256(want).digest()
    assert st.type_conflicts == ost.type_conflicts and st.dict_merges == ost.dict_merges


def _invariants(k, n, m, universe):
    for t in (k, n, m):
        u = t[0] ^ SIGN
        assert bool((u[1:] >= u[:-1]).all())
    cref = k[7]
    cnt = cref & 0xFFFFFF
    begin = cref >> 24
    tag = (k[5] >> 56) & 0xFF
    is_counter = tag == 0
    is_lww = (tag == 4) | (tag == 5)
    assert bool((cnt[~(is_counter | is_lww)] == 0).all())
    owners = {}
    for name, sel, child in (("nodes", is_counter, n), ("members", is_lww, m)):
        idx = torch.nonzero(sel & (cnt > 0), as_tuple=True)[0]
        c, b0 = cnt[idx], begin[idx]
        assert int(c.sum()) == child.shape[1], name
        order = torch.argsort(b0)
        idx, b0, c = idx[order], b0[order], c[order]
        assert int(b0[0]) == 0 and bool((b0[1:] == (b0 + c)[:-1]).all()), name
        owner = torch.repeat_interleave(idx, c)
        assert bool((child[0] == k[0][owner]).all()) and bool((child[1] == k[1][owner]).all()), name
        owners[name] = owner
    sums = torch.zeros(k.shape[1], dtype=torch.int64, device="cuda").index_add_(0, owners["nodes"], n[3])
    assert bool((sums[is_counter] == k[6][is_counter]).all())
    data = int((tag <= 5).sum())
    assert 0.9 * universe < data <= universe


@pytest.mark.timeout(900)
def test_full_c4_shard_records_buckets_equals_columns_dense(ctx):
    U = 62_500_000
    L = cdb.lib()
    cfg = configs.c4(cdb, U)
    rec = cdb.DevInput()
    g = cdb.GenConfig()
    ctypes.memmove(ctypes.byref(g), ctypes.byref(cfg), ctypes.sizeof(g))
    g.flags |= cdb.GEN_ROWS_RECORDS
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(g), ctypes.byref(rec)))
    try:
        assert rec.keys.stride == 6 and rec.nodes.stride == 5 and rec.members.stride == 5
        sort_into_runs(rec)  # one run per replica: the bench's input
        out, st = _merge(ctx, rec, dense=False)
        assert st.sorted_runs == 1 and st.key_rows_in > 250_000_000
        got = _compacted(ctx, out)
        out2, st2 = _merge(ctx, rec, dense=False)  # a second merge: bit-identical
        again = _compacted(ctx, out2)
        for a, b in zip(got, again):
            assert torch.equal(a, b)
        assert (st2.key_rows_out, st2.node_rows_out, st2.member_rows_out) == \
            (st.key_rows_out, st.node_rows_out, st.member_rows_out)
        del again
    finally:
        _release(ctx, rec)
    _invariants(*got, U)
    col = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(col)))
    try:
        assert col.keys.stride <= 1
        sort_into_runs(col)
        dout, st3 = _merge(ctx, col, dense=True)
        want = _cols(dout)
        _release(ctx, dout)
    finally:
        _release(ctx, col)
    assert st3.sorted_runs == 1
    for fam, (a, b) in enumerate(zip(got, want)):
        assert a.shape == b.shape, (fam, a.shape, b.shape)
        for c in range(a.shape[0]):
            assert torch.equal(a[c], b[c]), (fam, c)
    assert (st.type_conflicts, st.dict_merges) == (st3.type_conflicts, st3.dict_merges)
