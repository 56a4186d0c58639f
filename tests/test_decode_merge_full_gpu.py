"""The decoder feeding the merge at the bench's sizes (SURVEY §8f.1 -> §8a: pull.rs:64-79 then
:120-128 with the rows in HBM). Snapshots in the generator's order -- the reference's HashMap order,
no key order (db.rs:122-136) -- are decoded straight into HBM as records, each sorted into one run on
the device, and merged on the sorted-run path into the bucket layout:
  * C4's shape at 1M keys x 8 replicas: the result's canonical dump equals the C++ oracle's
    sequential fold of the same snapshots (oracle/cdb_oracle.cpp);
  * the full C4 shard (62.5M-key universe x 8 replicas, ~270M key rows, 15.6 GB of snapshots): the
    merge of the decoded rows equals, row for row, the merge of the same replicas generated in HBM
    (cdb_gen_device, whose rows equal the decoded snapshots' as multisets: tests/test_configs_gpu.py)
    in every field that does not name a source row (the decoder's src are entry indices, the
    generator's model coordinates): hashes, times, tags and fold positions, counter values and
    sums, child ranges."""
import ctypes
from concurrent.futures import ThreadPoolExecutor

import pytest
import torch

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import sort_into_runs, wrap

pytestmark = pytest.mark.gpu

NC = (("keys", 8), ("nodes", 6), ("members", 6))
SRC = 0xFFFFFFFFFFFF  # meta / win: the src bits


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _release(ctx, *sets):
    L = cdb.lib()
    for s in sets:
        for name, _ in NC:
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(s, name)))


def _merge(ctx, din, compact):
    L = cdb.lib()
    out = cdb.DevOutput()
    if compact:
        for name, nc in NC:
            r = cdb.DevRows()
            ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(din, name).n, nc))
            setattr(out, name, r)
    out.compact = 1 if compact else 0
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.merge_opts()), ctypes.byref(out),
                                 ctypes.byref(st), None))
    return out, st


def _dense(ctx, out):
    """A bucket-layout result as dense torch columns (cdb_dev_output_compact into fresh rows)."""
    L = cdb.lib()
    dense = cdb.DevOutput()
    for name, nc in NC:
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(out, name).n, nc))
        setattr(dense, name, r)
    dense.compact = 1
    ctx.check(L.cdb_dev_output_compact(ctx.handle, ctypes.byref(out), ctypes.byref(dense), None))
    cols = [torch.stack([wrap(getattr(dense, name).col[c], getattr(dense, name).n) for c in range(nc)]).clone()
            for name, nc in NC]
    _release(ctx, dense)
    return cols


def test_decoder_c4_1m_reference_order_vs_oracle(ctx):
    cfg = configs.c4(cdb, 1_000_000)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    rc, want, ost = cdb_oracle.fold(snaps)
    assert rc == 0
    batches, din = cdb.decode_snapshots_device(ctx, snaps, records=True)
    try:
        assert din.n_runs == 8 and din.keys.stride == 6
        out, st = _merge(ctx, din, compact=False)
        assert st.sorted_runs == 1 and st.key_rows_in > 4_000_000
        got = cdb.merged_from_device(ctx, out, batches, stats=st).canonical_dump()
        assert got == want
        assert st.type_conflicts == ost.type_conflicts
    finally:
        _release(ctx, din)


def _comparable(cols):
    """Every field that does not name a source row: meta keeps tag and pos; a Bytes key's win (the
    value's (pos, src)) and a side-map win keep pos; a counter's win (its sum) stays whole."""
    k, n, m = [c.clone() for c in cols]
    tag = (k[5] >> 56) & 0xFF
    k[5] &= ~SRC
    by_ref = (tag == 3) | (tag == 6) | (tag == 7)
    k[6] = torch.where(by_ref, k[6] & ~SRC, k[6])
    n[5] &= ~SRC
    m[5] &= ~SRC
    return k, n, m


@pytest.mark.timeout(600)
def test_decoder_full_c4_shard_equals_generator_rows(ctx):
    cfg = configs.c4(cdb, 62_500_000)
    with ThreadPoolExecutor(8) as ex:  # (the generator releases the GIL)
        snaps = list(ex.map(lambda r: cdb.gen_snapshot(cfg, r), range(8)))
    assert sum(len(s) for s in snaps) > 10_000_000_000
    batches, din = cdb.decode_snapshots_device(ctx, snaps, records=True)
    del snaps
    try:
        assert din.n_runs == 8
        out, st = _merge(ctx, din, compact=False)
        assert st.sorted_runs == 1 and st.key_rows_in > 250_000_000
        got = _comparable(_dense(ctx, out))
    finally:
        _release(ctx, din)
    del batches
    L = cdb.lib()
    gen = cdb.DevInput()
    g = cdb.GenConfig()
    ctypes.memmove(ctypes.byref(g), ctypes.byref(cfg), ctypes.sizeof(g))
    g.flags |= cdb.GEN_ROWS_RECORDS
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(g), ctypes.byref(gen)))
    try:
        sort_into_runs(gen, 8)
        out2, st2 = _merge(ctx, gen, compact=True)
        assert st2.sorted_runs == 1
        want = _comparable([torch.stack([wrap(getattr(out2, name).col[c], getattr(out2, name).n)
                                         for c in range(nc)]) for name, nc in NC])
        for fam, (a, b) in enumerate(zip(got, want)):
            assert a.shape == b.shape, (fam, a.shape, b.shape)
            for c in range(a.shape[0]):
                assert torch.equal(a[c], b[c]), (fam, c)
        assert (st.key_rows_in, st.key_rows_out, st.node_rows_out, st.member_rows_out, st.type_conflicts) == \
            (st2.key_rows_in, st2.key_rows_out, st2.node_rows_out, st2.member_rows_out, st2.type_conflicts)
        _release(ctx, out2)
    finally:
        _release(ctx, gen)
