"""The chip-wide child path's list merge (hot.hip.h: hot_lists_kernel / hot_merge_kernel).

Every merge tier writes a key's children in child_order (common.h), so replica states kept as this
engine's merge results (constdb_amd.runs.state_runs: each replica merged alone, read back with
cdb_dev_state_rows, moved to its fold position with cdb_dev_input_append) arrive with every
hot bucket's child lists sorted, and the chip-wide path merges them instead of radix-sorting
(stats.hot_merged_children). Checked here:
  * the same state-run input merged with the list merge and with the radix sort (CDB_HOT_MERGE=0)
    gives bit-identical results;
  * the state-run input and the generator's rows (plain runs, lists unsorted: the radix sort runs)
    give the same merged state -- every column equal except the meta words' src fields (entry
    indices: a state row's src is its index in the state) -- and the plain-run path is the one
    tests/test_runs_oracle_gpu.py and test_fullsize_gpu.py check against the oracle
    (type_counter.rs:59-87, lwwhash.rs:87-107, 319-323);
  * forced through the chip-wide path (force_tier 2, the LDS path off) with counters, sets, dicts,
    member GC and few id bits (runs of several ids: the successor-selection fold)."""
import ctypes

import pytest
import torch

import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import sort_into_runs, state_runs, wrap

pytestmark = pytest.mark.gpu

NC = (("keys", 8), ("nodes", 6), ("members", 6))
NAMES = ("keys", "nodes", "members")


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _gen(ctx, cfg):
    L = cdb.lib()
    din = cdb.DevInput()
    g = cdb.GenConfig()
    ctypes.memmove(ctypes.byref(g), ctypes.byref(cfg), ctypes.sizeof(g))
    g.flags |= cdb.GEN_ROWS_RECORDS
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(g), ctypes.byref(din)))
    return din


def _release(ctx, *sets):
    for s in sets:
        for name in NAMES:
            cdb.lib().cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(s, name)))


def _merge_cols(ctx, din, opts):
    """cdb_merge_device (bucket layout), compacted into dense columns: [keys 8, nodes 6, members 6]."""
    L = cdb.lib()
    out = cdb.DevOutput()
    out.compact = 0
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(out),
                                 ctypes.byref(st), None))
    dense = cdb.DevOutput()
    for name, nc in NC:
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), max(getattr(out, name).n, 1), nc))
        setattr(dense, name, r)
    dense.compact = 1
    ctx.check(L.cdb_dev_output_compact(ctx.handle, ctypes.byref(out), ctypes.byref(dense), None))
    cols = [torch.stack([wrap(getattr(dense, name).col[c], getattr(dense, name).n) for c in range(nc)]).clone()
            for name, nc in NC]
    _release(ctx, dense)
    return cols, st


def _state(cols):
    """The merged state without the meta words' src fields (key meta col 5; win col 6 -- a winner's
    (pos, src) -- except a counter's, which is its sum; child meta col 5): tags and positions stay."""
    k, n, m = (c.clone() for c in cols)
    hi = ~((1 << 48) - 1)
    k[5] &= hi
    tag = (k[5] >> 56) & 0xFF
    k[6] = torch.where(tag == 0, k[6], k[6] & hi)  # (TAG_COUNTER = 0)
    n[5] &= hi
    m[5] &= hi
    return k, n, m


def _opts(gc_members=None, force_tier=0):
    """Member GC only: DB::gc of Deletes (db.rs:82-119) pops in entry order and stops at the first
    live one, so it depends on the src numbering, which a state's rows renumber."""
    o = cdb.merge_opts(force_tier=force_tier)
    if gc_members is not None:
        o.flags |= cdb.MERGE_GC_MEMBERS
        o.gc_watermark = gc_members
    return o


def _check(ctx, monkeypatch, cfg, opts, expect_merge=True):
    plain = _gen(ctx, cfg)
    state = _gen(ctx, cfg)
    try:
        sort_into_runs(plain)
        want, stp = _merge_cols(ctx, plain, opts)
        assert stp.sorted_runs == 1 and stp.hot_merged_children == 0  # generator order: lists unsorted
        state_runs(cdb, ctx, state)
        assert state.n_runs == cfg.replica_hi - cfg.replica_lo
        got, sts = _merge_cols(ctx, state, opts)
        assert sts.sorted_runs == 1
        if expect_merge:
            assert sts.hot_merged_children > 0
        monkeypatch.setenv("CDB_HOT_MERGE", "0")
        again, str_ = _merge_cols(ctx, state, opts)
        monkeypatch.delenv("CDB_HOT_MERGE")
        assert str_.hot_merged_children == 0
    finally:
        _release(ctx, plain, state)
    for fam, (a, b) in enumerate(zip(got, again)):  # list merge == radix sort, bit for bit
        assert a.shape == b.shape and torch.equal(a, b), fam
    for fam, (a, b) in enumerate(zip(_state(got), _state(want))):  # == the generator rows' merge
        assert a.shape == b.shape, (fam, a.shape, b.shape)
        for c in range(a.shape[0]):
            assert torch.equal(a[c], b[c]), (fam, c)
    assert (sts.type_conflicts, sts.dict_merges, sts.members_gced) == \
        (stp.type_conflicts, stp.dict_merges, stp.members_gced)
    return sts


def test_c5_300k_state_runs_merged(ctx, monkeypatch):
    """C5's shape (Zipf hot keys, 10^4-10^5 children) at 300K keys / 3M events x 8 replicas."""
    cfg = configs.c5(cdb, universe=300_000, events=3_000_000)
    st = _check(ctx, monkeypatch, cfg, _opts())
    assert st.hot_buckets + st.mid_buckets > 0


@pytest.mark.parametrize("id_bits", [None, "4"])
def test_forced_chip_wide_state_runs_merged(ctx, monkeypatch, id_bits):
    """Every bucket through the chip-wide path's global sort (force_tier 2, CDB_HOT_LDS=0): counters,
    sets and dicts, member deletes GC'd, type conflicts and ties; with 4 id bits many W-runs hold
    several ids (successor-selection fold)."""
    monkeypatch.setenv("CDB_HOT_LDS", "0")
    if id_bits:
        monkeypatch.setenv("CDB_HOT_ID_BITS", id_bits)
    cfg = cdb.gen_config(seed=91, universe=40000, n_replicas=5, key_permille=600, mix_bytes=20, mix_counter=30,
                         mix_set=25, mix_dict=25, mean_members=20, side_permille=150, conflict_ppm=10000,
                         tie_permille=100, del_permille=300, replica_lo=0, replica_hi=5)
    wm = (configs.T0_MS + (1 << 19)) << 22
    st = _check(ctx, monkeypatch, cfg, _opts(gc_members=wm, force_tier=2))
    assert st.hot_buckets > 0 and st.members_gced > 0
    if id_bits:
        assert st.hot_slow_runs > 0


@pytest.mark.timeout(900)
def test_c5_bench_size_state_runs_merged(ctx, monkeypatch):
    """The bench's C5 input at its size (10M keys, 80M child events, 8 replicas): the state runs the
    bench times, merged with the list merge, equal the radix sort's result and the generator rows'."""
    st = _check(ctx, monkeypatch, configs.c5(cdb), _opts())
    assert st.hot_merged_children > 40_000_000


def test_one_list_out_of_order_falls_back(ctx, monkeypatch):
    """State runs with ONE pair of neighbouring children of the hottest key swapped in run 0: the
    sampled pairs almost surely miss it, round 0 of the merge finds it, and the batch is re-tagged
    and radix-sorted -- the result equals CDB_HOT_MERGE=0's on the same rows, and nothing counts
    as merged."""
    cfg = configs.c5(cdb, universe=300_000, events=3_000_000)
    state = _gen(ctx, cfg)
    try:
        state_runs(cdb, ctx, state)
        rows = state.members
        n0 = state.run_start[2][1]  # run 0's member rows
        kh = wrap(rows.col[0], rows.n)[:n0]
        rec = wrap(rows.col[1], rows.n * rows.stride).view(rows.n, rows.stride)[:n0]
        _, inv, counts = torch.unique_consecutive(kh, return_inverse=True, return_counts=True)
        hot = int(torch.argmax(counts))
        first = int(torch.nonzero(inv == hot)[0])
        assert int(counts[hot]) > 1000 and int(rec[first, 1]) != int(rec[first + 1, 1])
        a, b = rec[first].clone(), rec[first + 1].clone()
        rec[first].copy_(b)
        rec[first + 1].copy_(a)
        torch.cuda.synchronize()
        got, st = _merge_cols(ctx, state, _opts())
        assert st.sorted_runs == 1 and st.hot_merged_children == 0
        monkeypatch.setenv("CDB_HOT_MERGE", "0")
        want, _ = _merge_cols(ctx, state, _opts())
    finally:
        _release(ctx, state)
    for fam, (x, y) in enumerate(zip(got, want)):
        assert x.shape == y.shape and torch.equal(x, y), fam


def test_orphans_in_sorted_lists_fall_back_counted_once(ctx, monkeypatch):
    """State runs where three children of the hottest key in run 0 name a key that does not exist
    (their pkf changed, pkh kept, so the runs stay in hash order): an orphan takes the bucket's marker
    W, which breaks its list's order, so round 0 of the list merge finds it and the batch is re-tagged
    and radix-sorted. The orphans are counted once (the list merge's tag pass counted them already),
    and the result equals CDB_HOT_MERGE=0's bit for bit."""
    cfg = configs.c5(cdb, universe=300_000, events=3_000_000)
    state = _gen(ctx, cfg)
    try:
        state_runs(cdb, ctx, state)
        rows = state.members
        n0 = state.run_start[2][1]
        kh = wrap(rows.col[0], rows.n)[:n0]
        rec = wrap(rows.col[1], rows.n * rows.stride).view(rows.n, rows.stride)[:n0]
        _, inv, counts = torch.unique_consecutive(kh, return_inverse=True, return_counts=True)
        hot = int(torch.argmax(counts))
        first = int(torch.nonzero(inv == hot)[0])
        assert int(counts[hot]) > 1000
        for k in (10, 200, 700):  # (records: pkf is word 0)
            rec[first + k, 0] ^= 0x5A5A5A5A
        torch.cuda.synchronize()
        got, st = _merge_cols(ctx, state, _opts())
        assert st.sorted_runs == 1 and st.hot_merged_children == 0
        monkeypatch.setenv("CDB_HOT_MERGE", "0")
        want, st0 = _merge_cols(ctx, state, _opts())
    finally:
        _release(ctx, state)
    assert st.orphan_children == st0.orphan_children == 3
    for fam, (x, y) in enumerate(zip(got, want)):
        assert x.shape == y.shape and torch.equal(x, y), fam
