"""The sorted-run merge path -- the path every bench line measures -- against the oracle directly.

Rows are decoded on the host, uploaded (cdb_upload_batches), laid out as hash-ordered runs on the
device (constdb_amd/runs.py: one run per replica, or three key runs per replica -- DATAS, EXPIRES,
DELETES as an encoded snapshot lists them), or decoded on the GPU from snapshots this engine encoded
(cdb_decode_snapshots_device places each as one run),
merged by cdb_merge_device (asserted to take the sorted-run path), and the result's canonical
dump (cdb_merged_from_device) is compared byte for byte with the C++ oracle's sequential fold
(oracle/cdb_oracle.cpp: db.rs:31-119, object.rs:63-83, type_counter.rs:59-91,
crdt/lwwhash.rs:87-128,319-323). Configs: random small states, every forced tier, C1 at full size,
C3 at full size (with DB::gc removing Deletes), C4's shape at 1M keys, C5 at 300K keys; chained
merges (a result merged into again, on the host and in HBM) against the oracle's fold of all
snapshots; and bench.py's full C4 shard on the sorted-run path through size-independent
properties."""
import ctypes

import pytest
import torch

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import sort_into_runs, wrap

pytestmark = pytest.mark.gpu

SIGN = -(1 << 63)


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _arr(batches):
    return (ctypes.c_void_p * max(len(batches), 1))(*[b.handle for b in batches])


def _upload(ctx, batches):
    din = cdb.DevInput()
    ctx.check(cdb.lib().cdb_upload_batches(ctx.handle, _arr(batches), len(batches), ctypes.byref(din)))
    return din


def _out_for(ctx, din):
    L = cdb.lib()
    dout = cdb.DevOutput()
    for name, nc in (("keys", 8), ("nodes", 6), ("members", 6)):
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(din, name).n, nc))
        r.n = 0
        setattr(dout, name, r)
    dout.compact = 1
    return dout


def _release(ctx, *sets):
    L = cdb.lib()
    for s in sets:
        for name in ("keys", "nodes", "members"):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(s, name)))


def _merge_device(ctx, din, dout, **kw):
    opts = cdb.merge_opts(**kw)
    st = cdb.MergeStats()
    ctx.check(cdb.lib().cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(dout),
                                         ctypes.byref(st), None))
    return st


def runs_merge(ctx, snaps, sections=False, expect_runs=True, **kw):
    """Decoded snapshots merged on the sorted-run path; returns the host view of the result."""
    batches = [cdb.decode_snapshot(s) for s in snaps]
    din = _upload(ctx, batches)
    dout = _out_for(ctx, din)
    try:
        sort_into_runs(din, sections=sections)
        st = _merge_device(ctx, din, dout, **kw)
        if expect_runs:
            assert st.sorted_runs == 1
        return cdb.merged_from_device(ctx, dout, batches, stats=st)
    finally:
        _release(ctx, din, dout)


def _diff(got, want):
    gl, wl = got.split(b"\n"), want.split(b"\n")
    i = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b), min(len(gl), len(wl)))
    return (f"first diff at line {i}: gpu {gl[i][:200] if i < len(gl) else None!r} "
            f"oracle {wl[i][:200] if i < len(wl) else None!r} ({len(gl)} vs {len(wl)} lines)")


def check_runs(ctx, snaps, gc=None, gc_members=False, sections=False, **kw):
    flags = (cdb_oracle.FLAG_GC if gc is not None else 0) | (cdb_oracle.FLAG_GC_MEMBERS if gc_members else 0)
    rc, want, ost = cdb_oracle.fold(snaps, flags=flags, gc_watermark=gc or 0)
    assert rc == 0
    m = runs_merge(ctx, snaps, sections=sections, gc_watermark=gc, gc_members=gc_members, **kw)
    got = m.canonical_dump()
    assert got == want, _diff(got, want)
    assert m.stats.type_conflicts == ost.type_conflicts
    assert m.stats.dict_merges == ost.dict_merges
    return m


def _small(seed, universe, replicas, **kw):
    base = dict(seed=seed, universe=universe, n_replicas=replicas, replica_hi=replicas)
    base.update(kw)
    return cdb.gen_config(**base)


@pytest.mark.parametrize("seed", range(8))
def test_runs_random_vs_oracle(ctx, seed):
    """Random replica states with type conflicts, forced time ties, side maps, long member lists;
    one run per replica (even seeds) or three key runs per replica (odd)."""
    cfg = _small(100 + seed, 1500 + 2500 * seed, 1 + seed % 8, conflict_ppm=30000, tie_permille=150,
                 side_permille=250, mean_members=3 + seed, del_permille=300)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(cfg.n_replicas)]
    check_runs(ctx, snaps, sections=bool(seed % 2))


@pytest.mark.parametrize("tier", [1, 2, 3, 4])
def test_runs_forced_tiers_vs_oracle(ctx, tier):
    cfg = _small(140 + tier, 4000, 5, conflict_ppm=20000, side_permille=200, tie_permille=100)
    check_runs(ctx, [cdb.gen_snapshot(cfg, r) for r in range(5)], force_tier=tier)


def test_chip_wide_in_batches_vs_oracle(ctx, monkeypatch):
    """The chip-wide child path run in many batches (the key-table cap lowered from 2^23 to 2000 key
    rows by the CDB_HOT_KEY_CAP test hook), every bucket sent through it (force_tier 2): equal to
    the oracle. At full scale a child-heavy input of more than 2^23 key rows takes this path."""
    monkeypatch.setenv("CDB_HOT_KEY_CAP", "2000")
    cfg = _small(77, 30000, 4, mix_set=30, mix_dict=30, mean_members=12, side_permille=100, conflict_ppm=10000,
                 del_permille=300)
    check_runs(ctx, [cdb.gen_snapshot(cfg, r) for r in range(4)], force_tier=2)


@pytest.mark.parametrize("lds,id_bits,direct", [("1", None, None), ("0", None, None), ("1", "4", None),
                                                ("1", "12", None), ("1", None, "1"), ("1", "4", "1"),
                                                ("0", None, "0")])
def test_chip_wide_lds_and_global_sort_vs_oracle(ctx, monkeypatch, lds, id_bits, direct):
    """Run-order batches of buckets of at most 8192 children take the per-bucket LDS sort and fold
    (hot_sortfold_kernel); CDB_HOT_LDS=0 sends them through the global tag sort instead. Both equal
    the oracle on every bucket forced through the chip-wide path (force_tier 2), with counters,
    sets and dicts, GC of member deletes, and -- with few id-hash bits (CDB_HOT_ID_BITS) -- runs
    holding several exact ids, folded by successor selection. The LDS path's folds read the 32-B
    records the tag pass writes (default) or, with CDB_HOT_DIRECT=1, each child's row in the runs;
    the global path reads the rows (default) or, with CDB_HOT_DIRECT=0, the records."""
    monkeypatch.setenv("CDB_HOT_LDS", lds)
    if id_bits:
        monkeypatch.setenv("CDB_HOT_ID_BITS", id_bits)
    if direct:
        monkeypatch.setenv("CDB_HOT_DIRECT", direct)
    cfg = _small(91, 40000, 5, mix_set=25, mix_dict=25, mean_members=20, side_permille=150, conflict_ppm=10000,
                 tie_permille=100, del_permille=300)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(5)]
    wm = (configs.T0_MS + (1 << 19)) << 22
    m = check_runs(ctx, snaps, force_tier=2, gc=wm, gc_members=True)
    assert m.stats.hot_buckets > 0
    if id_bits == "4":  # (16 member ids per key over 16 id-bit values: runs of several ids)
        assert m.stats.hot_slow_runs > 0


def test_c5_hot_lds_vs_global_sort_identical(ctx, monkeypatch):
    """C5 at 300K keys on the sorted-run path: the LDS path (buckets of at most 8192 children) and
    the global sort give the same dump (the oracle's), and the big buckets stay on the global sort."""
    cfg = configs.c5(cdb, universe=300_000, events=3_000_000)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    a = check_runs(ctx, snaps).canonical_dump()
    monkeypatch.setenv("CDB_HOT_LDS", "0")
    assert runs_merge(ctx, snaps).canonical_dump() == a


def test_runs_gc_vs_oracle(ctx):
    cfg = _small(7, 20000, 4, mix_set=40, mix_dict=40, side_permille=300, del_permille=400)
    wm = (configs.T0_MS + (1 << 19)) << 22
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(4)]
    m = check_runs(ctx, snaps, gc=wm, sections=True)
    assert m.stats.deletes_gced > 0
    check_runs(ctx, snaps, gc=wm, gc_members=True)


def test_runs_c1_full_size_vs_oracle(ctx):
    """C1/C2 (2-node MEET, 1M Bytes + 1M counters per node) on the sorted-run path."""
    cfg = configs.c1(cdb)
    m = check_runs(ctx, [cdb.gen_snapshot(cfg, r) for r in range(2)], sections=True)
    assert 3_900_000 < m.stats.key_rows_in < 4_100_000


@pytest.mark.parametrize("gc", [None, (configs.T0_MS + (1 << 18)) << 22])
def test_runs_c4_1m_keys_vs_oracle(ctx, gc):
    """C4's shape (the bench's generator config) at a 1M-key universe x 8 replicas."""
    cfg = configs.c4(cdb, 1_000_000)
    m = check_runs(ctx, [cdb.gen_snapshot(cfg, r) for r in range(8)], gc=gc, sections=gc is not None)
    assert m.stats.key_rows_in > 4_000_000


def test_runs_c5_300k_vs_oracle(ctx):
    """C5 (Zipf hot keys: keys with 10^4-10^5 children) at 300K keys / 3M events."""
    cfg = configs.c5(cdb, universe=300_000, events=3_000_000)
    m = check_runs(ctx, [cdb.gen_snapshot(cfg, r) for r in range(8)])
    assert m.stats.hot_buckets + m.stats.mid_buckets > 0


def test_runs_c3_full_size_vs_oracle(ctx, c3_snaps):
    """C3 at full size: 4 replica states (10M sadd/srem/hset/hdel each on a synced state with
    Expires and Deletes), merged with DB::gc at the median member time. One type per key on every
    replica (type conflicts far below 1 % of key rows) and GC removes Deletes."""
    batches = [cdb.decode_snapshot(s) for s in c3_snaps]
    wm = configs.median_member_time(cdb, batches)
    del batches
    m = check_runs(ctx, c3_snaps, gc=wm, sections=True)
    st = m.stats
    assert st.member_rows_in > 1_000_000
    assert st.type_conflicts < 0.01 * st.key_rows_in
    assert st.deletes_gced > 0


# ------------------------------------------------------------------ chained merges (pull.rs:120-128)
def test_merge_into_chain_vs_oracle(ctx):
    """Two MEETs in a row: the local DB merges 3 peers, then 3 more into the result (cdb_merge_into,
    fold position 0 = the previous result) -- equal to the oracle's sequential fold of all 6."""
    cfg = _small(21, 30000, 6, conflict_ppm=20000, tie_permille=100, side_permille=150)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(6)]
    db = cdb.DB(ctx)
    first = db.merge_snapshots(snaps[:3])
    second = db.merge_into(first, [cdb.decode_snapshot(s) for s in snaps[3:]])
    rc, want, _ = cdb_oracle.fold(snaps)
    assert rc == 0
    got = second.canonical_dump()
    assert got == want, _diff(got, want)
    # a third step on top of the second, and an empty merge leaves the state as it is
    third = db.merge_into(second, [])
    assert third.canonical_dump() == want
    enc, _ = second.encode_snapshot(replicas=None)
    assert db.merge_snapshots([enc]).canonical_dump() == want


def _cat_runs(parts):
    """Device input of several (din, n_runs) parts, each already in runs: the columns
    concatenated family by family, the runs of each part after the previous part's."""
    L = cdb.lib()
    din = cdb.DevInput()
    tensors = []
    nr = sum(p.n_runs for p in parts)
    din.n_runs = nr
    din.n_pos = sum(p.n_pos for p in parts)
    for f, (name, nc) in enumerate((("keys", 7), ("nodes", 6), ("members", 6))):
        total = sum(getattr(p, name).n for p in parts)
        t = torch.empty((nc, max(total, 1)), dtype=torch.int64, device="cuda")
        at = 0
        r0 = 0
        for p in parts:
            rows = getattr(p, name)
            for c in range(nc):
                if rows.n:
                    t[c, at:at + rows.n].copy_(wrap(rows.col[c], rows.n))
            for r in range(p.n_runs):
                din.run_start[f][r0 + r] = at + p.run_start[f][r]
            at += rows.n
            r0 += p.n_runs
        din.run_start[f][nr] = at
        rr = cdb.DevRows()
        for c in range(nc):
            rr.col[c] = t[c].data_ptr()
        rr.n = total
        setattr(din, name, rr)
        tensors.append(t)
    torch.cuda.synchronize()
    return din, tensors


def test_device_state_chain_vs_oracle(ctx):
    """The same chain kept in HBM: merge 1's compacted output becomes fold position 0 of merge 2
    through cdb_dev_state_rows (one run), the next replicas' rows follow as runs of their own;
    merge 2 runs on the sorted-run path and its host view (state = merge 1's) equals the oracle."""
    L = cdb.lib()
    cfg = _small(23, 40000, 5, conflict_ppm=20000, tie_permille=100, side_permille=150)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(5)]
    b1 = [cdb.decode_snapshot(s) for s in snaps[:2]]
    b2 = [cdb.decode_snapshot(s) for s in snaps[2:]]
    din1 = _upload(ctx, b1)
    dout1 = _out_for(ctx, din1)
    sort_into_runs(din1)
    st1 = _merge_device(ctx, din1, dout1)
    state_host = cdb.merged_from_device(ctx, dout1, b1, stats=st1)
    # state rows (position 0, one run)
    sdin = cdb.DevInput()
    for name, nc in (("keys", 7), ("nodes", 6), ("members", 6)):
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(dout1, name).n, nc))
        setattr(sdin, name, r)
    ctx.check(L.cdb_dev_state_rows(ctx.handle, ctypes.byref(dout1), ctypes.byref(sdin.keys), ctypes.byref(sdin.nodes),
                                   ctypes.byref(sdin.members), None))
    sdin.n_pos, sdin.n_runs = 1, 1
    for f, name in enumerate(("keys", "nodes", "members")):
        sdin.run_start[f][0], sdin.run_start[f][1] = 0, getattr(sdin, name).n
    # the new replicas at positions 1.. (stamped by the upload as 0.., shifted here)
    din2 = _upload(ctx, b2)
    for name, nc in (("keys", 7), ("nodes", 6), ("members", 6)):
        rows = getattr(din2, name)
        if rows.n:
            meta = wrap(rows.col[nc - 1], rows.n)
            meta.add_(1 << 48)
    din2.n_pos = len(b2)
    sort_into_runs(din2, n_runs=len(b2) + 1)  # runs by pos: run 0 (pos 0) is empty
    both, keep = _cat_runs([sdin, din2])
    both.n_pos = 1 + len(b2)
    dout2 = _out_for(ctx, both)
    try:
        st2 = _merge_device(ctx, both, dout2)
        assert st2.sorted_runs == 1
        m = cdb.merged_from_device(ctx, dout2, b2, state=state_host, stats=st2)
        rc, want, _ = cdb_oracle.fold(snaps)
        assert rc == 0
        got = m.canonical_dump()
        assert got == want, _diff(got, want)
    finally:
        _release(ctx, din1, dout1, sdin, din2, dout2)
        del keep


# ------------------------------------------------------------------ a producer of sorted runs
def _hash_ordered_snapshots(ctx, snaps):
    """Each replica state as the engine would write it back (replica/pull.rs:120-128 then
    server.rs:183-215): merged once, encoded -- DATAS, EXPIRES and DELETES each in key-hash order."""
    db = cdb.DB(ctx)
    return [db.merge_snapshots([s]).encode_snapshot(replicas=None)[0] for s in snaps]


@pytest.mark.parametrize("seed,gc", [(0, False), (1, True), (2, False)])
def test_encode_decode_device_runs_vs_oracle(ctx, seed, gc):
    """encode -> GPU decode into HBM -> cdb_merge_device: the decoder places each snapshot's key rows
    as one key-hash-ordered run (its three sections merged), so the merge takes the sorted-run path
    with no setup sort; the result equals the oracle's fold of the same snapshots. Snapshots in
    generator order decoded with CDB_DECODE_STREAM_ORDER get no runs."""
    cfg = _small(300 + seed, 20000 + 10000 * seed, 3 + 2 * seed, conflict_ppm=20000, tie_permille=100,
                 side_permille=300, mix_set=20, mix_dict=20, del_permille=300)
    raw = [cdb.gen_snapshot(cfg, r) for r in range(cfg.n_replicas)]
    batches, din = cdb.decode_snapshots_device(ctx, raw, stream_order=True)
    assert din.n_runs == 0
    _release(ctx, din)
    encs = _hash_ordered_snapshots(ctx, raw)
    wm = (configs.T0_MS + (1 << 30)) << 22 if gc else None  # after every time: DB::gc takes every Delete
    rc, want, ost = cdb_oracle.fold(encs, flags=cdb_oracle.FLAG_GC if gc else 0, gc_watermark=wm or 0)
    assert rc == 0
    batches, din = cdb.decode_snapshots_device(ctx, encs)
    dout = _out_for(ctx, din)
    try:
        assert din.n_runs == len(encs)
        assert [din.run_start[0][r] for r in (0, len(encs))] == [0, din.keys.n]
        st = _merge_device(ctx, din, dout, gc_watermark=wm)
        assert st.sorted_runs == 1
        m = cdb.merged_from_device(ctx, dout, batches, stats=st)
        got = m.canonical_dump()
        assert got == want, _diff(got, want)
        assert st.type_conflicts == ost.type_conflicts
        if gc:
            assert st.deletes_gced > 0
    finally:
        _release(ctx, din, dout)


# ------------------------------------------------------------------ full size, sorted runs
def test_full_c4_shard_sorted_runs_invariants(ctx):
    """bench.py's workload on the path it measures (62.5M-key universe x 8 replicas, ~270M key
    rows in HBM, the decoder's run layout): a second merge is bit-identical; the output is in
    key-hash order (a sorted run again); child ranges tile the child outputs and every child names
    its key; a counter's win is the wrapping sum of its nodes (cal_sum, type_counter.rs:89-91);
    output counts are bounded by the distinct keys of the universe."""
    L = cdb.lib()
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(configs.c4(cdb, 62_500_000)), ctypes.byref(din)))
    dout = _out_for(ctx, din)
    try:
        sort_into_runs(din, sections=True)
        st = _merge_device(ctx, din, dout)
        assert st.sorted_runs == 1 and st.key_rows_in > 250_000_000
        k = torch.stack([wrap(dout.keys.col[c], dout.keys.n) for c in range(8)]).clone()
        n = torch.stack([wrap(dout.nodes.col[c], dout.nodes.n) for c in range(6)]).clone()
        m = torch.stack([wrap(dout.members.col[c], dout.members.n) for c in range(6)]).clone()
        st2 = _merge_device(ctx, din, dout)
        for t, rows, nc in ((k, dout.keys, 8), (n, dout.nodes, 6), (m, dout.members, 6)):
            assert rows.n == t.shape[1]
            for c in range(nc):
                assert torch.equal(t[c], wrap(rows.col[c], rows.n))
        assert st2.key_rows_out == st.key_rows_out
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
        assert 0.9 * 62_500_000 < data <= 62_500_000
    finally:
        _release(ctx, din, dout)
