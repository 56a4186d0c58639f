"""GPU parity: the HIP merge engine (through the C-ABI) vs the oracle, on the same snapshot
bytes. Bit-exact canonical dumps are required (integer/ordering work, no tolerance)."""
import pytest
import torch  # noqa: F401  -- before libcdbmerge loads: one HIP runtime per process (constdb_amd.lib)

import cdb_oracle
import constdb_amd as cdb
import constdb_oracle as o
from snapgen import gen_replicas

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def db():
    from constdb_amd import build
    build.build()
    return cdb.DB(cdb.Context(0))


def _oracle(snaps, gc=None, members=False):
    flags = 0
    if gc is not None:
        flags |= cdb_oracle.FLAG_GC | (cdb_oracle.FLAG_GC_MEMBERS if members else 0)
    rc, dump, st = cdb_oracle.fold(snaps, flags=flags, gc_watermark=gc or 0)
    assert rc == 0
    return dump, st


def _check(db, snaps, gc=None, members=False, tier=0):
    want, ost = _oracle(snaps, gc, members)
    m = db.merge_snapshots(snaps, gc_watermark=gc, gc_members=members, force_tier=tier)
    got = m.canonical_dump()
    if got != want:
        gl, wl = got.decode().splitlines(), want.decode().splitlines()
        for i, (a, b) in enumerate(zip(gl, wl)):
            if a != b:
                raise AssertionError(f"first diff at line {i}:\n gpu   : {a}\n oracle: {b}\n"
                                     f"(gpu {len(gl)} lines, oracle {len(wl)} lines)")
        raise AssertionError(f"length differs: gpu {len(gl)} lines, oracle {len(wl)} lines")
    assert m.stats.type_conflicts == ost.type_conflicts
    assert m.stats.dict_merges == ost.dict_merges
    return m


# ------------------------------------------------------------------ KATs through the GPU
def _snap(objs=None, deletes=None, expires=None):
    d = o.DB()
    d.data.update(objs or {})
    d.deletes.update(deletes or {})
    d.expires.update(expires or {})
    return o.dump_all(d, o.NodeHeader())


def _counter(nodes, ct=1):
    c = o.Counter()
    c.data.update(nodes)
    c.cal_sum()
    return o.Object(ct, 0, 0, o.OBJECT_ENC_COUNTER, c)


def _set(adds, dels=None):
    s = o.Set()
    for m, t in adds.items():
        s.set(m, None, t)
    for m, t in (dels or {}).items():
        s.rem(m, t)
    return o.Object(1, 0, 0, o.OBJECT_ENC_SET, s)


def test_kat_bytes_ties_and_maxima(db):
    _check(db, [_snap({b"k": o.Object(10, 3, 1, o.OBJECT_ENC_BYTES, b"A")}),
                _snap({b"k": o.Object(10, 9, 0, o.OBJECT_ENC_BYTES, b"B")}),
                _snap({b"k": o.Object(9, 50, 70, o.OBJECT_ENC_BYTES, b"C")})])


def test_kat_counter_order_dependence(db):
    for order in ([(5, 10), (7, 11), (6, 12)], [(5, 10), (6, 12), (7, 11)]):
        _check(db, [_snap({b"c": _counter({1: vt})}) for vt in order])


def test_kat_counter_unmerged_keeps_load_total(db):
    _check(db, [_snap({b"c": _counter({1: (5, 10), 2: (6, 1)})})])


def test_kat_type_conflict(db):
    m = _check(db, [_snap({b"k": _counter({1: (1, 1)})}),
                    _snap({b"k": o.Object(99, 0, 0, o.OBJECT_ENC_BYTES, b"X")}),
                    _snap({b"k": _counter({1: (4, 2)})})])
    assert m.stats.type_conflicts == 1


def test_kat_set_ties_and_remote_dels(db):
    _check(db, [_snap({b"s": _set({b"a": 5, b"b": 7}, {b"d": 10})}),
                _snap({b"s": _set({b"d": 10, b"e": 1}, {b"a": 9})}),
                _snap({b"s": _set({b"b": 6})})])


def test_kat_side_maps_and_gc(db):
    snaps = [_snap(deletes={b"a": 5, b"b": 50, b"c": 6}, expires={b"x": 9}),
             _snap(deletes={b"a": 20}, expires={b"x": 3})]
    _check(db, snaps)
    for wm in (0, 5, 6, 20, 49, 50, 1000):
        _check(db, snaps, gc=wm)


def test_strict_dict_panic(db):
    d1, d2 = o.Dict(), o.Dict()
    d1.set(b"f", b"x", 5)
    d2.set(b"f", b"z", 6)
    snaps = [_snap({b"h": o.Object(1, 0, 0, o.OBJECT_ENC_DICT, d1)}),
             _snap({b"h": o.Object(1, 0, 0, o.OBJECT_ENC_DICT, d2)})]
    _check(db, snaps)
    with pytest.raises(cdb.DictMergeUnimplemented):
        db.merge_snapshots(snaps, strict_dict_panic=True)


def test_empty_inputs(db):
    _check(db, [_snap()])
    _check(db, [_snap(), _snap()])
    assert db.merge_snapshots([]).canonical_dump() == b""


# ------------------------------------------------------------------ randomized parity
@pytest.mark.parametrize("seed", range(60))
def test_random_small(db, seed):
    snaps = gen_replicas(seed, n_replicas=1 + seed % 6, n_keys=30 + seed, big_times=seed % 3 == 0,
                         p_conflict=0.1, p_side=0.2)
    _check(db, snaps)


@pytest.mark.parametrize("tier", [1, 2, 3, 4])
@pytest.mark.parametrize("seed", range(12))
def test_random_forced_tier(db, seed, tier):
    """The LDS workgroup tier (1), the chip-wide child path of over-capacity buckets (2), the
    wide wave kernel (3) and the one-workgroup global-scratch kernel (4) on every bucket."""
    snaps = gen_replicas(900 + seed, n_replicas=1 + seed % 5, n_keys=40, p_conflict=0.1, p_side=0.3)
    _check(db, snaps, gc=(seed % 7) if seed % 2 else None, members=bool(seed % 4 == 1), tier=tier)


def test_mid_tier_natural(db):
    """Buckets of a few hundred rows (above one wave, within the LDS pool)."""
    objs1, objs2 = {}, {}
    for k in range(6):
        s1, s2 = o.Set(), o.Set()
        for j in range(90):
            s1.set(b"m%d" % j, None, (j * 7 + k) % 23)
            if j % 2:
                s2.set(b"m%d" % j, None, (j * 5 + k) % 19)
        objs1[b"s%d" % k] = o.Object(1, 0, 0, o.OBJECT_ENC_SET, s1)
        objs2[b"s%d" % k] = o.Object(2, 0, 0, o.OBJECT_ENC_SET, s2)
    _check(db, [_snap(objs1), _snap(objs2)])


@pytest.mark.parametrize("seed", range(20))
def test_random_gc(db, seed):
    snaps = gen_replicas(500 + seed, n_replicas=3, p_side=0.5)
    _check(db, snaps, gc=seed % 9, members=bool(seed % 2))


def test_many_replicas(db):
    _check(db, gen_replicas(77, n_replicas=63, n_keys=50, p_key=0.3))


@pytest.mark.parametrize("universe,replicas,seed", [(2000, 2, 1), (20000, 4, 2), (60000, 8, 3)])
def test_generator_medium(db, universe, replicas, seed):
    """C1/C2-shaped inputs (generator), thousands of buckets, two partition levels."""
    cfg = cdb.gen_config(seed=seed, universe=universe, n_replicas=replicas, replica_hi=replicas)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(replicas)]
    _check(db, snaps)


def test_wave_tiers_natural(db):
    """Bucket sizes vary: some buckets exceed 64 key rows (wide wave kernel) or 64 child rows
    (two child rows per lane); all stay exact."""
    cfg = cdb.gen_config(seed=21, universe=120000, n_replicas=8, replica_hi=8, mean_members=6)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    m = _check(db, snaps)
    assert m.stats.wide_buckets > 0
    assert m.stats.mid_buckets + m.stats.hot_buckets < m.stats.wide_buckets
    m3 = _check(db, snaps, tier=3)
    assert m3.stats.wide_buckets > m.stats.wide_buckets


def _wide_children_snaps():
    cfg = cdb.gen_config(seed=33, universe=30000, n_replicas=8, replica_hi=8, mix_bytes=10, mix_counter=10,
                         mix_set=40, mix_dict=40, mean_members=12, member_universe=24, del_permille=300)
    return [cdb.gen_snapshot(cfg, r) for r in range(8)]


@pytest.mark.parametrize("tier", [0, 3])
def test_wide_children(db, tier, monkeypatch):
    """Set/dict keys with up to 8 x 24 member rows: buckets of 129..256 child rows take the
    wide kernel's four-rows-per-lane path. (More than 8 children per key: the default plan
    makes large buckets for the chip-wide child path, so wave-sized ones are asked for here.)"""
    monkeypatch.setenv("CDB_PLAN_TARGET", "40")
    monkeypatch.setenv("CDB_PLAN_CTARGET", "80")
    m = _check(db, _wide_children_snaps(), tier=tier)
    assert m.stats.wide_buckets > 0


def test_child_heavy_default_plan(db):
    """The same input under the default plan for child-heavy inputs (make_plan, engine.hip):
    a few large buckets, merged by the over-capacity tiers."""
    m = _check(db, _wide_children_snaps())
    assert m.stats.mid_buckets + m.stats.hot_buckets > 0


def test_generator_set_heavy_gc(db):
    """C3-shaped: set/dict heavy with tombstones, GC at the median time."""
    cfg = cdb.gen_config(seed=3, universe=5000, n_replicas=4, replica_hi=4, mix_bytes=0, mix_counter=0,
                         mix_set=50, mix_dict=50, mean_members=12, member_universe=40, del_permille=400,
                         side_permille=300)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(4)]
    wm = (1700000000000 + (1 << 19)) << 22
    _check(db, snaps)
    _check(db, snaps, gc=wm, members=True)


def test_hot_bucket_path(db):
    """A key whose members exceed the LDS capacity goes through the global-scratch path."""
    big1, big2 = o.Set(), o.Set()
    for j in range(3000):
        big1.set(b"m%d" % j, None, j % 17)
        if j % 3 == 0:
            big2.set(b"m%d" % j, None, j % 13)
        if j % 7 == 0:
            big2.rem(b"x%d" % j, 5)
    c1, c2 = o.Counter(), o.Counter()
    for n in range(1500):
        c1.data[n] = (n, n % 5)
        c2.data[n] = (n * 2, n % 4)
    objs1 = {b"big": o.Object(1, 0, 0, o.OBJECT_ENC_SET, big1), b"cnt": o.Object(1, 0, 0, o.OBJECT_ENC_COUNTER, c1)}
    objs2 = {b"big": o.Object(2, 0, 0, o.OBJECT_ENC_SET, big2), b"cnt": o.Object(2, 0, 0, o.OBJECT_ENC_COUNTER, c2)}
    m = _check(db, [_snap(objs1), _snap(objs2)])
    assert m.stats.hot_buckets >= 1
    _check(db, [_snap(objs1), _snap(objs2)], tier=4)  # the one-workgroup global-scratch kernel


def test_deterministic(db):
    snaps = gen_replicas(9, n_replicas=4)
    a = db.merge_snapshots(snaps).canonical_dump()
    b = db.merge_snapshots(snaps).canonical_dump()
    assert a == b


@pytest.mark.parametrize("shift,universe", [(1, 20000), (3, 20000), (3, 300000)])
def test_key_shift_parity(db, shift, universe):
    """Multi-GPU ranks bucket on the hash bits below the owner bits; any shift is exact (the
    300K-key case takes the row-level + per-segment plan)."""
    cfg = cdb.gen_config(seed=5, universe=universe, n_replicas=4, replica_hi=4)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(4)]
    want, _ = _oracle(snaps)
    batches = [cdb.decode_snapshot(s) for s in snaps]
    import ctypes
    n = len(batches)
    arr = (ctypes.c_void_p * n)(*[b.handle for b in batches])
    opts = cdb.MergeOpts()
    opts.key_shift = shift
    st = cdb.MergeStats()
    h = ctypes.c_void_p()
    db.ctx.check(cdb.lib().cdb_merge(db.ctx.handle, arr, n, ctypes.byref(opts), ctypes.byref(h), ctypes.byref(st)))
    assert cdb.Merged(db.ctx, h, st, batches).canonical_dump() == want


@pytest.mark.parametrize("ncols,bits", [(7, 1), (6, 3), (8, 0)])
def test_partition_owner(db, ncols, bits):
    import ctypes
    import torch
    n = 50_000 + bits
    g = torch.Generator().manual_seed(ncols * 10 + bits)
    src = torch.randint(-2**62, 2**62, (ncols, n), dtype=torch.int64, generator=g).cuda()
    dst = torch.empty_like(src)
    rin, rout = cdb.DevRows(), cdb.DevRows()
    for c in range(ncols):
        rin.col[c] = src[c].data_ptr()
        rout.col[c] = dst[c].data_ptr()
    rin.n = n
    counts = (ctypes.c_uint64 * (1 << bits))()
    db.ctx.check(cdb.lib().cdb_partition_owner(db.ctx.handle, ctypes.byref(rin), ncols, bits, ctypes.byref(rout),
                                               counts, None))
    torch.cuda.synchronize()
    s, d = src.cpu(), dst.cpu()
    own = (s[0].view(torch.int64) >> (64 - bits)) & ((1 << bits) - 1) if bits else torch.zeros(n, dtype=torch.int64)
    assert [counts[i] for i in range(1 << bits)] == torch.bincount(own, minlength=1 << bits).tolist()
    downer = (d[0] >> (64 - bits)) & ((1 << bits) - 1) if bits else torch.zeros(n, dtype=torch.int64)
    assert bool((downer[1:] >= downer[:-1]).all())              # grouped by owner
    key = lambda t: sorted(map(tuple, t.T.tolist()))             # same multiset of rows
    assert key(s) == key(d)


# ------------------------------------------------------------------ BASELINE-scale checks
def _c4(universe, replicas=8, seed=4):
    """bench.py's C4 generator config at a given key universe."""
    return cdb.gen_config(seed=seed, universe=universe, n_replicas=replicas, key_permille=500, mix_bytes=60,
                          mix_counter=30, mix_set=5, mix_dict=5, conflict_ppm=1000, tie_permille=20, max_nodes=8,
                          mean_members=4, member_universe=16, del_permille=200, side_permille=20, value_min=8,
                          value_max=32, replica_hi=replicas)


@pytest.mark.parametrize("gc", [None, 1])
def test_c4_shape_1m_keys_bit_exact(db, gc):
    """C4's shape at a 1M-key universe x 8 replicas (~4.3M entries): the large-plan path (row
    level + per-segment final level, ~100K buckets) against the C++ oracle, bit for bit."""
    cfg = _c4(1_000_000)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(8)]
    wm = None if gc is None else (1700000000000 + (1 << 18)) << 22
    _check(db, snaps, gc=wm)


def _dev_merge(ctx, din, torch):
    """Merges device rows into torch-owned output columns; returns (outputs, stats)."""
    L = cdb.lib()
    dout = cdb.DevOutput()
    outs = []
    for fam, (rows, ncol) in enumerate(((din.keys, 8), (din.nodes, 6), (din.members, 6))):
        t = torch.empty((ncol, max(rows.n, 1)), dtype=torch.int64, device="cuda")
        r = cdb.DevRows()
        for c in range(ncol):
            r.col[c] = t[c].data_ptr()
        r.n = 0
        setattr(dout, ("keys", "nodes", "members")[fam], r)
        outs.append(t)
    dout.compact = 1
    st = cdb.MergeStats()
    import ctypes
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.MergeOpts()), ctypes.byref(dout),
                                 ctypes.byref(st), None))
    torch.cuda.synchronize()
    return [outs[0][:, :dout.keys.n], outs[1][:, :dout.nodes.n], outs[2][:, :dout.members.n]], st


def test_full_c4_shard_invariants(db):
    """bench.py's full workload (62.5M-key universe x 8 replicas, ~270M key rows, generated in
    HBM): size-independent properties of the result, checked on the GPU with torch.
      * determinism: a second merge of the same rows is bit-identical;
      * every key's child range lies inside the child outputs, ranges tile them exactly, and
        every child row names its key (pkh, pkf == kh, kf);
      * a merged counter's `win` is the wrapping sum of its nodes' values (cal_sum).
    The same generator at a 1M-key universe is checked bit-exact against the oracle above."""
    import ctypes
    ctx = db.ctx
    L = cdb.lib()
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(_c4(62_500_000)), ctypes.byref(din)))
    try:
        (k, n, m), st = _dev_merge(ctx, din, torch)
        assert st.key_rows_in > 250_000_000 and st.key_rows_out > 0
        (k2, n2, m2), _ = _dev_merge(ctx, din, torch)
        for a, b in ((k, k2), (n, n2), (m, m2)):
            assert a.shape == b.shape and torch.equal(a, b)
        del k2, n2, m2
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
            assert int(b0[0]) == 0 and bool((b0[1:] == (b0 + c)[:-1]).all()), name  # ranges tile the rows
            owner = torch.repeat_interleave(idx, c)          # child row -> its key row
            assert bool((child[0] == k[0][owner]).all()) and bool((child[1] == k[1][owner]).all()), name
            owners[name] = owner
        # cal_sum (type_counter.rs:89-91): a counter's win is the wrapping sum of its nodes' v
        # (the generator never repeats a node id inside one counter, so merged or not)
        sums = torch.zeros(k.shape[1], dtype=torch.int64, device="cuda").index_add_(0, owners["nodes"], n[3])
        assert bool((sums[is_counter] == k[6][is_counter]).all())
    finally:
        for fam in (din.keys, din.nodes, din.members):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))


# ------------------------------------------------------------------ replica metadata (§8f.4)
@pytest.mark.parametrize("seed", range(8))
def test_replica_metadata_merge(db, seed):
    """cdb_merged_replicas vs the oracle's fold_replicas on random replica tables with tied
    times, self-references and add/del interleavings (replica/pull.rs:131-156)."""
    import random
    rng = random.Random(seed)
    addrs = [f"10.0.0.{i}:9000" for i in range(6)]
    hdrs = []
    for r in range(1 + seed % 4):
        adds = [(rng.randint(1, 8), rng.choice([1, 2, 3, 7]), f"n{rng.randint(0, 9)}", rng.choice(addrs),
                 rng.randint(0, 1 << 40)) for _ in range(rng.randint(0, 6))]
        dels = [(rng.choice(addrs), rng.randint(1, 8)) for _ in range(rng.randint(0, 4))]
        hdrs.append(o.NodeHeader(node_id=1 + r, replicas_add=adds, replicas_del=dels))
    snaps = [o.dump_all(o.DB(), h) for h in hdrs]
    m = db.merge_snapshots(snaps)
    assert m.replicas() == o.fold_replicas(snaps)
