"""Several device slots in one process (cdb_ctx_create_multi / cdb_merge_sharded).

The box has one GPU, so the slots name device 0 more than once: the library then moves rows by
device copies instead of RCCL (the split, the plan, the per-device merges with key_shift =
log2(N) and the outputs are the same code either way). Checks: the shards' outputs, concatenated
in slot order, equal the single-device merge of every replica row for row (keys in key-hash
order, so slot d holds the keys whose top log2(N) hash bits are d; child ranges are slot-local);
the same through the oracle's canonical dump; inputs in sorted runs stay on the sorted-run path;
inputs not in runs, or with a run out of order, are grouped by owner first and still merge the
same."""
import ctypes

import pytest
import torch

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import SIGN, sort_into_runs, wrap

pytestmark = pytest.mark.gpu

KCOLS = (("keys", 7), ("nodes", 6), ("members", 6))
OCOLS = (("keys", 8), ("nodes", 6), ("members", 6))


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _gen(c, cfg, lo, hi, records=False):
    L = cdb.lib()
    g = cdb.GenConfig()
    ctypes.memmove(ctypes.byref(g), ctypes.byref(cfg), ctypes.sizeof(g))
    g.replica_lo, g.replica_hi = lo, hi
    if records:
        g.flags |= cdb.GEN_ROWS_RECORDS
    din = cdb.DevInput()
    c.check(L.cdb_gen_device(c.handle, ctypes.byref(g), ctypes.byref(din)))
    din.n_pos = cfg.n_replicas
    return din


def _release(c, *sets):
    for s in sets:
        for name, _ in KCOLS:
            cdb.lib().cdb_dev_rows_release(c.handle, ctypes.byref(getattr(s, name)))


def _single(ctx, cfg, runs=True):
    """Reference: every replica on one context, merged by cdb_merge_device."""
    L = cdb.lib()
    din = _gen(ctx, cfg, 0, cfg.n_replicas)
    if runs:
        sort_into_runs(din, cfg.n_replicas)
    dout = cdb.DevOutput()
    for name, nc in OCOLS:
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(r), getattr(din, name).n, nc))
        setattr(dout, name, r)
    dout.compact = 1
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.merge_opts()), ctypes.byref(dout),
                                 ctypes.byref(st), None))
    out = [torch.stack([wrap(getattr(dout, name).col[c], getattr(dout, name).n) for c in range(nc)]).clone()
           for name, nc in OCOLS]
    _release(ctx, din, dout)
    return out, st


def _concat(outs):
    """Slot outputs concatenated in slot order, child ranges made absolute."""
    fam = []
    base = [0, 0]
    keys = []
    for o in outs:
        k = torch.stack([wrap(o.keys.col[c], o.keys.n) for c in range(8)]).clone() if o.keys.n else \
            torch.zeros((8, 0), dtype=torch.int64, device="cuda")
        tag = (k[5] >> 56) & 0xFF
        cnt = k[7] & 0xFFFFFF
        shift = torch.where(tag == 0, base[0], torch.where((tag == 4) | (tag == 5), base[1], 0))
        k[7] = (((k[7] >> 24) + torch.where(cnt > 0, shift, 0)) << 24) | cnt
        keys.append(k)
        base[0] += o.nodes.n
        base[1] += o.members.n
    fam.append(torch.cat(keys, dim=1))
    for name, nc in OCOLS[1:]:
        parts = [torch.stack([wrap(getattr(o, name).col[c], getattr(o, name).n) for c in range(nc)])
                 for o in outs if getattr(o, name).n]
        fam.append(torch.cat(parts, dim=1) if parts else torch.zeros((nc, 0), dtype=torch.int64, device="cuda"))
    return fam


def _sharded(mctx, cfg, runs=True, scramble=None, records=False):
    N = mctx.n_devices
    R = cfg.n_replicas
    ins = []
    for i in range(N):
        d = _gen(mctx.shard(i), cfg, i * R // N, (i + 1) * R // N, records)
        if runs:
            sort_into_runs(d, R)
        ins.append(d)
    if scramble is not None:  # slot `scramble` claims runs its rows do not form
        d = ins[scramble]
        kh = wrap(d.keys.col[0], d.keys.n)
        kh.copy_(kh.flip(0))
        for c in range(1, 7):
            col = wrap(d.keys.col[c], d.keys.n)
            col.copy_(col.flip(0))
        torch.cuda.synchronize()
    outs, sts, xs = cdb.merge_sharded(mctx, ins)
    got = _concat(outs)
    for i in range(N):
        _release(mctx.shard(i), ins[i])
    return got, sts, xs


def _owner_ok(keys, N):
    b = N.bit_length() - 1
    u = keys[0] ^ SIGN
    assert bool((u[1:] >= u[:-1]).all()), "concatenated slots must be in key-hash order"


@pytest.mark.parametrize("slots,runs", [(1, True), (2, True), (4, True), (2, False), (4, False)])
def test_sharded_equals_single_merge(ctx, slots, runs):
    cfg = configs.c4(cdb, 300_000)
    want, st1 = _single(ctx, cfg)
    mctx = cdb.Context(devices=[0] * slots)
    try:
        got, sts, xs = _sharded(mctx, cfg, runs=runs)
        for g, w in zip(got, want):
            assert g.shape == w.shape and torch.equal(g, w)
        _owner_ok(got[0], slots)
        assert sum(s.key_rows_in for s in sts) == st1.key_rows_in
        assert sum(s.type_conflicts for s in sts) == st1.type_conflicts
        assert xs.n_devices == slots and xs.transport == (0 if slots == 1 else 2)
        if runs:
            assert all(s.sorted_runs == 1 for s in sts)
            assert xs.packed == 0
        elif slots > 1:
            assert xs.packed == slots
        if slots > 1:
            moved = sum(xs.link_bytes[i][j] for i in range(slots) for j in range(slots) if i != j)
            assert moved == xs.bytes_moved > 0 and xs.bytes_local > 0
    finally:
        mctx.close()


@pytest.mark.parametrize("slots,runs", [(2, True), (4, True), (2, False)])
def test_sharded_records_equals_single_merge(ctx, slots, runs):
    """Records inputs (hash column + records, cdb_dev_rows.stride): the exchange moves two arrays per
    slice, the received rows are records, and the result equals the single-device merge."""
    cfg = configs.c4(cdb, 300_000)
    want, _ = _single(ctx, cfg)
    mctx = cdb.Context(devices=[0] * slots)
    try:
        got, sts, xs = _sharded(mctx, cfg, runs=runs, records=True)
        for g, w in zip(got, want):
            assert g.shape == w.shape and torch.equal(g, w)
        if runs:
            assert all(s.sorted_runs == 1 for s in sts) and xs.packed == 0
    finally:
        mctx.close()


def test_sharded_run_out_of_order_is_packed(ctx):
    cfg = configs.c4(cdb, 200_000)
    want, _ = _single(ctx, cfg)
    mctx = cdb.Context(devices=[0, 0])
    try:
        got, sts, xs = _sharded(mctx, cfg, scramble=1)
        assert xs.packed == 1
        for g, w in zip(got, want):
            assert torch.equal(g, w)
    finally:
        mctx.close()


def test_sharded_vs_oracle(ctx):
    """Replica snapshots decoded, uploaded to their slots (fold position = replica index), merged
    sharded; the concatenated result's canonical dump equals the oracle's fold."""
    cfg = cdb.gen_config(seed=31, universe=40_000, n_replicas=6, replica_hi=6, conflict_ppm=20000,
                         tie_permille=100, side_permille=200, mix_set=20, mix_dict=20, del_permille=300)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(6)]
    batches = [cdb.decode_snapshot(s) for s in snaps]
    rc, want, _ = cdb_oracle.fold(snaps)
    assert rc == 0
    N = 2
    mctx = cdb.Context(devices=[0] * N)
    try:
        ins = []
        for i in range(N):
            lo, hi = i * 6 // N, (i + 1) * 6 // N
            c = mctx.shard(i)
            d = cdb.DevInput()
            arr = (ctypes.c_void_p * (hi - lo))(*[b.handle for b in batches[lo:hi]])
            c.check(cdb.lib().cdb_upload_batches(c.handle, arr, hi - lo, ctypes.byref(d)))
            for name, nc in KCOLS:
                rows = getattr(d, name)
                if rows.n:
                    wrap(rows.col[nc - 1], rows.n).add_(lo << 48)
            d.n_pos = 6
            sort_into_runs(d, 6)
            ins.append(d)
        outs, sts, xs = cdb.merge_sharded(mctx, ins)
        got = _concat(outs)
        for i in range(N):
            _release(mctx.shard(i), ins[i])
        keep = [t.contiguous() for t in got]
        dout = cdb.DevOutput()
        for f, (name, nc) in enumerate(OCOLS):
            r = cdb.DevRows()
            for c in range(nc):
                r.col[c] = keep[f][c].data_ptr()
            r.n = keep[f].shape[1]
            setattr(dout, name, r)
        dout.compact = 1
        m = cdb.merged_from_device(ctx, dout, batches)
        assert m.canonical_dump() == want
    finally:
        mctx.close()


def test_sharded_8_slots_records_vs_oracle(ctx):
    """The north star's node shape (server.rs:95,128-130 with 8 GPUs): 8 slots, 3 owner bits, one replica
    per slot, C4's shape at 1M keys in the records layout. Each slot's replica is decoded on the host,
    uploaded to its slot with its fold position, laid out as one run; cdb_merge_sharded splits every run
    into 8 owner slices, moves 56 of them between slots and merges each shard; the concatenated result's
    canonical dump equals the oracle's sequential fold of the 8 snapshots."""
    from constdb_amd.runs import to_records
    R = N = 8
    cfg = configs.c4(cdb, 1_000_000)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(R)]
    batches = [cdb.decode_snapshot(s) for s in snaps]
    rc, want, ost = cdb_oracle.fold(snaps)
    assert rc == 0
    mctx = cdb.Context(devices=[0] * N)
    try:
        ins = []
        for i in range(N):
            c = mctx.shard(i)
            d = cdb.DevInput()
            arr = (ctypes.c_void_p * 1)(batches[i].handle)
            c.check(cdb.lib().cdb_upload_batches(c.handle, arr, 1, ctypes.byref(d)))
            for name, nc in KCOLS:
                rows = getattr(d, name)
                if rows.n:
                    wrap(rows.col[nc - 1], rows.n).add_(i << 48)
            to_records(cdb, c, d)
            assert d.keys.stride == 6 and d.nodes.stride == 5
            d.n_pos = R
            sort_into_runs(d, R)
            ins.append(d)
        outs, sts, xs = cdb.merge_sharded(mctx, ins)
        assert xs.n_devices == N and xs.transport == 2
        assert all(s.sorted_runs == 1 for s in sts)
        assert sum(s.type_conflicts for s in sts) == ost.type_conflicts
        moved = [[xs.link_bytes[i][j] for j in range(N)] for i in range(N)]
        assert all(moved[i][j] > 0 for i in range(N) for j in range(N) if i != j)  # every pair exchanged rows
        got = _concat(outs)
        for i in range(N):
            _release(mctx.shard(i), ins[i])
        _owner_ok(got[0], N)
        keep = [t.contiguous() for t in got]
        dout = cdb.DevOutput()
        for f, (name, nc) in enumerate(OCOLS):
            r = cdb.DevRows()
            for c in range(nc):
                r.col[c] = keep[f][c].data_ptr()
            r.n = keep[f].shape[1]
            setattr(dout, name, r)
        dout.compact = 1
        m = cdb.merged_from_device(ctx, dout, batches)
        assert m.canonical_dump() == want
    finally:
        mctx.close()


@pytest.mark.parametrize("slots", [1, 2])
def test_sharded_output_passed_back_is_rejected(ctx, slots):
    """A previous call's outputs live in the library's workspace, which the next call may regrow:
    passing them back as inputs is refused (CDB_BAD_ARGUMENT), at one slot as at several."""
    cfg = configs.c4(cdb, 50_000)
    mctx = cdb.Context(devices=[0] * slots)
    try:
        ins = []
        for i in range(slots):
            d = _gen(mctx.shard(i), cfg, i * cfg.n_replicas // slots, (i + 1) * cfg.n_replicas // slots, False)
            sort_into_runs(d, cfg.n_replicas)
            ins.append(d)
        outs, _, _ = cdb.merge_sharded(mctx, ins)
        back = []
        for o in outs:
            d = cdb.DevInput()
            d.keys, d.nodes, d.members = o.keys, o.nodes, o.members
            d.n_pos = cfg.n_replicas
            back.append(d)
        with pytest.raises(ValueError, match="workspace"):
            cdb.merge_sharded(mctx, back)
        for i in range(slots):
            _release(mctx.shard(i), ins[i])
    finally:
        mctx.close()
