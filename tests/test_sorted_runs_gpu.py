"""The sorted-run merge path (constdb_amd/csrc/runs.hip.h): rows grouped into one run per replica,
each ordered by key hash, merged in place without the partition pass. Its result must equal the
partition path's row for row (both emit keys in exact key-hash order inside a bucket); the
partition path itself is pinned to the oracle by tests/test_gpu_parity.py. Also: a merge result
is itself a sorted run, a run out of order falls back to the partition path, empty runs, every
bucket tier (materialised rows of the workgroup tiers), GC and key_shift."""
import ctypes

import pytest
import torch

import constdb_amd as cdb
from constdb_amd import configs

pytestmark = pytest.mark.gpu

NCOLS = (7, 6, 6)
OUT_COLS = (8, 6, 6)
SIGN = -(1 << 63)


@pytest.fixture(scope="module")
def ctx():
    from constdb_amd import build
    build.build()
    return cdb.Context(0)


def _wrap(ptr, n):
    class _Cai:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 2}
    return torch.as_tensor(_Cai(), device="cuda")


def _family_tensor(rows, ncols):
    if rows.n == 0:
        return torch.zeros((ncols, 1), dtype=torch.int64, device="cuda")
    return torch.stack([_wrap(rows.col[c], rows.n) for c in range(ncols)]).clone()


def _as_rows(t, n):
    r = cdb.DevRows()
    for c in range(t.shape[0]):
        r.col[c] = t[c].data_ptr()
    r.n = n
    return r


def _gen(ctx, cfg):
    """Device-generated replica rows copied into torch tensors (rows in key-index order)."""
    L = cdb.lib()
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
    fams = [(_family_tensor(r, NCOLS[f]), r.n) for f, r in enumerate((din.keys, din.nodes, din.members))]
    for r in (din.keys, din.nodes, din.members):
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(r))
    return fams, din.n_pos


def _sort_runs(fams, n_pos, extra_empty=False):
    """Rows of every family ordered by (pos, key hash): one run per fold position."""
    out = []
    starts = []
    for t, n in fams:
        if n == 0:
            out.append((t, 0))
            starts.append([0] * (n_pos + 1))
            continue
        key = t[0, :n] ^ SIGN                       # unsigned order as signed
        o = torch.sort(key, stable=True).indices
        pos = ((t[t.shape[0] - 1, :n] >> 48) & 0xFF)[o]
        o = o[torch.sort(pos, stable=True).indices]
        s = t[:, :n][:, o].contiguous()
        counts = torch.bincount(((s[s.shape[0] - 1] >> 48) & 0xFF), minlength=n_pos).tolist()
        st = [0]
        for c in counts[:n_pos]:
            st.append(st[-1] + c)
        out.append((s, n))
        starts.append(st)
    if extra_empty:  # an empty run in the middle
        starts = [st[:2] + [st[1]] + st[2:] for st in starts]
    return out, starts


def _input(fams, n_pos, starts=None):
    din = cdb.DevInput()
    din.keys, din.nodes, din.members = (_as_rows(t, n) for t, n in fams)
    din.n_pos = n_pos
    if starts:
        din.n_runs = len(starts[0]) - 1
        for f in range(3):
            for r, v in enumerate(starts[f]):
                din.run_start[f][r] = v
    return din


def _merge(ctx, din, **kw):
    L = cdb.lib()
    outs = [torch.empty((OUT_COLS[f], max(r.n, 1)), dtype=torch.int64, device="cuda")
            for f, r in enumerate((din.keys, din.nodes, din.members))]
    dout = cdb.DevOutput()
    dout.keys, dout.nodes, dout.members = (_as_rows(t, 0) for t in outs)
    dout.compact = 1
    opts = cdb.MergeOpts()
    for k, v in kw.items():
        setattr(opts, k, v)
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(dout),
                                 ctypes.byref(st), None))
    torch.cuda.synchronize()
    return [outs[0][:, :dout.keys.n], outs[1][:, :dout.nodes.n], outs[2][:, :dout.members.n]], st


def _same(a, b):
    for x, y in zip(a, b):
        assert x.shape == y.shape and torch.equal(x, y)


def _both(ctx, cfg, extra_empty=False, **kw):
    fams, n_pos = _gen(ctx, cfg)
    ref, st0 = _merge(ctx, _input(fams, n_pos), **kw)
    assert st0.sorted_runs == 0
    sfams, starts = _sort_runs(fams, n_pos, extra_empty)
    got, st1 = _merge(ctx, _input(sfams, n_pos, starts), **kw)
    assert st1.sorted_runs == 1
    _same(ref, got)
    for f in ("type_conflicts", "dict_merges", "deletes_gced", "members_gced", "orphan_children"):
        assert getattr(st0, f) == getattr(st1, f), f
    return got, st1, sfams, starts, n_pos


def _small(seed, universe, replicas, **kw):
    base = dict(seed=seed, universe=universe, n_replicas=replicas, replica_hi=replicas)
    base.update(kw)
    return cdb.gen_config(**base)


@pytest.mark.parametrize("seed", range(6))
def test_runs_equal_partition_random(ctx, seed):
    _both(ctx, _small(seed, 2000 + 3000 * seed, 1 + seed % 8, conflict_ppm=20000, tie_permille=100,
                      side_permille=200, mean_members=5))


@pytest.mark.parametrize("tier", [1, 2, 3, 4])
def test_runs_forced_tiers(ctx, tier):
    """Every bucket through the materialised workgroup tiers (1, 2) or the wide runs kernel (3)."""
    _both(ctx, _small(40 + tier, 3000, 5, conflict_ppm=20000, side_permille=200), force_tier=tier)


def test_runs_c4_shape_large(ctx):
    """C4's shape at 1M keys x 8 replicas: ~100K buckets, wide buckets, the row-level plan size."""
    got, st, *_ = _both(ctx, configs.c4(cdb, 1_000_000))
    assert st.wide_buckets > 0


def test_runs_gc_and_members(ctx):
    wm = (configs.T0_MS + (1 << 19)) << 22
    _both(ctx, _small(7, 20000, 4, mix_set=40, mix_dict=40, side_permille=300, del_permille=400),
          flags=cdb.MERGE_GC_DELETES | cdb.MERGE_GC_MEMBERS, gc_watermark=wm)


def test_runs_key_shift(ctx):
    """A multi-GPU rank's shard: every key hash shares its top bits; buckets use the bits below."""
    cfg = _small(9, 40000, 4)
    cfg.shard, cfg.n_shards = 1, 2
    _both(ctx, cfg, key_shift=1)


def test_runs_hot_keys(ctx):
    """C5 (Zipf hot keys) at a small size: buckets over the LDS capacity through the materialised
    global-scratch tier."""
    _, st, *_ = _both(ctx, configs.c5(cdb, universe=50_000, events=400_000))
    assert st.hot_buckets + st.mid_buckets > 0


def test_runs_empty_run(ctx):
    _both(ctx, _small(11, 5000, 3), extra_empty=True)


def test_out_of_order_run_falls_back(ctx):
    fams, n_pos = _gen(ctx, _small(12, 5000, 3))
    ref, _ = _merge(ctx, _input(fams, n_pos))
    sfams, starts = _sort_runs(fams, n_pos)
    t, n = sfams[0]
    t[:, [starts[0][1], starts[0][1] + 1]] = t[:, [starts[0][1] + 1, starts[0][1]]]  # swap two rows of run 1
    got, st = _merge(ctx, _input(sfams, n_pos, starts))
    assert st.sorted_runs == 0
    _same(ref, got)


def test_merge_output_is_a_sorted_run(ctx):
    """The merged keys (and the children, by parent) leave in key-hash order, so a merge result
    is a valid run for the next merge."""
    got, *_ = _both(ctx, configs.c4(cdb, 300_000))
    for t in got:
        if t.shape[1] > 1:
            u = t[0] ^ SIGN
            assert bool((u[1:] >= u[:-1]).all())


def test_bad_run_bounds_rejected(ctx):
    fams, n_pos = _gen(ctx, _small(13, 1000, 2))
    sfams, starts = _sort_runs(fams, n_pos)
    starts[0][-1] -= 1
    with pytest.raises(ValueError):
        _merge(ctx, _input(sfams, n_pos, starts))


def _ranges_equal(ctx, cfg, ranges):
    fams, n_pos = _gen(ctx, cfg)
    sfams, starts = _sort_runs(fams, n_pos)
    stats = []
    for mk in (lambda: _input(fams, n_pos), lambda: _input(sfams, n_pos, starts)):
        ref, st0 = _merge(ctx, mk(), pipe_ranges=1)
        got, st1 = _merge(ctx, mk(), pipe_ranges=ranges)
        _same(ref, got)
        for f in ("type_conflicts", "dict_merges", "deletes_gced", "members_gced", "orphan_children",
                  "hot_buckets", "mid_buckets", "wide_buckets"):
            assert getattr(st0, f) == getattr(st1, f), f
        stats.append(st1)
    return stats


@pytest.mark.parametrize("ranges", [2, 8, 300])
def test_pipelined_ranges_equal_one_range(ctx, ranges):
    """The bucket phase in bucket ranges, each scanned and compacted on a side stream while the
    next merges (automatic from 64M rows; cdb_merge_opts.pipe_ranges forces it): row for row the
    single-range result, on the partition and the sorted-run path."""
    _ranges_equal(ctx, configs.c4(cdb, 400_000), ranges)


def test_pipelined_ranges_more_than_buckets(ctx):
    """More ranges asked for than there are buckets: one bucket per range."""
    _ranges_equal(ctx, _small(13, 1500, 3, side_permille=200), 1 << 30)


def test_pipelined_ranges_with_workgroup_tiers(ctx):
    """Hot keys (C5): buckets reach the workgroup tiers after every range merged, so the range
    compactions stand down and the whole output is compacted again at the end."""
    for st in _ranges_equal(ctx, configs.c5(cdb, universe=50_000, events=400_000), 8):
        assert st.hot_buckets + st.mid_buckets > 0
