"""Multi-GPU path on CPU: the exchange plumbing of constdb_amd.dist over gloo (world_size 2
and 4), and the sharding decomposition (per-key independence) checked with the oracle."""
import os
import socket

import numpy as np
import pytest

import cdb_oracle
import constdb_amd as cdb
from constdb_amd import dist as cdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SIGN = -(1 << 63)


def _runs(rank, n_runs, n=997):
    """Rank `rank`'s rows as n_runs runs (some empty), each ascending in unsigned key hash:
    [cols, n] with column 0 = key hash, plus the run offsets."""
    rng = np.random.default_rng(1000 + rank)
    sizes = rng.multinomial(n, [1 / n_runs] * n_runs)
    sizes[rank % n_runs] = 0  # an empty run
    parts = []
    for r, m in enumerate(sizes):
        kh = rng.integers(0, 2**63, size=m, dtype=np.int64) * 2 + rng.integers(0, 2, size=m)
        kh = np.sort(kh.view(np.uint64)).view(np.int64)
        payload = rng.integers(-2**62, 2**62, size=(6, m), dtype=np.int64)
        payload[0] = r  # the run a row came from
        parts.append(np.vstack([kh[None, :], payload]))
    starts = [0] + np.cumsum(sizes).tolist()
    return np.hstack(parts), starts


def _owner(col0, world):
    b = cdist.owner_bits(world)
    return (col0.astype(np.uint64) >> np.uint64(64 - b)).astype(np.int64) if b else np.zeros_like(col0)


def _worker(rank, world, port, q, piece=None):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        R = 3
        # three families of different widths, as key rows / nodes / members
        data = [_runs(rank + 17 * f, R) for f in range(3)]
        cols = [np.ascontiguousarray(d[0][: 6 + (f == 0)]) for f, d in enumerate(data)]
        # the records layout dist.py moves: (hash [n], records [n, ncols - 1])
        fams = [(torch.from_numpy(c[0].copy()), torch.from_numpy(np.ascontiguousarray(c[1:].T))) for c in cols]
        starts = [d[1] for d in data]
        plan = cdist.make_plan(fams, starts, world, rank)
        recv = cdist.recv_buffers(plan.total, "cpu")
        kw = {"max_piece_bytes": piece} if piece else {}
        ops = cdist.exchange_runs(fams, plan, recv, **kw)
        ok = True
        for f in range(3):
            nc = cols[f].shape[0]
            h, rec = recv[f]
            got = np.vstack([h[:plan.total[f]].numpy()[None, :], rec[:plan.total[f]].numpy().T])
            allr = [_runs(s + 17 * f, R) for s in range(world)]
            want = np.hstack([r[:, _owner(r[0], world) == rank] for r, _ in allr])
            want = want[:nc]
            ok = ok and sorted(map(tuple, got.T.tolist())) == sorted(map(tuple, want.T.tolist()))
            ok = ok and bool(np.all(_owner(got[0], world) == rank))
            st = plan.run_start[f]
            # every receiver run: one source run (cdb_shard_recv_plan: source-major), sorted
            ok = ok and plan.runs == sorted(plan.runs)
            for i, (s_, r) in enumerate(plan.runs):
                seg = got[:, st[i]:st[i + 1]]
                u = seg[0].view(np.uint64)
                ok = ok and bool(np.all(u[1:] >= u[:-1])) and bool(np.all(seg[1] == r))
        # pieces: every transfer is cut at `piece` bytes on both sides; two arrays per slice
        # (hash column, records)
        lim = piece or cdist.MAX_PIECE_BYTES
        want_ops = 0
        for peer in range(world):
            if peer == rank:
                continue
            for f in range(3):
                w = cols[f].shape[0] - 1
                for r in range(R):
                    a, e = plan.splits[f][r][peer], plan.splits[f][r][peer + 1]
                    n_in = plan.recv[peer][f][r]
                    for words in (1, w):
                        want_ops += -(-((e - a) * words) // max(1, lim // 8))
                        want_ops += -(-(n_in * words) // max(1, lim // 8))
        ok = ok and ops == want_ops
        if piece is None:  # one transfer per (peer, family, run, array): at most 2 x 3 R (N - 1) sends
            ok = ok and ops <= 2 * (2 * 3 * R * (world - 1))
        # the bench line's exchange bytes: what all ranks send to others == what all receive from others
        sent = cdist.sent_bytes(plan, fams)
        got_b = sum(plan.recv[s][f][r] * cols[f].shape[0] * 8 for s in range(world) if s != rank
                    for f in range(3) for r in range(R))
        tot = torch.tensor([float(sum(sent)), float(got_b)], dtype=torch.float64)
        dist.all_reduce(tot)
        ok = ok and sent[rank] == 0 and tot[0].item() == tot[1].item() and (world == 1 or tot[0].item() > 0)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,piece", [(2, None), (4, None), (2, 800), (4, 2000)])
def test_exchange_gloo(world, piece):
    """The run-slice exchange: every rank receives exactly the rows it owns, each source run's
    slice as one receiver run still in key-hash order; a small piece limit cuts every transfer
    into pieces on both sides (the 1 GiB limit at full size), with the op count pinned."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, piece)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


def test_owner_splits_cpu():
    import torch
    rows, starts = _runs(5, 4, n=3000)
    kh = torch.from_numpy(rows[0].copy())
    for world in (1, 2, 4, 8):
        sp = cdist.owner_splits(kh, starts, world).tolist()
        for r in range(4):
            a, e = starts[r], starts[r + 1]
            own = _owner(rows[0, a:e], world)
            assert sp[r][0] == a and sp[r][world] == e
            for d in range(world):
                assert np.all(own[sp[r][d] - a:sp[r][d + 1] - a] == d)


def _records(dump: bytes):
    recs, cur = [], []
    for line in dump.decode().splitlines():
        if not line.startswith(" ") and cur:
            recs.append("\n".join(cur))
            cur = []
        cur.append(line)
    if cur:
        recs.append("\n".join(cur))
    return recs


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shard_decomposition(world):
    """Merging per owner shard and concatenating == merging everything."""
    base = dict(seed=11, universe=4000, n_replicas=4, replica_hi=4)
    full = [cdb.gen_snapshot(cdb.gen_config(**base), r) for r in range(4)]
    rc, want, _ = cdb_oracle.fold(full)
    assert rc == 0
    parts = []
    for shard in range(world):
        cfg = cdb.gen_config(shard=shard, n_shards=world, **base)
        rc, d, _ = cdb_oracle.fold([cdb.gen_snapshot(cfg, r) for r in range(4)])
        assert rc == 0
        parts += _records(d)
    assert sorted(parts) == sorted(_records(want))
    assert cdist.owner_of(0xC000000000000000, 4) == 3 and cdist.owner_of(123, 1) == 0
    with pytest.raises(ValueError):
        cdist.owner_bits(3)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_library_plan_cpu(world):
    """The one exchange plan (cdb_shard_splits / cdb_shard_recv_plan: what cdb_merge_sharded runs and
    what dist.py's Plan takes its receive layout from), on the host at N = 2, 4, 8: the library's
    splits equal torch.searchsorted's (dist.owner_splits) and cut every run into owner slices; the
    receive layout of every destination holds exactly the rows owned by it, one run per (source,
    source run) with rows, in (source, run) order, and the totals add up."""
    import ctypes
    import torch
    L = cdb.lib()
    R = 3
    srcs = [[_runs(s + 17 * f, R) for f in range(3)] for s in range(world)]
    for src in srcs:
        for rows, starts in src:
            kh = np.ascontiguousarray(rows[0]).view(np.uint64)
            out = (ctypes.c_uint64 * (R * (world + 1)))()
            rs = (ctypes.c_uint64 * (R + 1))(*starts)
            assert L.cdb_shard_splits(kh.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), rs, R, world, out) == 0
            lib_sp = [[out[r * (world + 1) + d] for d in range(world + 1)] for r in range(R)]
            assert lib_sp == cdist.owner_splits(torch.from_numpy(rows[0].copy()), starts, world).tolist()
            for r in range(R):
                own = _owner(rows[0, starts[r]:starts[r + 1]], world)
                for d in range(world):
                    assert np.all(own[lib_sp[r][d] - starts[r]:lib_sp[r][d + 1] - starts[r]] == d)
    for dst in range(world):
        recv = [[[0] * R for _ in range(3)] for _ in range(world)]
        for s in range(world):
            for f in range(3):
                rows, starts = srcs[s][f]
                for r in range(R):
                    seg = rows[0, starts[r]:starts[r + 1]]
                    recv[s][f][r] = int((_owner(seg, world) == dst).sum())
        plan = cdist.Plan([[[0] * (world + 1)] * R] * 3, recv, world, dst, R)
        want_runs = [(s, r) for s in range(world) for r in range(R) if any(recv[s][f][r] for f in range(3))]
        assert plan.runs == want_runs
        for f in range(3):
            assert plan.total[f] == sum(recv[s][f][r] for s in range(world) for r in range(R))
            st = plan.run_start[f]
            assert st[0] == 0 and st[-1] == plan.total[f]
            for i, (s, r) in enumerate(plan.runs):
                assert st[i + 1] - st[i] == recv[s][f][r] and plan.dest(f, r, s) == st[i]
    # more runs than the caller's room: refused, with the count
    k = ctypes.c_uint32()
    cnt = (ctypes.c_uint64 * 6)(1, 1, 0, 0, 0, 0)
    nr = (ctypes.c_uint32 * 1)(2)
    a, b = (ctypes.c_uint32 * 1)(), (ctypes.c_uint32 * 1)()
    st = (ctypes.c_uint64 * 6)()
    tot = (ctypes.c_uint64 * 3)()
    assert L.cdb_shard_recv_plan(1, nr, cnt, 1, ctypes.byref(k), a, b, st, tot) == cdb.BAD_ARGUMENT and k.value == 2


def test_multi_context_refuses_missing_rccl(monkeypatch):
    """cdb_ctx_create_multi over distinct devices never falls back silently to another transport:
    with RCCL unloadable (CDB_RCCL_LIB naming a missing file) it returns CDB_DEVICE_ERROR with the
    reason in cdb_last_error(NULL), before touching any device (so this runs without a GPU).
    CDB_SHARD_TRANSPORT=peer asks for HIP peer copies explicitly and passes that check (here it then
    finds no device). A device listed twice (slots sharing a GPU) never needs RCCL."""
    import ctypes
    from constdb_amd import build
    build.build()
    L = cdb.lib()
    devs = (ctypes.c_int * 2)(0, 1)
    h = ctypes.c_void_p()
    monkeypatch.setenv("CDB_RCCL_LIB", "/nonexistent/librccl.so.1")
    monkeypatch.delenv("CDB_SHARD_TRANSPORT", raising=False)
    assert L.cdb_ctx_create_multi(ctypes.byref(h), 2, devs) == cdb.DEVICE_ERROR and not h.value
    assert b"cannot load RCCL" in L.cdb_last_error(None)
    with pytest.raises(Exception, match="cannot load RCCL"):
        cdb.Context(devices=[0, 1])
    monkeypatch.setenv("CDB_SHARD_TRANSPORT", "peer")
    st = L.cdb_ctx_create_multi(ctypes.byref(h), 2, devs)
    if st == cdb.OK:  # (a GPU box: a context over peer copies)
        L.cdb_ctx_destroy(h)
    else:
        assert st == cdb.NO_DEVICE
    monkeypatch.delenv("CDB_SHARD_TRANSPORT")
    same = (ctypes.c_int * 2)(0, 0)
    st = L.cdb_ctx_create_multi(ctypes.byref(h), 2, same)
    if st == cdb.OK:
        L.cdb_ctx_destroy(h)
    else:
        assert st == cdb.NO_DEVICE
