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
        payload = rng.integers(-2**62, 2**62, size=(5, m), dtype=np.int64)
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
        fams = [torch.from_numpy(np.ascontiguousarray(d[0][: 6 + (f == 0)] if d[0].shape[0] >= 6 else d[0]))
                for f, d in enumerate(data)]
        starts = [d[1] for d in data]
        plan = cdist.make_plan(fams, starts, world, rank)
        recv = [torch.empty((fams[f].shape[0], max(plan.total[f], 1)), dtype=torch.int64) for f in range(3)]
        kw = {"max_piece_bytes": piece} if piece else {}
        ops = cdist.exchange_runs(fams, plan, recv, **kw)
        ok = True
        for f in range(3):
            got = recv[f][:, :plan.total[f]].numpy()
            allr = [_runs(s + 17 * f, R) for s in range(world)]
            want = np.hstack([r[:, _owner(r[0], world) == rank] for r, _ in allr])
            want = want[: fams[f].shape[0]]
            ok = ok and sorted(map(tuple, got.T.tolist())) == sorted(map(tuple, want.T.tolist()))
            ok = ok and bool(np.all(_owner(got[0], world) == rank))
            st = plan.run_start[f]
            for i, (r, s) in enumerate(plan.runs):  # every receiver run: one source run, sorted
                seg = got[:, st[i]:st[i + 1]]
                u = seg[0].view(np.uint64)
                ok = ok and bool(np.all(u[1:] >= u[:-1])) and bool(np.all(seg[1] == r))
        # pieces: every transfer is cut at `piece` bytes on both sides
        p_rows = max(1, (piece or cdist.MAX_PIECE_BYTES) // 8)
        want_ops = 0
        for peer in range(world):
            if peer == rank:
                continue
            for f in range(3):
                nc = fams[f].shape[0]
                for r in range(R):
                    a, e = plan.splits[f][r][peer], plan.splits[f][r][peer + 1]
                    want_ops += nc * (-(-(e - a) // p_rows))
                    want_ops += nc * (-(-plan.recv[peer][f][r] // p_rows))
        ok = ok and ops == want_ops
        # the bench line's exchange bytes: what all ranks send to others == what all receive from others
        sent = cdist.sent_bytes(plan, fams)
        got_b = sum(plan.recv[s][f][r] * fams[f].shape[0] * 8 for s in range(world) if s != rank
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
