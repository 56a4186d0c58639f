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


def _rows(rank, n=997):
    rng = np.random.default_rng(1000 + rank)
    kh = rng.integers(0, 2**63, size=n, dtype=np.int64) * 2 + rng.integers(0, 2, size=n)
    payload = rng.integers(-2**62, 2**62, size=(5, n), dtype=np.int64)
    return np.vstack([kh[None, :], payload])  # [cols, n]; column 0 = key hash


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
        rows = _rows(rank)
        own = _owner(rows[0], world)
        order = np.argsort(own, kind="stable")          # the pack step (cdb_partition_owner on GPU)
        packed = rows[:, order]
        counts = np.bincount(own, minlength=world).tolist()
        recv_counts = cdist.exchange_counts([counts])
        cols = [torch.from_numpy(np.ascontiguousarray(packed[c])) for c in range(packed.shape[0])]
        kw = {"max_piece_bytes": piece} if piece else {}
        got = cdist.exchange_columns(cols, counts, recv_counts[0], **kw)
        got = np.vstack([g.numpy()[None, :] for g in got])
        want = np.hstack([r[:, _owner(r[0], world) == rank] for r in (_rows(s) for s in range(world))])
        ok = sorted(map(tuple, got.T.tolist())) == sorted(map(tuple, want.T.tolist()))
        ok = ok and bool(np.all(_owner(got[0], world) == rank)) and sum(recv_counts[0]) == got.shape[1]
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,piece", [(2, None), (4, None), (2, 800), (4, 2000)])
def test_exchange_gloo(world, piece):
    """The column exchange; a small piece limit forces the multi-round path that keeps every
    (source, destination) transfer under RCCL's 2^31-byte limit at full size."""
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
