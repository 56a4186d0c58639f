"""The sharded merge end to end on the GPU with two ranks: each rank generates
its replicas in HBM as key-hash-ordered runs, sends every run's owner slice (top key-hash bit)
to its owner (gloo through host copies: both ranks share this box's one GPU, which RCCL
refuses), and merges the received runs on the sorted-run path with key_shift = 1. The union of the two shards' outputs must equal the single-GPU merge of all
replicas: the same key rows and the same child rows under the same keys."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch  # noqa: F401  -- before libcdbmerge loads (one HIP runtime per process)

import constdb_amd as cdb

pytestmark = pytest.mark.gpu

UNIVERSE, REPLICAS, SEED = 200_000, 8, 12


def _cfg(lo, hi):
    return cdb.gen_config(seed=SEED, universe=UNIVERSE, n_replicas=REPLICAS, replica_lo=lo, replica_hi=hi,
                          mean_members=4, max_nodes=4)


def _canon(outs):
    """Order-free form of a merge result: key rows without the child-range word, child rows
    keyed by their parent (pkh, pkf) -- child positions differ between layouts."""
    k, n, m = (t.cpu().numpy().view(np.uint64) for t in outs)
    keys = np.unique(k[:7].T, axis=0)
    nodes = np.unique(n.T, axis=0) if n.shape[1] else n.T
    mems = np.unique(m.T, axis=0) if m.shape[1] else m.T
    return keys, nodes, mems


def _worker(rank, world, port, outdir):
    import ctypes
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import constdb_amd as cdb2
        from constdb_amd import dist as cdist
        torch.cuda.set_device(0)
        ctx = cdb2.Context(0)
        L = cdb2.lib()
        din = cdb2.DevInput()
        lo, hi = rank * REPLICAS // world, (rank + 1) * REPLICAS // world
        ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(_cfg(lo, hi)), ctypes.byref(din)))
        outs, st, plan = cdist.sharded_merge(cdb2, ctx, din, REPLICAS)
        assert st.sorted_runs == 1 and len(plan.runs) == REPLICAS  # one receiver run per replica
        k, n, m = _canon(outs)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), k=k, n=n, m=m)
        for fam in (din.keys, din.nodes, din.members):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_merge_equals_single():
    import ctypes
    import torch.multiprocessing as mp
    from test_gpu_parity import _dev_merge
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(r, 2, port, d)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        parts = [np.load(os.path.join(d, f"r{r}.npz")) for r in range(2)]
    c = cdb.Context(0)
    L = cdb.lib()
    din = cdb.DevInput()
    c.check(L.cdb_gen_device(c.handle, ctypes.byref(_cfg(0, REPLICAS)), ctypes.byref(din)))
    try:
        outs, st = _dev_merge(c, din, torch)
        want = _canon(outs)
    finally:
        for fam in (din.keys, din.nodes, din.members):
            L.cdb_dev_rows_release(c.handle, ctypes.byref(fam))
    assert st.key_rows_in > 164_000 * 4  # large enough for the row-level + per-segment plan
    for i, name in enumerate(("keys", "nodes", "members")):
        got = np.unique(np.concatenate([p[name[0]] for p in parts]), axis=0)
        assert got.shape == want[i].shape and np.array_equal(got, want[i]), name
        # each shard holds only its own keys: no row appears on both ranks
        assert sum(p[name[0]].shape[0] for p in parts) == want[i].shape[0], name
