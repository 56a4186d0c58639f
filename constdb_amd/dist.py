"""Multi-GPU snapshot merge: key-hash sharding with an RCCL all-to-all.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI). Replica r lives on
rank r*N/R. Every key has ONE owner rank: owner = top log2(N) bits of its key hash (children
use their parent's hash, so a key and its children travel together). A merge step:
  1. pack   : cdb_partition_owner groups each family's rows by owner (HIP multisplit);
  2. counts : all_to_all of the per-owner row counts (N x 3 integers);
  3. rows   : one all_to_all_single per column, split sizes = row counts (RCCL);
  4. merge  : cdb_merge_device on the received rows with key_shift = log2(N), so the local
              buckets use the hash bits below the owner bits. Outputs stay sharded.
There is no other collective on the data path: merging is per key.
"""
from __future__ import annotations

import ctypes
import time
from typing import List, Sequence

FAMILY_COLS = (7, 6, 6)     # key rows, counter nodes, set/dict members (input layout)
OUT_COLS = (8, 6, 6)


def owner_bits(world: int) -> int:
    b = 0
    while (1 << b) < world:
        b += 1
    if (1 << b) != world:
        raise ValueError("world size must be a power of two (owner = top log2(N) hash bits)")
    return b


def owner_of(h: int, world: int) -> int:
    """Owner rank of a (parent) key hash."""
    b = owner_bits(world)
    return (h >> (64 - b)) if b else 0


def exchange_counts(send_counts: Sequence[Sequence[int]], device=None) -> List[List[int]]:
    """send_counts[f][d] = rows of family f this rank sends to rank d. Returns
    recv_counts[f][s] = rows of family f received from rank s."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    nf = len(send_counts)
    t = torch.tensor([[send_counts[f][d] for f in range(nf)] for d in range(world)], dtype=torch.int64,
                     device=device)
    r = torch.empty_like(t)
    dist.all_to_all_single(r, t)
    r = r.cpu().tolist()
    return [[r[s][f] for s in range(world)] for f in range(nf)]


# Largest piece one (source, destination) pair moves in one collective: RCCL's point-to-point
# transfers misbehave past 2^31 bytes (a 2.2 GB self-transfer never completed on MI355X), so
# bigger pairs move in several rounds.
MAX_PIECE_BYTES = 1 << 30


def exchange_columns(send_cols, send_counts: Sequence[int], recv_counts: Sequence[int], recv_cols=None,
                     max_piece_bytes: int = MAX_PIECE_BYTES):
    """All-to-all of one family's columns. send_cols: list of 1-D int64 tensors grouped by
    destination (rows for rank 0 first, ...). Returns the received columns (source-rank
    order). Works with any torch.distributed backend (RCCL on GPUs, gloo in CPU tests).
    Each column moves with dist.all_to_all over per-peer views (no staging copies), in as
    many rounds as the largest (source, destination) piece needs."""
    import torch
    import torch.distributed as dist
    world = len(send_counts)
    total = int(sum(recv_counts))
    soff = [0] * (world + 1)
    roff = [0] * (world + 1)
    for d in range(world):
        soff[d + 1] = soff[d] + int(send_counts[d])
        roff[d + 1] = roff[d] + int(recv_counts[d])
    out = []
    for c, col in enumerate(send_cols):
        dst = recv_cols[c][:total] if recv_cols is not None else torch.empty(total, dtype=col.dtype,
                                                                             device=col.device)
        piece = max(1, max_piece_bytes // col.element_size())
        # every rank runs the same number of rounds: the largest pair anywhere decides
        most = torch.tensor([max(max(send_counts), max(recv_counts))], dtype=torch.int64, device=col.device)
        dist.all_reduce(most, op=dist.ReduceOp.MAX)
        rounds = max(1, -(-int(most.item()) // piece))
        if rounds == 1:
            dist.all_to_all_single(dst, col[:soff[world]], output_split_sizes=[int(x) for x in recv_counts],
                                   input_split_sizes=[int(x) for x in send_counts])
            out.append(dst)
            continue
        lists = dist.get_backend() != "gloo"  # gloo has no list all_to_all: stage each round
        for r in range(rounds):
            a = r * piece
            ins = [col[soff[d] + min(a, int(send_counts[d])): soff[d] + min(a + piece, int(send_counts[d]))]
                   for d in range(world)]
            outs = [dst[roff[s] + min(a, int(recv_counts[s])): roff[s] + min(a + piece, int(recv_counts[s]))]
                    for s in range(world)]
            if lists:
                dist.all_to_all(outs, ins)
            else:
                got = torch.empty(sum(o.numel() for o in outs), dtype=col.dtype, device=col.device)
                dist.all_to_all_single(got, torch.cat(ins), output_split_sizes=[o.numel() for o in outs],
                                       input_split_sizes=[i.numel() for i in ins])
                k = 0
                for o in outs:
                    o.copy_(got[k:k + o.numel()])
                    k += o.numel()
        out.append(dst)
    return out


def _rows_from_tensor(cdb, t, n):
    """cdb_dev_rows view of a [ncols, cap] int64 CUDA tensor (first n rows of each column)."""
    r = cdb.DevRows()
    for c in range(t.shape[0]):
        r.col[c] = t[c].data_ptr()
    r.n = n
    return r


def _log(rank, msg):
    import sys
    print(f"[rank {rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def run_bench(cdb, args, rank, world, local_rank, c4_config, alg_bytes):
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    _log(rank, "process group up")
    ob = owner_bits(world)
    L = cdb.lib()
    ctx = cdb.Context(local_rank)
    R = args.replicas
    lo, hi = rank * R // world, (rank + 1) * R // world
    universe = args.universe_per_gpu * world
    cfg = c4_config(cdb, universe, R, args.seed, lo, hi)
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
    _log(rank, f"generated {din.keys.n} key rows")
    fams_in = [din.keys, din.nodes, din.members]
    n_in = [f.n for f in fams_in]
    send = [torch.empty((FAMILY_COLS[f], max(n_in[f], 1)), dtype=torch.int64, device=dev) for f in range(3)]
    opts = cdb.MergeOpts()
    opts.key_shift = ob
    st = cdb.MergeStats()
    counts = (ctypes.c_uint64 * world)()
    state = {}
    # One explicit stream for the whole step: torch makes it wait for each RCCL collective, and
    # the library's kernels run on it too (the legacy default stream's handle is 0, which the
    # library would read as "use the context's own stream" -- unordered with the exchange).
    cs = torch.cuda.Stream(device=dev)

    def step():
        with torch.cuda.stream(cs):
            _step()

    def _step():
        stream = torch.cuda.current_stream().cuda_stream
        assert stream, "the merge must run on the exchange's (non-default) stream"
        send_counts = []
        for f in range(3):
            out_rows = _rows_from_tensor(cdb, send[f], n_in[f])
            ctx.check(L.cdb_partition_owner(ctx.handle, ctypes.byref(fams_in[f]), FAMILY_COLS[f], ob,
                                            ctypes.byref(out_rows), counts, ctypes.c_void_p(stream)))
            send_counts.append([counts[d] for d in range(world)])
        _log(rank, "packed") if not state.get("quiet") else None
        recv_counts = exchange_counts(send_counts, device=dev)
        _log(rank, f"counts exchanged {recv_counts}") if not state.get("quiet") else None
        recv = []
        for f in range(3):
            total = sum(recv_counts[f])
            buf = state.get(("recv", f))
            if buf is None or buf.shape[1] < max(total, 1):
                buf = torch.empty((FAMILY_COLS[f], max(total, 1) + max(total, 1) // 8), dtype=torch.int64,
                                  device=dev)
                state[("recv", f)] = buf
            cols = [send[f][c][:n_in[f]] for c in range(FAMILY_COLS[f])]
            exchange_columns(cols, send_counts[f], recv_counts[f], recv_cols=buf)
            recv.append((buf, total))
        if not state.get("quiet"):  # first (warmup) step: locate a stall in the log
            torch.cuda.current_stream().synchronize()
            _log(rank, "rows exchanged")
        din2 = cdb.DevInput()
        din2.keys = _rows_from_tensor(cdb, recv[0][0], recv[0][1])
        din2.nodes = _rows_from_tensor(cdb, recv[1][0], recv[1][1])
        din2.members = _rows_from_tensor(cdb, recv[2][0], recv[2][1])
        din2.n_pos = R
        dout = cdb.DevOutput()
        outs = []
        for f, fam in enumerate((dout.keys, dout.nodes, dout.members)):
            buf = state.get(("out", f))
            need = max(recv[f][1], 1)
            if buf is None or buf.shape[1] < need:
                buf = torch.empty((OUT_COLS[f], need + need // 8), dtype=torch.int64, device=dev)
                state[("out", f)] = buf
            outs.append(buf)
        dout.keys = _rows_from_tensor(cdb, outs[0], 0)
        dout.nodes = _rows_from_tensor(cdb, outs[1], 0)
        dout.members = _rows_from_tensor(cdb, outs[2], 0)
        dout.compact = 1
        ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din2), ctypes.byref(opts), ctypes.byref(dout),
                                     ctypes.byref(st), ctypes.c_void_p(stream)))
        _log(rank, "merged") if not state.get("quiet") else None
        state["quiet"] = True

    for i in range(args.warmup):
        step()
        _log(rank, f"warmup step {i} done")
    bucket_ms = 0.0
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        bucket_ms += st.bucket_ms
    torch.cuda.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    tot = torch.tensor([n_in[0], n_in[1], n_in[2]], dtype=torch.int64, device=dev)
    dist.all_reduce(tot)
    ms = el.item() * 1e3 / args.steps
    entries = int(tot[0].item())
    B = alg_bytes(st)
    bk = bucket_ms / args.steps
    res = {
        "metric": "merged CRDT entries/sec (snapshot merge)",
        "value": entries / (ms * 1e-3),
        "unit": "entries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: seeded GenModel replica states generated in HBM (keys 'key:<i>')",
        "config": {"workload": f"C4 anti-entropy: {universe} keys x {R} replicas, replica r on rank r*N/R, "
                               f"rows routed to owner = top log2(N) key-hash bits via RCCL all-to-all",
                   "replicas": R, "key_rows_in_total": entries, "parallelism": f"key-hash sharding x{world}"},
        "roofline": {"bound": "hbm", "kernel": "bucket_wave_kernel (rank 0)",
                     "achieved": B / (bk * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                     "frac": B / (bk * 1e-3) / 1e9 / 8000.0, "traffic": None},
    }
    dist.barrier()
    for fam in (din.keys, din.nodes, din.members):
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
    dist.destroy_process_group()
    return res


def sharded_merge(cdb, ctx, din, n_pos: int, stream=None):
    """One sharded merge step, outside the bench's timing harness: pack this rank's rows by
    owner (cdb_partition_owner), exchange them (RCCL on GPU tensors; gloo through host copies),
    merge the received shard with key_shift = log2(N). Returns ([keys, nodes, members] output
    column tensors, MergeStats). Used by the multi-process tests; bench.py runs the same steps
    with persistent buffers."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    ob = owner_bits(world)
    L = cdb.lib()
    dev = torch.device("cuda", torch.cuda.current_device())
    on_host = dist.get_backend() == "gloo"
    fams = [din.keys, din.nodes, din.members]
    counts = (ctypes.c_uint64 * world)()
    send, send_counts = [], []
    for f, fam in enumerate(fams):
        t = torch.empty((FAMILY_COLS[f], max(fam.n, 1)), dtype=torch.int64, device=dev)
        ctx.check(L.cdb_partition_owner(ctx.handle, ctypes.byref(fam), FAMILY_COLS[f], ob,
                                        ctypes.byref(_rows_from_tensor(cdb, t, fam.n)), counts, stream))
        send.append(t)
        send_counts.append([counts[d] for d in range(world)])
    recv_counts = exchange_counts(send_counts, device=None if on_host else dev)
    recv = []
    for f in range(3):
        cols = [send[f][c][:fams[f].n] for c in range(FAMILY_COLS[f])]
        if on_host:
            cols = [c.cpu() for c in cols]
        got = exchange_columns(cols, send_counts[f], recv_counts[f])
        total = int(sum(recv_counts[f]))
        buf = torch.empty((FAMILY_COLS[f], max(total, 1)), dtype=torch.int64, device=dev)
        for c, g in enumerate(got):
            buf[c][:total].copy_(g)
        recv.append((buf, total))
    torch.cuda.synchronize()
    d2 = cdb.DevInput()
    d2.keys, d2.nodes, d2.members = (_rows_from_tensor(cdb, b, n) for b, n in recv)
    d2.n_pos = n_pos
    dout = cdb.DevOutput()
    outs = []
    for f, (b, n) in enumerate(recv):
        t = torch.empty((OUT_COLS[f], max(n, 1)), dtype=torch.int64, device=dev)
        outs.append(t)
    dout.keys, dout.nodes, dout.members = (_rows_from_tensor(cdb, t, 0) for t in outs)
    dout.compact = 1
    opts = cdb.MergeOpts()
    opts.key_shift = ob
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(d2), ctypes.byref(opts), ctypes.byref(dout),
                                 ctypes.byref(st), stream))
    torch.cuda.synchronize()
    return [outs[0][:, :dout.keys.n], outs[1][:, :dout.nodes.n], outs[2][:, :dout.members.n]], st
