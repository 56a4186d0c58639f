"""Multi-GPU snapshot merge: key-hash sharding with RCCL point-to-point over xGMI.

One process per GPU (torch.distributed, backend "nccl" = RCCL). Replica r lives on rank
r*N/R, as one run: its rows in key-hash order (runs.py), in the records layout (the key-hash
column plus one record per row, cdb_merge.h). Every key has ONE owner rank: the top log2(N) bits
of its key hash (children use their parent's hash, so a key and its children travel together).
Because a run is in hash order, the rows a rank owes owner d are ONE contiguous slice of every run
-- of the hash column and of the records alike -- so there is no pack pass. A merge step:
  1. splits : per (family, run), the owner boundaries by binary search (torch.searchsorted; the
              same search as cdb_shard_splits, which cdb_merge_sharded runs on the devices);
  2. counts : one all_to_all of the (family, run) row counts, then ONE host copy of the
              split table and the received counts (the step's only host synchronisation); the
              receive layout is cdb_shard_recv_plan's (the one plan both drivers use);
  3. rows   : one batch of point-to-point transfers (dist.batch_isend_irecv -> one RCCL
              group): per (peer, family, run) two contiguous slices -- hash column and records --
              in pieces of at most max_piece_bytes; this rank's own slices are device copies;
  4. merge  : the received slices are again runs in key-hash order (one per source run), so
              cdb_merge_device takes the sorted-run path (no partition pass) with
              key_shift = log2(N). Outputs stay sharded.
There is no other collective on the data path: merging is per key.
"""
from __future__ import annotations

import ctypes
import time
from typing import Sequence

from .runs import FAMILY_COLS, SIGN, sort_into_runs, wrap

OUT_COLS = (8, 6, 6)
REC_WORDS = tuple(c - 1 for c in FAMILY_COLS)  # record words per family (7 - 1, 6 - 1, 6 - 1)

# Largest single transfer. A 2.2 GB (2.2e9-byte, 2.75e8-element) RCCL transfer never completed
# on MI355X in round 1 while every transfer below 2^31 bytes did: the limit is a byte count
# crossing 2^31, so every slice moves in pieces of at most 1 GiB. Both sides of a transfer
# cut the same pieces from the same row count, so no collective is needed to agree on them.
MAX_PIECE_BYTES = 1 << 30


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


def _signed(u: int) -> int:
    u &= (1 << 64) - 1
    return u - (1 << 64) if u >= (1 << 63) else u


def owner_splits(kh, starts: Sequence[int], world: int):
    """kh: int64 tensor (key-hash bits) of one family whose rows form runs [starts[r],
    starts[r+1]), each ascending in unsigned order. Returns an int64 tensor [R, world + 1] of
    absolute row offsets: rows of run r owned by rank d are [s[r, d], s[r, d + 1])."""
    import torch
    b = owner_bits(world)
    R = len(starts) - 1
    out = torch.empty((R, world + 1), dtype=torch.int64, device=kh.device)
    bounds = torch.tensor([_signed((d << (64 - b)) ^ (1 << 63)) if b else _signed(1 << 63) for d in range(world)],
                          dtype=torch.int64, device=kh.device)
    for r in range(R):
        a, e = int(starts[r]), int(starts[r + 1])
        if e > a:
            out[r, :world] = torch.searchsorted(kh[a:e] ^ SIGN, bounds) + a
        else:
            out[r, :world] = a
        out[r, world] = e
    return out


def _pieces(a: int, e: int, piece_rows: int):
    while a < e:
        b = min(e, a + piece_rows)
        yield a, b
        a = b


class Plan:
    """Who sends what to whom in one step (host integers, from the one synchronised copy). The
    receive layout is cdb_shard_recv_plan's: one run per (source rank, source run) with rows, in
    (source, run) order."""

    def __init__(self, splits, recv, world: int, rank: int, n_runs: int):
        import constdb_amd as cdb
        self.world, self.rank, self.R = world, rank, n_runs
        self.splits = splits      # [3][R][world + 1] absolute offsets in this rank's rows
        self.recv = recv          # [world(src)][3][R] rows this rank receives
        cap = world * n_runs
        counts = (ctypes.c_uint64 * max(1, 3 * cap))(*[recv[s][f][r] for s in range(world) for f in range(3)
                                                      for r in range(n_runs)])
        nruns = (ctypes.c_uint32 * world)(*([n_runs] * world))
        k = ctypes.c_uint32()
        src = (ctypes.c_uint32 * max(1, cap))()
        run = (ctypes.c_uint32 * max(1, cap))()
        starts = (ctypes.c_uint64 * (3 * (cap + 1)))()
        tot = (ctypes.c_uint64 * 3)()
        st = cdb.lib().cdb_shard_recv_plan(world, nruns, counts, cap, ctypes.byref(k), src, run, starts, tot)
        if st != cdb.OK:
            raise RuntimeError(f"cdb_shard_recv_plan: status {st}")
        n = k.value
        self.runs = [(src[i], run[i]) for i in range(n)]   # receiver runs: (source rank, source run)
        self.run_start = [[starts[f * (cap + 1) + i] for i in range(n + 1)] for f in range(3)]
        self.total = [tot[f] for f in range(3)]
        self._index = {sr: i for i, sr in enumerate(self.runs)}

    def dest(self, f: int, r: int, s: int) -> int:
        """First receive-buffer row of source s's run r in family f."""
        return self.run_start[f][self._index[(s, r)]]


def make_plan(fams, starts, world: int, rank: int, device=None) -> Plan:
    """fams: this rank's three families as (hash [n], records [n, w]) tensor pairs, rows as runs;
    starts: three lists of R + 1 run offsets. One all_to_all of the counts, one host copy."""
    import torch
    import torch.distributed as dist
    R = len(starts[0]) - 1
    sp = torch.stack([owner_splits(fams[f][0], starts[f], world) for f in range(3)])  # [3, R, world+1]
    cnt = (sp[:, :, 1:] - sp[:, :, :-1]).permute(2, 0, 1).contiguous()             # [world(dst), 3, R]
    if device is not None:
        cnt = cnt.to(device)
    got = torch.empty_like(cnt)
    if world > 1:
        dist.all_to_all_single(got, cnt)
    else:
        got.copy_(cnt)
    host = torch.cat([sp.reshape(-1).to(got.device), got.reshape(-1)]).cpu().tolist()
    k = 3 * R * (world + 1)
    flat_sp, flat_got = host[:k], host[k:]
    splits = [[flat_sp[(f * R + r) * (world + 1):(f * R + r + 1) * (world + 1)] for r in range(R)] for f in range(3)]
    recv = [[flat_got[(s * 3 + f) * R:(s * 3 + f + 1) * R] for f in range(3)] for s in range(world)]
    return Plan(splits, recv, world, rank, R)


def exchange_runs(fams, plan: Plan, recv_bufs, max_piece_bytes: int = MAX_PIECE_BYTES) -> int:
    """Moves every owed slice into recv_bufs (three (hash [>= total], records [>= total, w]) tensor
    pairs on the same device as fams) at the plan's run offsets: per (peer, family, run) the hash
    slice and the record slice, each one contiguous range. One batch of point-to-point operations;
    own slices are local copies. Returns the number of point-to-point operations posted."""
    import torch.distributed as dist
    world, me = plan.world, plan.rank
    ops = []
    for peer in range(world):
        for f in range(3):
            for r in range(plan.R):
                # what I send to peer: my run r's slice owned by peer
                a, e = plan.splits[f][r][peer], plan.splits[f][r][peer + 1]
                # what I receive from peer: peer's run r's slice owned by me
                n_in = plan.recv[peer][f][r]
                d0 = plan.dest(f, r, peer) if n_in else 0
                for t, buf in zip(fams[f], recv_bufs[f]):
                    if peer == me:
                        if e > a:
                            buf[d0:d0 + (e - a)].copy_(t[a:e])
                        continue
                    src, dst = t[a:e].reshape(-1), buf[d0:d0 + n_in].reshape(-1)
                    piece = max(1, max_piece_bytes // t.element_size())
                    for x, y in _pieces(0, src.numel(), piece):
                        ops.append(dist.P2POp(dist.isend, src[x:y], peer))
                    for x, y in _pieces(0, dst.numel(), piece):
                        ops.append(dist.P2POp(dist.irecv, dst[x:y], peer))
    if ops:
        works = dist.batch_isend_irecv(ops)
        # RCCL: the same deadline as the library's exchange (shard.hip: 60 s + 1 ms per MB moved): a
        # peer that never posts its half ends the step with an error instead of a hang (gloo's
        # transfers progress inside wait(), under the process group's own timeout)
        moved = sum(op.tensor.numel() * op.tensor.element_size() for op in ops)
        # (polled every 0.1 ms for the exchange's expected length, then backing off to 5 ms: a slow
        # or stuck peer does not keep a host core spinning for the whole deadline)
        t0 = time.monotonic()
        deadline = t0 + 60.0 + moved / 1e9
        nap = 1e-4
        while dist.get_backend() == "nccl" and not all(w.is_completed() for w in works):
            now = time.monotonic()
            if now > deadline:
                raise TimeoutError(f"rank {me}: row exchange not complete after {60.0 + moved / 1e9:.0f} s "
                                   f"({len(ops)} point-to-point operations, {moved} bytes)")
            if now - t0 > 0.05 + moved / 50e9:
                nap = min(2 * nap, 5e-3)
            time.sleep(nap)
        for w in works:
            w.wait()
    return len(ops)


def recv_buffers(totals, device, pad: int = 2):
    """Receive buffers of the three families: (hash, records) tensor pairs for `totals` rows (plus
    `pad` rows: the merge may read up to the next 16 B past the last row)."""
    import torch
    return [(torch.empty(max(totals[f], 1) + pad, dtype=torch.int64, device=device),
             torch.empty((max(totals[f], 1) + pad, REC_WORDS[f]), dtype=torch.int64, device=device))
            for f in range(3)]


def _rows_from_tensor(cdb, t, n):
    """cdb_dev_rows view of a [ncols, cap] int64 CUDA tensor (first n rows of each column)."""
    r = cdb.DevRows()
    for c in range(t.shape[0]):
        r.col[c] = t[c].data_ptr()
    r.n = n
    return r


def _rows_from_records(cdb, pair, n):
    """cdb_dev_rows view (records layout) of a (hash [cap], records [cap, w]) tensor pair."""
    h, rec = pair
    r = cdb.DevRows()
    r.col[0] = h.data_ptr()
    for c in range(1, rec.shape[1] + 1):
        r.col[c] = rec.data_ptr() + 8 * (c - 1)
    r.n = n
    r.stride = rec.shape[1]
    return r


def _input_tensors(din):
    """The input families as (hash [n], records [n, w]) torch tensor pairs (copies, from either
    input layout; setup, outside any timed step)."""
    import torch
    out = []
    for rows, nc in zip((din.keys, din.nodes, din.members), FAMILY_COLS):
        n = rows.n
        if not n:
            out.append((torch.zeros(0, dtype=torch.int64, device="cuda"),
                        torch.zeros((0, nc - 1), dtype=torch.int64, device="cuda")))
        elif rows.stride > 1:
            out.append((wrap(rows.col[0], n).clone(), wrap(rows.col[1], n * (nc - 1)).view(n, nc - 1).clone()))
        else:
            out.append((wrap(rows.col[0], n).clone(),
                        torch.stack([wrap(rows.col[c], n) for c in range(1, nc)], dim=1).contiguous()))
    return out


def _merge_input(cdb, recv, plan: Plan, n_pos: int):
    d = cdb.DevInput()
    d.keys, d.nodes, d.members = (_rows_from_records(cdb, recv[f], plan.total[f]) for f in range(3))
    d.n_pos = n_pos
    if len(plan.runs) <= cdb.MAX_RUNS:
        d.n_runs = len(plan.runs)
        for f in range(3):
            for i, v in enumerate(plan.run_start[f]):
                d.run_start[f][i] = v
    return d


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
    cfg.flags |= cdb.GEN_ROWS_RECORDS
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
    din.n_pos = R
    sort_into_runs(din, R)  # setup: this rank's replica states as key-hash-ordered runs
    fams = _input_tensors(din)
    starts = [[din.run_start[f][r] for r in range(R + 1)] for f in range(3)]
    n_in = [din.keys.n, din.nodes.n, din.members.n]
    for fam in (din.keys, din.nodes, din.members):
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
    _log(rank, f"generated {n_in[0]} key rows as {R} runs")
    opts = cdb.MergeOpts()
    opts.key_shift = ob
    st = cdb.MergeStats()
    state = {}
    # One explicit stream for the whole step: torch orders it after each RCCL transfer, and
    # the library's kernels run on it too (the legacy default stream's handle is 0, which the
    # library would read as "use the context's own stream" -- unordered with the exchange).
    cs = torch.cuda.Stream(device=dev)

    def bufs(totals):
        b = state.get("recv")
        if b is None or any(b[f][0].shape[0] < totals[f] + 2 for f in range(3)):
            b = recv_buffers([t + t // 8 for t in totals], dev)
            state["recv"] = b
        return b

    ev = []  # per timed step: (start, exchanged) events on the step's stream

    def step(timed=False):
        with torch.cuda.stream(cs):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(cs)
            if world == 1:  # every row is this rank's own: the runs are the merge input as they lie
                d2 = cdb.DevInput()
                d2.keys, d2.nodes, d2.members = (_rows_from_records(cdb, fams[f], n_in[f]) for f in range(3))
                d2.n_pos = R
                d2.n_runs = R
                for f in range(3):
                    for r in range(R + 1):
                        d2.run_start[f][r] = starts[f][r]
                state["ops"], state["runs"] = 0, R
                state["sent"] = [0] * world
                total = n_in
            else:
                plan = make_plan(fams, starts, world, rank)
                recv = bufs(plan.total)
                state["ops"] = exchange_runs(fams, plan, recv)
                state["runs"] = len(plan.runs)
                state["sent"] = sent_bytes(plan, fams)
                d2 = _merge_input(cdb, recv, plan, R)
                total = plan.total
            if timed:
                e1.record(cs)
                ev.append((e0, e1))
            dout = cdb.DevOutput()
            dout.compact = 0  # the bucket layout (as the N = 1 line): rows stay in the rank's workspace
            stream = torch.cuda.current_stream().cuda_stream
            assert stream, "the merge must run on the exchange's (non-default) stream"
            ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(d2), ctypes.byref(opts), ctypes.byref(dout),
                                         ctypes.byref(st), ctypes.c_void_p(stream)))

    for i in range(args.warmup):
        step()
        _log(rank, f"warmup step {i} done ({state['ops']} p2p ops, {state['runs']} runs, "
                   f"sorted-run path {st.sorted_runs})")
    dev_ms = 0.0
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
        dev_ms += st.device_ms
    torch.cuda.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    xch_ms = sum(a.elapsed_time(b) for a, b in ev) / max(1, len(ev))
    B = alg_bytes(st)
    dm = dev_ms / args.steps
    sent = state["sent"]
    # max over ranks: step time, exchange time, merge time, largest per-link bytes; sums: rows, B_alg, bytes
    mx = torch.tensor([t1 - t0, xch_ms, dm, float(max(sent) if sent else 0)], dtype=torch.float64, device=dev)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = torch.tensor([float(n_in[0]), B, float(sum(sent))], dtype=torch.float64, device=dev)
    dist.all_reduce(sm)
    ms = mx[0].item() * 1e3 / args.steps
    xms, mms, link_max = mx[1].item(), mx[2].item(), mx[3].item()
    entries, B_tot, moved = int(sm[0].item()), sm[1].item(), sm[2].item()
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
        "data": "synthetic: seeded GenModel replica states generated in HBM (keys 'key:<i>'), "
                "each replica one key-hash-ordered run",
        "config": {"workload": f"C4 anti-entropy: {universe} keys x {R} replicas, replica r on rank r*N/R, "
                               f"owner = top log2(N) key-hash bits; every run's owner slice moves by RCCL "
                               f"point-to-point, merged on the sorted-run path",
                   "config": "c4", "replicas": R, "key_rows_in_total": entries,
                   "parallelism": f"key-hash sharding x{world}", "p2p_ops_per_step": state["ops"],
                   "merge_path": "sorted runs" if st.sorted_runs else "partition"},
        # the all-to-all replaced by point-to-point slices, reported apart from the merge
        "exchange": {"ms": xms, "bytes_moved_per_step": moved,
                     "max_link_bytes": link_max,
                     "max_link_GBps": link_max / (xms * 1e-3) / 1e9 if xms > 0 else None,
                     "link_peak_GBps": XGMI_LINK_GBPS,
                     "note": "ms = owner splits + count all_to_all + point-to-point transfers on the step's stream "
                             "(HIP events), max over ranks; link = one (source, destination) rank pair"},
        "merge_ms": mms,
        "roofline": {"bound": "hbm", "kernel": "merge pipeline of every rank (cdb_merge_device, HIP events); "
                                               "B_alg summed over ranks / slowest rank's merge time",
                     "achieved": B_tot / (mms * 1e-3) / 1e9, "peak": 8000.0 * world, "unit": "GB/s",
                     "frac": B_tot / (mms * 1e-3) / 1e9 / (8000.0 * world), "alg_bytes": B_tot,
                     "traffic": None,
                     "traffic_note": "PMC counters are collected on the 1-GPU line (profiles/), whose per-rank "
                                     "work is the same (weak scaling)"},
    }
    dist.barrier()
    dist.destroy_process_group()
    return res


XGMI_LINK_GBPS = 153.0  # one xGMI link, per direction (MI355X: 7 links per GPU)


def sent_bytes(plan: Plan, fams):
    """Bytes this rank sends to each peer in one step (its own slices excluded)."""
    out = [0] * plan.world
    for peer in range(plan.world):
        if peer == plan.rank:
            continue
        for f in range(3):
            nc = 1 + fams[f][1].shape[1]  # the hash word + the record
            for r in range(plan.R):
                out[peer] += (plan.splits[f][r][peer + 1] - plan.splits[f][r][peer]) * nc * 8
    return out


def sharded_merge(cdb, ctx, din, n_pos: int, stream=None, max_piece_bytes: int = MAX_PIECE_BYTES):
    """One sharded merge step outside the bench's timing harness: this rank's rows as runs
    (sorted here when din carries none), the owner slices exchanged (RCCL on GPU tensors; gloo
    through host copies), the received runs merged with key_shift = log2(N). Returns ([keys,
    nodes, members] output column tensors, MergeStats, Plan). Used by the multi-process tests."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    ob = owner_bits(world)
    L = cdb.lib()
    dev = torch.device("cuda", torch.cuda.current_device())
    on_host = dist.get_backend() == "gloo"
    din.n_pos = n_pos
    if din.n_runs == 0:
        sort_into_runs(din, n_pos)
    R = din.n_runs
    starts = [[din.run_start[f][r] for r in range(R + 1)] for f in range(3)]
    fams = _input_tensors(din)
    if on_host:
        fams = [(h.cpu(), r.cpu()) for h, r in fams]
    plan = make_plan(fams, starts, world, rank)
    recv = recv_buffers(plan.total, fams[0][0].device)
    exchange_runs(fams, plan, recv, max_piece_bytes)
    recv = [(h.to(dev), r.to(dev)) for h, r in recv]
    torch.cuda.synchronize()
    d2 = _merge_input(cdb, recv, plan, n_pos)
    dout = cdb.DevOutput()
    outs = [torch.empty((OUT_COLS[f], max(plan.total[f], 1)), dtype=torch.int64, device=dev) for f in range(3)]
    dout.keys, dout.nodes, dout.members = (_rows_from_tensor(cdb, t, 0) for t in outs)
    dout.compact = 1
    opts = cdb.MergeOpts()
    opts.key_shift = ob
    st = cdb.MergeStats()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(d2), ctypes.byref(opts), ctypes.byref(dout),
                                 ctypes.byref(st), stream))
    torch.cuda.synchronize()
    return [outs[0][:, :dout.keys.n], outs[1][:, :dout.nodes.n], outs[2][:, :dout.members.n]], st, plan
