"""Sorted runs on the host side of the C-ABI (setup helpers, torch on device columns).

A replica state this engine produced -- a merge result, or a snapshot encoded from one --
holds its rows in key-hash order. Grouping a batch's rows into runs ordered by key hash lets
cdb_merge_device take the sorted-run path (runs.hip.h: run directories, no partition pass), and
lets the multi-GPU exchange (dist.py) send each owner its rows as contiguous slices of every run.

Two layouts:
  * one run per fold position (every key row of a replica in one hash-ordered run): what a merge
    result kept in HBM as the next merge's position 0 is (cdb_dev_state_rows);
  * three key runs per fold position -- DATAS, EXPIRES, DELETES, each hash-ordered -- and one
    child run (padded with two empty runs): the sections of a snapshot this engine encoded as
    they lie in the stream (cdb_decode_snapshots_device merges them back into one run per
    snapshot on decode; this layout exercises runs of very different lengths).
These helpers establish a layout for generated inputs; they are setup, never part of a timed
merge step.
"""
from __future__ import annotations

SIGN = -(1 << 63)           # xor: unsigned 64-bit order as signed int64 order
FAMILY_COLS = (7, 6, 6)     # key rows, counter nodes, set/dict members (cdb_merge.h)


def wrap(ptr: int, n: int):
    """A torch int64 view of n words at device address ptr (memory owned by the library)."""
    import torch

    class _Cai:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 2}
    return torch.as_tensor(_Cai(), device="cuda")


def run_order(kh, meta, sections: bool = False, key_family: bool = False):
    """Permutation ordering rows by (fold position, [section,] unsigned key hash), stable, and the
    run index of every row (pos, or 3 pos + section with `sections`). kh / meta: int64 tensors of
    one family; key_family: meta's tag gives the section (data / expires / deletes)."""
    import torch
    o = torch.sort(kh ^ SIGN, stable=True).indices
    pos = (meta >> 48) & 0xFF
    if sections:
        sec = torch.zeros_like(pos)
        if key_family:
            tag = (meta >> 56) & 0xFF
            sec = torch.where(tag == 6, 1, torch.where(tag == 7, 2, 0))
        run = 3 * pos + sec
    else:
        run = pos
    o = o[torch.sort(run[o], stable=True).indices]
    return o, run


def sort_into_runs(din, n_runs: int | None = None, sections: bool = False) -> None:
    """Reorders every family's device rows of a cdb_dev_input in place into runs -- one per fold
    position, or with `sections` three per position (see the module doc) -- and records them in
    din.n_runs / din.run_start."""
    import torch
    R = din.n_pos if n_runs is None else n_runs
    if sections:
        R = 3 * din.n_pos
    din.n_runs = R
    for f, (rows, ncol) in enumerate(zip((din.keys, din.nodes, din.members), FAMILY_COLS)):
        n = rows.n
        if n == 0:
            for r in range(R + 1):
                din.run_start[f][r] = 0
            continue
        kh = wrap(rows.col[0], n)
        if rows.stride > 1:  # records layout: the hash column + one record of `stride` words per row
            rec = wrap(rows.col[1], n * rows.stride).view(n, rows.stride)
            meta = rec[:, rows.stride - 1].contiguous()
        else:
            rec = None
            meta = wrap(rows.col[ncol - 1], n)
        o, run = run_order(kh, meta, sections, key_family=(f == 0))
        counts = torch.bincount(run, minlength=R).tolist()
        del run, meta
        if rec is not None:
            kh.copy_(kh[o])
            rec.copy_(rec[o])
        else:
            for c in range(ncol):
                col = wrap(rows.col[c], n)
                col.copy_(col[o])
        del o
        st = 0
        for r in range(R):
            din.run_start[f][r] = st
            st += counts[r]
        din.run_start[f][R] = st
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def to_records(cdb, ctx, din) -> None:
    """Setup helper: moves every family of a cdb_dev_input from plain columns into the records layout
    (cdb_dev_rows_alloc_records; the column memory is released)."""
    import ctypes
    import torch
    L = cdb.lib()
    for f, (name, ncol) in enumerate(zip(("keys", "nodes", "members"), FAMILY_COLS)):
        rows = getattr(din, name)
        if rows.stride > 1:
            continue
        n = rows.n
        rec = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc_records(ctx.handle, ctypes.byref(rec), n, ncol))
        if n:
            wrap(rec.col[0], n).copy_(wrap(rows.col[0], n))
            r = wrap(rec.col[1], n * (ncol - 1)).view(n, ncol - 1)
            for c in range(1, ncol):
                r[:, c - 1].copy_(wrap(rows.col[c], n))
            torch.cuda.synchronize()
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(rows))
        setattr(din, name, rec)


def _run_view(cdb, rows, a: int, n: int):
    """cdb_dev_rows of rows [a, a + n) of `rows` (plain columns or the records layout)."""
    v = cdb.DevRows()
    v.n, v.stride, v.stride0 = n, rows.stride, rows.stride0
    for c in range(8):
        if rows.col[c]:
            step = (rows.stride0 if c == 0 else rows.stride) or 1
            v.col[c] = rows.col[c] + 8 * a * step
    return v


def state_runs(cdb, ctx, din, opts=None) -> None:
    """Setup helper: replaces every replica's rows by that replica's state as this engine keeps it --
    its rows merged alone (cdb_merge_device, bucket layout) and read back as position-0 rows
    (cdb_dev_state_rows), moved to the replica's fold position (cdb_dev_input_append). That is what
    a node holding merge results has: one key-hash-ordered run per replica whose children follow
    every merge tier's child order (common.h child_order), so the chip-wide path merges those runs
    instead of sorting them. The replicas' content is unchanged (a single-replica merge folds
    nothing). din must be in the records layout; its rows are released and replaced."""
    import ctypes
    L = cdb.lib()
    names = ("keys", "nodes", "members")
    sort_into_runs(din)
    R = din.n_runs
    mopts = opts if opts is not None else cdb.MergeOpts()
    dst = cdb.DevInput()
    for name, ncol in zip(names, FAMILY_COLS):
        r = cdb.DevRows()
        ctx.check(L.cdb_dev_rows_alloc_records(ctx.handle, ctypes.byref(r), max(getattr(din, name).n, 1), ncol))
        r.n = 0
        setattr(dst, name, r)
    for rep in range(R):
        one = cdb.DevInput()
        for f, name in enumerate(names):
            a, b = din.run_start[f][rep], din.run_start[f][rep + 1]
            setattr(one, name, _run_view(cdb, getattr(din, name), a, b - a))
            one.run_start[f][0], one.run_start[f][1] = 0, b - a
        one.n_pos, one.n_runs = rep + 1, 1
        out = cdb.DevOutput()
        out.compact = 0
        st = cdb.MergeStats()
        ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(one), ctypes.byref(mopts), ctypes.byref(out),
                                     ctypes.byref(st), None))
        sdin = cdb.DevInput()
        for name, ncol in zip(names, FAMILY_COLS):
            r = cdb.DevRows()
            ctx.check(L.cdb_dev_rows_alloc_records(ctx.handle, ctypes.byref(r), max(getattr(out, name).n, 1), ncol))
            setattr(sdin, name, r)
        ctx.check(L.cdb_dev_state_rows(ctx.handle, ctypes.byref(out), ctypes.byref(sdin.keys),
                                       ctypes.byref(sdin.nodes), ctypes.byref(sdin.members), None))
        sdin.n_pos, sdin.n_runs = 1, 1
        for f, name in enumerate(names):
            sdin.run_start[f][0], sdin.run_start[f][1] = 0, getattr(sdin, name).n
        if rep == 0:
            dst.n_runs = 0  # (the first append sets the runs: dst has no rows yet)
        ctx.check(L.cdb_dev_input_append(ctx.handle, ctypes.byref(dst), ctypes.byref(sdin), rep, None))
        if rep == 0:  # an empty dst is not "in runs": the first state becomes run 0 explicitly
            dst.n_runs = 1
            for f, name in enumerate(names):
                dst.run_start[f][0], dst.run_start[f][1] = 0, getattr(dst, name).n
        for name in names:
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(sdin, name)))
    for name in names:
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(getattr(din, name)))
    ctypes.memmove(ctypes.byref(din), ctypes.byref(dst), ctypes.sizeof(din))
