"""Sorted runs on the host side of the C-ABI (setup helpers, torch on device columns).

A replica state this engine produced -- a merge result, or a snapshot encoded from one --
holds its rows in key-hash order. Grouping a batch's rows into one such run per fold position
(replica) lets cdb_merge_device take the sorted-run path (runs.hip.h: run directories, no
partition pass), and lets the multi-GPU exchange (dist.py) send each owner its rows as
contiguous slices of every run. These helpers establish that layout for generated inputs;
they are setup, never part of a timed merge step.
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


def run_order(kh, meta):
    """Permutation ordering rows by (fold position, unsigned key hash), stable; and the row
    count of every position. kh / meta: int64 tensors of one family."""
    import torch
    o = torch.sort(kh ^ SIGN, stable=True).indices
    pos = (meta >> 48) & 0xFF
    o = o[torch.sort(pos[o], stable=True).indices]
    return o, pos


def sort_into_runs(din, n_runs: int | None = None) -> None:
    """Reorders every family's device rows of a cdb_dev_input by (fold position, key hash) in
    place -- one run per position -- and records the runs in din.n_runs / din.run_start."""
    import torch
    R = din.n_pos if n_runs is None else n_runs
    din.n_runs = R
    for f, (rows, ncol) in enumerate(zip((din.keys, din.nodes, din.members), FAMILY_COLS)):
        n = rows.n
        if n == 0:
            for r in range(R + 1):
                din.run_start[f][r] = 0
            continue
        kh = wrap(rows.col[0], n)
        meta = wrap(rows.col[ncol - 1], n)
        o, pos = run_order(kh, meta)
        counts = torch.bincount(pos, minlength=R).tolist()
        del pos
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
