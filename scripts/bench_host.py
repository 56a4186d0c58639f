"""Host-boundary merge bench: the rate a caller of the host-level ABI sees.

R seeded snapshots (cdb_gen_snapshot) are decoded on the host (cdb_decode_snapshot), then
merged with cdb_merge, which uploads the batches over PCIe, runs the merge pipeline and
downloads the result into host memory. Prints one JSON line with entries/s for the device
pipeline alone (HIP events), for the whole cdb_merge call (PCIe-inclusive) and for
decode + merge (snapshots decoded one after another, or one thread per snapshot). Input key
rows (data + expires + deletes) are the entries, as in bench.py."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402,F401  -- one HIP runtime per process

import constdb_amd as cdb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--universe", type=int, default=8_000_000)
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--decode-threads", type=int, default=8)
    a = ap.parse_args()
    cfg = cdb.gen_config(seed=4, universe=a.universe, n_replicas=a.replicas, replica_hi=a.replicas)
    t = time.perf_counter()
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(a.replicas)]
    print(f"generated {sum(map(len, snaps)) / 1e6:.1f} MB in {time.perf_counter() - t:.1f} s", file=sys.stderr)
    t = time.perf_counter()
    batches = [cdb.decode_snapshot(s) for s in snaps]
    decode_s = time.perf_counter() - t
    # the snapshots are independent: one host thread per snapshot (ctypes drops the GIL)
    t = time.perf_counter()
    with ThreadPoolExecutor(max_workers=min(a.replicas, a.decode_threads)) as ex:
        batches = list(ex.map(cdb.decode_snapshot, snaps))
    decode_par_s = time.perf_counter() - t
    db = cdb.DB(cdb.Context(0))
    db.merge_batches(batches)  # warm-up: allocations, code objects
    best = None
    for _ in range(a.reps):
        t = time.perf_counter()
        m = db.merge_batches(batches)
        wall = time.perf_counter() - t
        if best is None or wall < best[0]:
            best = (wall, m.stats)
        del m
    wall, st = best
    entries = st.key_rows_in
    out = {"metric": "merged CRDT entries/sec at the host boundary (cdb_merge)", "universe": a.universe,
           "replicas": a.replicas, "snapshot_bytes": sum(map(len, snaps)), "key_rows_in": entries,
           "node_rows_in": st.node_rows_in, "member_rows_in": st.member_rows_in,
           "key_rows_out": st.key_rows_out, "device_ms": st.device_ms, "merge_call_ms": wall * 1e3,
           "host_decode_ms": decode_s * 1e3, "host_decode_parallel_ms": decode_par_s * 1e3,
           "decode_threads": min(a.replicas, a.decode_threads),
           "entries_per_s_device": entries / (st.device_ms / 1e3),
           "entries_per_s_merge_call": entries / wall,
           "entries_per_s_decode_plus_merge": entries / (wall + decode_s),
           "entries_per_s_parallel_decode_plus_merge": entries / (wall + decode_par_s)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
