"""Snapshot decode bench: one seeded replica snapshot decoded by the host decoder
(cdb_decode_snapshot) and by the GPU path (cdb_decode_snapshot_gpu: host entry index, HIP
count/emit kernels, staged download into the host batch). Prints one JSON line, best of --reps."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402,F401  -- one HIP runtime per process

import constdb_amd as cdb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--universe", type=int, default=8_000_000)
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    cfg = cdb.gen_config(seed=4, universe=a.universe, n_replicas=a.replicas, replica_hi=a.replicas)
    snap = cdb.gen_snapshot(cfg, 0)
    ctx = cdb.Context(0)
    cdb.decode_snapshot_gpu(ctx, snap)  # warm-up
    host = gpu = None
    for _ in range(a.reps):
        t = time.perf_counter()
        b = cdb.decode_snapshot(snap)
        dt = time.perf_counter() - t
        host = dt if host is None else min(host, dt)
        info = b.info()
        del b
        tm = {}
        t = time.perf_counter()
        b = cdb.decode_snapshot_gpu(ctx, snap, timing=tm)
        dt = time.perf_counter() - t
        if gpu is None or dt < gpu[0]:
            gpu = (dt, tm)
        del b
    out = {"metric": "snapshot decode: bytes/s", "universe": a.universe, "snapshot_bytes": len(snap),
           "key_rows": info.n_data + info.n_expires + info.n_deletes, "node_rows": info.n_nodes, "member_rows": info.n_members,
           "host_ms": host * 1e3, "gpu_call_ms": gpu[0] * 1e3, "gpu_index_ms": gpu[1]["index_ms"],
           "gpu_device_ms": gpu[1]["device_ms"], "host_mb_s": len(snap) / host / 1e6,
           "gpu_mb_s": len(snap) / gpu[0] / 1e6}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
