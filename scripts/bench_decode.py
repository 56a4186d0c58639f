"""Snapshot decode bench: one seeded replica snapshot decoded by the host decoder
(cdb_decode_snapshot) and by the GPU path (cdb_decode_snapshot_gpu: host entry index, HIP
count/emit kernels, staged download into the host batch); then R replica snapshots (generator
order: the reference's unordered HashMap layout, sorted into runs on the device) decoded straight
into HBM, with the library's phase clock (CDB_DECODE_TRACE), and that decode followed by the
cdb_merge_device of its rows (bucket layout) beside the merge alone. Prints one JSON line, best of
--reps."""
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
    ap.add_argument("--device-snapshots", type=int, default=8,
                    help="replica snapshots decoded straight into HBM (0: skip)")
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
    # decode -> merge handoff: R snapshots straight into HBM (cdb_decode_snapshots_device)
    # against host decode + cdb_upload_batches of the same snapshots
    import ctypes
    from constdb_amd.runs import FAMILY_COLS  # noqa: F401
    R = a.device_snapshots
    if R:
        snaps = [snap] + [cdb.gen_snapshot(cfg, r) for r in range(1, R)]
        L = cdb.lib()

        def release(din):
            for fam in (din.keys, din.nodes, din.members):
                L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
        import tempfile
        trace = os.path.join(tempfile.mkdtemp(), "decode_trace.jsonl")
        os.environ["CDB_DECODE_TRACE"] = trace

        def merge(din):
            dout = cdb.DevOutput()
            dout.compact = 0
            opts = cdb.merge_opts()
            st = cdb.MergeStats()
            torch.cuda.synchronize()
            t = time.perf_counter()
            ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(dout),
                                         ctypes.byref(st), None))
            torch.cuda.synchronize()
            return time.perf_counter() - t, st
        bs, din = cdb.decode_snapshots_device(ctx, snaps, records=True)  # warm-up
        merge(din)
        release(din)
        del bs
        dev = up = mrg = None
        for _ in range(a.reps):
            tm = {}
            t = time.perf_counter()
            bs, din = cdb.decode_snapshots_device(ctx, snaps, timing=tm, records=True)
            dt = time.perf_counter() - t
            with open(trace) as f:
                phases = json.loads(f.read().strip().split("\n")[-1])
            mt, mst = merge(din)
            if dev is None or dt < dev[0]:
                dev = (dt, tm, phases, din.n_runs)
            mrg = (mt, mst) if mrg is None or mt < mrg[0] else mrg
            release(din)
            del bs
            t = time.perf_counter()
            hb = [cdb.decode_snapshot(x) for x in snaps]
            din = cdb.DevInput()
            arr = (ctypes.c_void_p * R)(*[b.handle for b in hb])
            ctx.check(L.cdb_upload_batches(ctx.handle, arr, R, ctypes.byref(din)))
            dt = time.perf_counter() - t
            up = dt if up is None else min(up, dt)
            release(din)
            del hb
        nbytes = sum(len(x) for x in snaps)
        out["device_resident"] = {"snapshots": R, "bytes": nbytes, "layout": "records", "runs": dev[3],
                                  "decode_to_hbm_ms": dev[0] * 1e3, "index_ms": dev[1]["index_ms"],
                                  "device_ms": dev[1]["device_ms"], "phases": dev[2],
                                  "effective_gbs": nbytes / dev[0] / 1e9,
                                  "host_decode_plus_upload_ms": up * 1e3}
        out["decode_plus_merge"] = {"decode_ms": dev[0] * 1e3, "merge_ms": mrg[0] * 1e3,
                                    "total_ms": (dev[0] + mrg[0]) * 1e3,
                                    "total_over_merge": (dev[0] + mrg[0]) / mrg[0],
                                    "sorted_runs": mrg[1].sorted_runs, "key_rows_out": mrg[1].key_rows_out}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
