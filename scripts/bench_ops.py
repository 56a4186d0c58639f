"""Op-stream apply bench: a C1-shaped merged state on one GPU, then a replicate
stream of N commands applied in one cdb_apply_ops call. Prints one JSON line: host decode rate,
device apply rate (HIP events around the device pipeline; H2D/D2H excluded) and, with
--cpu-sample, the oracle's rate on a bounded sample (Python restatement, 1 core)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import torch  # noqa: E402,F401  -- one HIP runtime per process

import constdb_amd as cdb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--universe", type=int, default=2_000_000)
    ap.add_argument("--ops", type=int, default=4_000_000)
    ap.add_argument("--zipf", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=0)
    a = ap.parse_args()
    cfg = cdb.gen_config(seed=1, universe=a.universe, n_replicas=2)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(2)]
    ctx = cdb.Context(0)
    db = cdb.DB(ctx)
    state = db.merge_snapshots(snaps)
    stream = cdb.gen_ops(cfg, a.ops, 0, a.zipf)
    t = time.perf_counter()
    ops = cdb.decode_ops(stream, 0)
    dec_s = time.perf_counter() - t
    info = ops.info()
    # the same decode with the per-message work on the GPU (cdb_decode_ops_gpu), best of reps
    gdec, gtm = None, None
    for _ in range(a.reps):
        tm = {}
        t = time.perf_counter()
        gops = cdb.decode_ops_gpu(ctx, stream, 0, timing=tm)
        dt = time.perf_counter() - t
        if gdec is None or dt < gdec:
            gdec, gtm = dt, tm
        del gops
    best, st = None, None
    for _ in range(a.reps):
        t = time.perf_counter()
        m = state.apply_ops(ops)
        wall = time.perf_counter() - t
        st = m.apply_stats
        best = st.device_ms if best is None else min(best, st.device_ms)
        del m
    out = {"metric": "op-stream apply: replicate commands/s", "ops": info.n_ops,
           "node_args": info.n_node_args, "member_args": info.n_member_args,
           "state_key_rows": st.key_rows_in, "zipf_milli": a.zipf,
           "device_ms": best, "device_ops_per_s": info.n_ops / (best / 1e3),
           "call_wall_ms": wall * 1e3, "host_decode_ms": dec_s * 1e3,
           "host_decode_msgs_per_s": info.n_messages / dec_s, "stream_mb": len(stream) / 1e6,
           "gpu_decode_ms": gdec * 1e3, "gpu_decode_msgs_per_s": info.n_messages / gdec,
           "gpu_decode_host_part_ms": gtm["host_ms"], "gpu_decode_used_gpu": gtm["used_gpu"],
           "type_errors": st.type_errors, "key_rows_out": st.key_rows_out}
    if a.cpu_sample:
        import constdb_oracle as o
        import constdb_ops_oracle as oo
        scfg = cdb.gen_config(seed=1, universe=max(1000, a.cpu_sample // 4), n_replicas=2)
        odb = o.fold_snapshots([cdb.gen_snapshot(scfg, r) for r in range(2)])
        s = cdb.gen_ops(scfg, a.cpu_sample, 0, a.zipf)
        t = time.perf_counter()
        oo.apply_replicates(odb, s, 0)
        dt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": a.cpu_sample / dt, "unit": "commands/s", "cores": 1, "kind": "port",
                               "sample": f"{a.cpu_sample} commands over a {scfg.universe}-key state, Python oracle"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
