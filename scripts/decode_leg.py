"""The C4 shard's decode leg alone (bench.py's decode_leg): the 8 replicas' snapshots (62.5M-key
universe, ~2 GB each, the reference's HashMap order) decoded straight into HBM as records by
cdb_decode_snapshots_device, --reps times, each with the library's phase clock (CDB_DECODE_TRACE).
Prints one JSON line per rep. Run under rocprofv3 --kernel-trace --memory-copy-trace for the
timeline (scripts/dec_timeline.py)."""
import argparse
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402,F401  -- one HIP runtime per process

import constdb_amd as cdb  # noqa: E402
from constdb_amd import configs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--universe", type=int, default=62_500_000)
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    cfg = configs.c4(cdb, a.universe, a.replicas)
    with ThreadPoolExecutor(min(a.replicas, 16)) as ex:
        snaps = list(ex.map(lambda r: cdb.gen_snapshot(cfg, r), range(a.replicas)))
    nbytes = sum(len(s) for s in snaps)
    ctx = cdb.Context(0)
    L = cdb.lib()
    import ctypes
    for rep in range(a.reps):
        trace = os.path.join(tempfile.mkdtemp(), "trace.jsonl")
        os.environ["CDB_DECODE_TRACE"] = trace
        t = time.perf_counter()
        batches, din = cdb.decode_snapshots_device(ctx, snaps, records=True)
        ms = (time.perf_counter() - t) * 1e3
        del os.environ["CDB_DECODE_TRACE"]
        with open(trace) as fh:
            phases = json.loads(fh.read().strip().split("\n")[-1])
        for fam in (din.keys, din.nodes, din.members):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
        del batches
        print(json.dumps({"rep": rep, "bytes": nbytes, "decode_ms": ms, "pcie_floor_ms": nbytes / 56e9 * 1e3,
                          "runs": din.n_runs, "phases": phases}), flush=True)
        time.sleep(0.5)  # (a gap in the trace between reps)


if __name__ == "__main__":
    main()
