#!/usr/bin/env python3
"""Benchmark: ConstDB snapshot merge on MI355X (BASELINE.json metric:
"merged CRDT entries/sec + achieved HBM GB/s, snapshot merge at 1/2/4/8 GPUs").

One step = one full merge of R=8 replica snapshots already resident in HBM as columnar
rows (anti-entropy): bucket partition -> fused bucket merge ->
dense compaction, i.e. everything DB::merge_entry/Object::merge would do for those
entries. Weak scaling: every GPU owns a fixed 1/8-of-C4 key universe (62.5M keys); at
N=8 the job is exactly C4 (500M keys x 8 replicas). For N>1 replica r lives on GPU
r*N/8 and rows are routed to the GPU owning their key hash by an RCCL all-to-all
(torch.distributed "nccl" backend) inside the timed step.

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# SURVEY.md §8d algorithmic row widths (bytes): compulsory read + write per row
W_KEY, W_NODE, W_SET, W_DICT = 50, 33, 34, 42
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--universe-per-gpu", type=int, default=62_500_000)
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--cpu-universe", type=int, default=1_000_000,
                    help="key universe of the bounded CPU-baseline sample (same generator config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the multi-GPU (RCCL all-to-all) path even when WORLD_SIZE == 1")
    return ap.parse_args()


def c4_config(cdb, universe, replicas, seed, lo, hi, shard=0, n_shards=1):
    # C4: type mix 60/30/5/5, counters 1-8 nodes (mean 2), sets/dicts mean 4 members,
    # 0.1 % cross-replica type conflicts, ~2 % forced time ties, p(key in replica) = 0.5
    return cdb.gen_config(seed=seed, universe=universe, n_replicas=replicas, key_permille=500,
                          mix_bytes=60, mix_counter=30, mix_set=5, mix_dict=5, conflict_ppm=1000,
                          tie_permille=20, max_nodes=8, mean_members=4, member_universe=16,
                          del_permille=200, side_permille=20, value_min=8, value_max=32,
                          shard=shard, n_shards=n_shards, replica_lo=lo, replica_hi=hi)


def alg_bytes(st, set_frac=0.5):
    """Compulsory bytes of one merge: inputs + outputs at the survey's row
    widths. Member rows are priced half set (34 B) half dict (42 B) as in C4's 5/5 mix."""
    wm = set_frac * W_SET + (1 - set_frac) * W_DICT
    return ((st.key_rows_in + st.key_rows_out) * W_KEY + (st.node_rows_in + st.node_rows_out) * W_NODE
            + (st.member_rows_in + st.member_rows_out) * wm)


def pmc_traffic():
    """HBM bytes per launch of the bucket phase, from the committed rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this same bench command (scripts/gpu_round.sh -> pmc_traffic.py);
    None when no such measurement is committed."""
    f = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
    try:
        with open(f) as fh:
            return float(json.load(fh)["bucket_phase_bytes"])
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(cdb, args):
    """The oracle's single-thread C++ fold (kind "port": the Rust reference cannot be built
    here) on a bounded sample of the same generator config; decode is excluded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cdb_oracle
    cfg = c4_config(cdb, args.cpu_universe, args.replicas, args.seed, 0, args.replicas)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(args.replicas)]
    ns, entries = cdb_oracle.time_fold(snaps, reps=2)
    return {"value": entries / (ns * 1e-9), "unit": "entries/s", "cores": 1, "kind": "port",
            "sample": f"C4 generator config, {args.cpu_universe} keys x {args.replicas} replicas "
                      f"({entries} entries, decode excluded, best of 2), oracle/cdb_oracle.cpp "
                      f"std::unordered_map fold",
            "host_cpus": os.cpu_count()}


def main():
    args = parse()
    # RCCL and the HIP runtime may print banners on the C-level stdout: keep fd 1 for the
    # single JSON line and send everything else to stderr.
    json_fd = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(os.dup(2), "w")
    import constdb_amd as cdb
    from constdb_amd import build as b
    b.build()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1 or args.force_dist:
        from constdb_amd import dist
        res = dist.run_bench(cdb, args, rank, world, local_rank, c4_config, alg_bytes)
    else:
        res = run_single(cdb, args)
    if rank != 0:
        os.close(json_fd)
        return
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(cdb, args)
    with os.fdopen(json_fd, "w") as out:
        out.write(json.dumps(res) + "\n")


def run_single(cdb, args):
    ctx = cdb.Context(0)
    L = cdb.lib()
    cfg = c4_config(cdb, args.universe_per_gpu, args.replicas, args.seed, 0, args.replicas)
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
    dout = cdb.DevOutput()
    ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(dout.keys), din.keys.n, 8))
    ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(dout.nodes), din.nodes.n, 6))
    ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(dout.members), din.members.n, 6))
    dout.compact = 1
    opts = cdb.MergeOpts()
    st = cdb.MergeStats()

    def step():
        ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(dout),
                                     ctypes.byref(st), None))

    for _ in range(args.warmup):
        step()
    bucket_ms = part_ms = fin_ms = dev_ms = 0.0
    t0 = time.perf_counter()  # cdb_merge_device synchronises its stream before returning
    for _ in range(args.steps):
        step()
        bucket_ms += st.bucket_ms
        part_ms += st.partition_ms
        fin_ms += st.finish_ms
        dev_ms += st.device_ms
    t1 = time.perf_counter()
    ms = (t1 - t0) * 1e3 / args.steps
    entries = st.key_rows_in
    B = alg_bytes(st)
    bk = bucket_ms / args.steps
    res = {
        "metric": "merged CRDT entries/sec (snapshot merge)",
        "value": entries / (ms * 1e-3),
        "unit": "entries/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: seeded GenModel replica states generated in HBM (keys 'key:<i>')",
        "config": {"workload": f"C4 anti-entropy shard: {args.universe_per_gpu} keys/GPU x {args.replicas} "
                               f"replicas (N=8 -> exactly C4's 500M keys)",
                   "replicas": args.replicas, "key_rows_in": st.key_rows_in, "node_rows_in": st.node_rows_in,
                   "member_rows_in": st.member_rows_in, "key_rows_out": st.key_rows_out,
                   "parallelism": "single GPU"},
        "hbm_gbs_alg": B / (ms * 1e-3) / 1e9,
        "phases_ms": {"partition": part_ms / args.steps, "bucket_merge": bk, "finish": fin_ms / args.steps,
                      "device_total": dev_ms / args.steps},
        "roofline": {"bound": "hbm",
                     "kernel": "bucket phase = bucket_wave_kernel + bucket_wide_kernel + bucket_mid_kernel",
                     "achieved": B / (bk * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": B / (bk * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "alg_bytes": B, "traffic": pmc_traffic()},
        "stats": {"type_conflicts": st.type_conflicts, "dict_merges": st.dict_merges,
                  "hot_buckets": st.hot_buckets, "wide_buckets": st.wide_buckets,
                  "mid_buckets": st.mid_buckets, "orphans": st.orphan_children},
    }
    for fam in (dout.keys, dout.nodes, dout.members, din.keys, din.nodes, din.members):
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
    return res


if __name__ == "__main__":
    main()
