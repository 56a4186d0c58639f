#!/usr/bin/env python3
"""Benchmark: ConstDB snapshot merge on MI355X (BASELINE.json metric:
"merged CRDT entries/sec + achieved HBM GB/s, snapshot merge at 1/2/4/8 GPUs").

One step = one full merge of R replica states already resident in HBM (cdb_merge_device): the
run directories of the key-hash-ordered runs, the fused bucket merge into the bucket layout (the
result every consumer reads; --output dense adds the compaction into dense columns), i.e.
everything DB::merge_entry / Object::merge / DB::delete / DB::expire_at (and DB::gc for C3) would
do for those entries. Configs (constdb_amd/configs.py):
  c4 (default)  8-replica anti-entropy. Weak scaling: every GPU owns a 62.5M-key universe; at
                N=8 the job is exactly C4 (500M keys x 8 replicas). For N>1 replica r lives on
                GPU r*N/8 and rows go to the GPU owning their key hash inside the timed step:
                by default in ONE process over a multi-device context (cdb_merge_sharded: owner
                splits, RCCL point-to-point inside the library, per-device merges -- the C-ABI
                path INTEGRATION.md §5 gives the reference's one server process); under a
                launcher (torch.distributed.run, WORLD_SIZE=N) rank 0 drives every GPU that way
                and the other ranks only join the barriers. --dist: one process per GPU instead
                (constdb_amd/dist.py, torch.distributed "nccl" point-to-point).
  c1            2-node MEET, 1M Bytes + 1M counters per node, 50 % overlap (C1/C2).
  c3            4 replicas built by replaying 10M sadd/srem/hset/hdel each, merge + DB::gc.
  c5            Zipf hot keys: 10M keys, 80M node/member rows over 8 replicas.

Prints ONE JSON line (rank 0) per config run.
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
# committed measurements, newest round first (a config not yet re-measured keeps its older record)
PROFILE_DIRS = [os.path.join(ROOT, "profiles", r) for r in ("r06", "r05")]


def profile_file(name):
    for d in PROFILE_DIRS:
        f = os.path.join(d, name)
        if os.path.exists(f):
            return f
    return os.path.join(PROFILE_DIRS[0], name)
# the merge pipeline's kernels (everything cdb_merge_device launches; not the generator)
MERGE_KERNEL_PREFIXES = ("part_", "bucket_", "compact", "scan_", "stats_reduce", "gc_lastbad", "set_dir",
                         "stamp_pos", "iota", "hot_", "sorted_", "seg_", "run_", "mat_", "radix_hist",
                         "radix_scatter")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=["c1", "c3", "c4", "c5"])
    ap.add_argument("--universe-per-gpu", type=int, default=62_500_000)
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--cpu-universe", type=int, default=10_000_000,
                    help="key universe of the bounded C4 CPU-baseline sample (same generator config)")
    ap.add_argument("--cpu-reps", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the multi-GPU (RCCL all-to-all) path even when WORLD_SIZE == 1")
    ap.add_argument("--c3-ops", type=int, default=10_000_000, help="ops per replica of config c3")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives every device slot: a multi-device context (cdb_ctx_create_multi) and "
                         "cdb_merge_sharded, rows exchanged by RCCL inside the library (the default for --gpus N > 1; "
                         "this flag also takes it at N = 1, e.g. with --devices 0,0)")
    ap.add_argument("--dist", action="store_true",
                    help="N > 1: one process per GPU (torch.distributed, constdb_amd/dist.py) instead of the "
                         "single-process cdb_merge_sharded path")
    ap.add_argument("--devices", default=None,
                    help="--single-process: device slots, e.g. 0,1,2,3 (default 0..gpus-1); a device listed twice "
                         "gives two shards on one GPU (rows then move by device copies)")
    ap.add_argument("--no-general", action="store_true",
                    help="skip the general_input figures (the same rows merged unsorted, on the partition path)")
    ap.add_argument("--force-tier", type=int, default=0, help="testing: cdb_merge_opts.force_tier")
    ap.add_argument("--no-decode-leg", action="store_true",
                    help="c4 at N=1: skip the decode_leg sub-object (the same replicas as snapshots in the "
                         "reference's HashMap order, decoded into HBM and merged)")
    ap.add_argument("--layout", default="records", choices=["records", "columns"],
                    help="input rows: records (the key-hash column + one record per row, cdb_dev_rows.stride) or "
                         "plain columns")
    ap.add_argument("--output", default="buckets", choices=["buckets", "dense"],
                    help="merge result: the engine's bucket layout (cdb_dev_output.compact = 0, what the next merge, "
                         "the canonical dump and encode read) or dense columns (compact = 1: one more pass)")
    ap.add_argument("--input-order", default="sorted", choices=["sorted", "hash-random"],
                    help="sorted: every replica's rows form one run in key-hash order (as this engine's merge "
                         "output and snapshots encoded from it are; the sorted-run path); hash-random: rows "
                         "in generator (key-index) order, i.e. random in hash (the partition path)")
    return ap.parse_args()


def c4_config(cdb, universe, replicas, seed, lo, hi, shard=0, n_shards=1):
    from constdb_amd import configs
    return configs.c4(cdb, universe, replicas, seed, lo, hi, shard, n_shards)


def alg_bytes(st, dict_share=0.5):
    """Compulsory bytes of one merge: inputs + outputs at the survey's row
    widths (member rows priced at the config's set/dict share)."""
    wm = (1 - dict_share) * W_SET + dict_share * W_DICT
    return ((st.key_rows_in + st.key_rows_out) * W_KEY + (st.node_rows_in + st.node_rows_out) * W_NODE
            + (st.member_rows_in + st.member_rows_out) * wm)


def pmc_traffic(config):
    """HBM bytes per merge step, from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
    this same bench command (scripts/gpu_round.sh -> scripts/pmc_traffic.py): every merge-pipeline
    kernel, and the bucket phase alone. None when no such measurement is committed."""
    f = profile_file(f"pmc_traffic_{config}.json")
    try:
        with open(f) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    total = bucket = 0.0
    per = {}
    for k, v in d.get("kernels", {}).items():
        if not k.startswith(MERGE_KERNEL_PREFIXES):
            continue
        b = (v["fetch_bytes"] + v["write_bytes"]) * v.get("per_step", 1)
        per[k] = b
        total += b
        if k.startswith("bucket_"):
            bucket += b
    return {"total": total, "bucket_phase": bucket, "per_kernel": per, "source": os.path.relpath(f, ROOT)}


def host_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "host_cpus": os.cpu_count()}


def cpu_baseline(cdb, args, snaps, sample):
    """The oracle's single-thread C++ fold (kind "port": the Rust reference cannot be built
    here) over already-decoded entries, best of --cpu-reps; decode excluded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cdb_oracle
    ns = None
    for rep in range(args.cpu_reps):  # one rep per call: progress on stderr between reps
        t, entries = cdb_oracle.time_fold(snaps, reps=1)
        ns = t if ns is None else min(ns, t)
        log(f"cpu baseline rep {rep}: {entries / (t * 1e-9) / 1e6:.2f} M entries/s")
    out = {"value": entries / (ns * 1e-9), "unit": "entries/s", "cores": 1, "kind": "port",
           "sample": f"{sample} ({entries} entries, decode excluded, best of {args.cpu_reps}), "
                     f"oracle/cdb_oracle.cpp std::unordered_map fold",
           **host_info()}
    ref = profile_file(f"cpu_baseline_{args.config}_10m.json")
    if os.path.exists(ref):
        with open(ref) as fh:
            out["larger_sample"] = json.load(fh)
    return out


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def setup(cdb, ctx, args):
    """Device-resident inputs of the chosen config. Returns (din, opts, info) where info holds
    the workload description and a callable producing the CPU-baseline sample."""
    from constdb_amd import configs
    L = cdb.lib()
    din = cdb.DevInput()
    opts = cdb.MergeOpts()
    c = args.config
    rec_flag = cdb.GEN_ROWS_RECORDS if args.layout == "records" else 0
    if c == "c4":
        cfg = configs.c4(cdb, args.universe_per_gpu, args.replicas, args.seed)
        cfg.flags |= rec_flag
        ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
        work = (f"C4 anti-entropy shard: {args.universe_per_gpu} keys/GPU x {args.replicas} replicas "
                f"(N=8 -> exactly C4's 500M keys)")

        def sample():
            scfg = configs.c4(cdb, args.cpu_universe, args.replicas, args.seed)
            snaps = []
            for r in range(args.replicas):
                snaps.append(cdb.gen_snapshot(scfg, r))
                log(f"cpu baseline sample: replica {r} snapshot {len(snaps[-1])} bytes")
            return (snaps,
                    f"C4 generator config, {args.cpu_universe} keys x {args.replicas} replicas")
    elif c == "c1":
        cfg = configs.c1(cdb)
        cfg.flags |= rec_flag
        ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
        work = "C1/C2 2-node MEET: 1M Bytes + 1M counters per node, 50 % key overlap, B merged into A"

        def sample():
            return [cdb.gen_snapshot(cfg, r) for r in range(2)], "C1 at full size"
    elif c == "c5":
        cfg = configs.c5(cdb)
        cfg.flags |= rec_flag
        ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
        work = "C5 Zipf hot keys: 10M keys, children ~ rank^-1.1, 80M node/member rows over 8 replicas"

        def sample():
            scfg = configs.c5(cdb, universe=1_000_000, events=8_000_000)
            return [cdb.gen_snapshot(scfg, r) for r in range(8)], "C5 generator at 1M keys / 8M children"
    else:  # c3
        log("building C3 replica states through the device op apply")
        snaps = configs.c3_snapshots(cdb, ctx, ops_per_replica=args.c3_ops, log=log)
        batches = [cdb.decode_snapshot(s) for s in snaps]
        arr = (ctypes.c_void_p * len(batches))(*[b.handle for b in batches])
        ctx.check(L.cdb_upload_batches(ctx.handle, arr, len(batches), ctypes.byref(din)))
        if args.layout == "records":
            from constdb_amd.runs import to_records
            to_records(cdb, ctx, din)
        opts.flags = cdb.MERGE_GC_DELETES
        opts.gc_watermark = configs.median_member_time(cdb, batches)
        work = (f"C3 set/dict add-win merge: 4 replicas x {args.c3_ops} sadd/srem/hset/hdel replayed over "
                f"100K keys (Zipf members), merge + DB::gc at the median member time")

        def sample():
            return snaps, "C3 at full size (the same 4 snapshots)"
    return din, opts, {"workload": work, "sample": sample}


SIGN = -(1 << 63)


def timed_merges(cdb, ctx, din, opts, args, steps):
    """`warmup` untimed merges, then `steps` timed ones (host wall: cdb_merge_device synchronises
    its stream before returning). Returns (ms per step, per-phase HIP-event ms, last stats)."""
    L = cdb.lib()
    dout = cdb.DevOutput()
    dense = args.output == "dense"
    if dense:  # caller-allocated dense columns; the bucket layout's rows are the library's
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(dout.keys), din.keys.n, 8))
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(dout.nodes), din.nodes.n, 6))
        ctx.check(L.cdb_dev_rows_alloc(ctx.handle, ctypes.byref(dout.members), din.members.n, 6))
    st = cdb.MergeStats()

    def step():
        dout.compact = 1 if dense else 0
        ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(opts), ctypes.byref(dout),
                                     ctypes.byref(st), None))

    for _ in range(args.warmup):
        step()
    acc = dict(partition=0.0, bucket=0.0, finish=0.0, device=0.0)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
        acc["bucket"] += st.bucket_ms
        acc["partition"] += st.partition_ms
        acc["finish"] += st.finish_ms
        acc["device"] += st.device_ms
    t1 = time.perf_counter()
    if dense:
        for fam in (dout.keys, dout.nodes, dout.members):
            L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
    return (t1 - t0) * 1e3 / steps, {k: v / steps for k, v in acc.items()}, st


def run_single(cdb, args):
    import torch  # noqa: F401 -- before libcdbmerge: one HIP runtime per process
    ctx = cdb.Context(0)
    L = cdb.lib()
    din, opts, info = setup(cdb, ctx, args)
    opts.force_tier = args.force_tier
    from constdb_amd import configs
    general = None
    if args.input_order == "sorted" and not args.no_general:
        # the same rows in the order the setup left them (generator / batch order: random in key hash),
        # merged on the general (partition) path -- what a caller whose rows are not in runs gets
        log("general-input path (partition) on the unsorted rows")
        gms, gper, gst = timed_merges(cdb, ctx, din, opts, args, args.steps)
        gB = alg_bytes(gst, configs.DICT_MEMBER_SHARE[args.config])
        gtr = pmc_traffic(args.config + "_general")
        general = {"ms_per_step": gms, "value": gst.key_rows_in / (gms * 1e-3), "merge_path": "partition",
                   "phases_ms": {"partition": gper["partition"], "bucket_merge": gper["bucket"],
                                 "finish": gper["finish"], "device_total": gper["device"]},
                   "roofline_frac": gB / (gper["device"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                   "traffic": gtr["total"] if gtr else None,
                   "traffic_over_alg": gtr["total"] / gB if gtr else None,
                   "traffic_source": gtr["source"] if gtr else None}
    if args.input_order == "sorted":
        from constdb_amd.runs import sort_into_runs, state_runs
        if args.config in ("c1", "c4", "c5") and args.layout == "records":
            # each replica's rows as this engine keeps a replica state: merged alone, read back as
            # position-0 rows, moved to the replica's position (setup, untimed)
            log("replica states: each replica merged alone and kept as state rows")
            state_runs(cdb, ctx, din)
            info["workload"] += ("; input: one key-hash-ordered run per replica, each the replica's own merge "
                                 "result kept in HBM as state rows (cdb_dev_state_rows, cdb_dev_input_append): "
                                 "the sorted-run path")
        else:
            sort_into_runs(din)
            info["workload"] += ("; input: one key-hash-ordered run per replica (a merge result kept as position 0, "
                                 "or a snapshot this engine encoded, decoded by cdb_decode_snapshots_device): "
                                 "the sorted-run path")
    else:
        info["workload"] += "; input: rows in generator order, random in key hash: the partition path"
    ms, per, st = timed_merges(cdb, ctx, din, opts, args, args.steps)
    B = alg_bytes(st, configs.DICT_MEMBER_SHARE[args.config])
    tr = pmc_traffic(args.config if args.input_order == "sorted" else args.config + "_general")
    res = {
        "metric": "merged CRDT entries/sec (snapshot merge)",
        "value": st.key_rows_in / (ms * 1e-3),
        "unit": "entries/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: seeded GenModel replica states resident in HBM (keys 'key:<i>')",
        "config": {"workload": info["workload"], "config": args.config, "replicas": din.n_pos,
                   "key_rows_in": st.key_rows_in, "node_rows_in": st.node_rows_in,
                   "member_rows_in": st.member_rows_in, "key_rows_out": st.key_rows_out,
                   "node_rows_out": st.node_rows_out, "member_rows_out": st.member_rows_out,
                   "gc_watermark": opts.gc_watermark, "input_order": args.input_order,
                   "input_layout": args.layout, "output_layout": args.output,
                   "merge_path": "sorted runs" if st.sorted_runs else "partition", "parallelism": "single GPU"},
        "child_rows_per_s": (st.node_rows_in + st.member_rows_in) / (ms * 1e-3),
        "phases_ms": {"partition": per["partition"], "bucket_merge": per["bucket"], "finish": per["finish"],
                      "device_total": per["device"]},
        # achieved = B_alg / t_merge over the WHOLE merge (HIP events on the merge
        # stream around partition -> bucket merge -> compaction)
        "roofline": {"bound": "hbm",
                     "kernel": ("whole merge pipeline (run directories / partition + bucket merge + "
                                + ("compaction" if args.output == "dense" else "bucket directory scans") + "), HIP events"),
                     "achieved": B / (per["device"] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": B / (per["device"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "alg_bytes": B,
                     "traffic": tr["total"] if tr else None,
                     "traffic_over_alg": tr["total"] / B if tr else None,
                     "traffic_source": tr["source"] if tr else None,
                     "phase_frac": {"bucket_merge": B / (per["bucket"] * 1e-3) / 1e9 / HBM_PEAK_GBS}},
        "stats": {"type_conflicts": st.type_conflicts, "dict_merges": st.dict_merges,
                  "deletes_gced": st.deletes_gced, "hot_buckets": st.hot_buckets,
                  "wide_buckets": st.wide_buckets, "mid_buckets": st.mid_buckets,
                  "orphans": st.orphan_children, "hot_slow_runs": st.hot_slow_runs,
                  "hot_merged_children": st.hot_merged_children,
                  "wave_pipe_buckets": st.wave_pipe_buckets, "wave_pipe_units": st.wave_pipe_units},
    }
    if tr:
        res["roofline"]["traffic_per_kernel"] = tr["per_kernel"]
    if general is not None:
        res["general_input"] = general
    for fam in (din.keys, din.nodes, din.members):
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
    if args.config == "c4" and not args.no_decode_leg and args.input_order == "sorted":
        res["decode_leg"] = decode_leg(cdb, ctx, args, ms)
    res["_sample"] = info["sample"]
    return res


def decode_leg(cdb, ctx, args, merge_ms):
    """The same replicas as snapshots in the reference's HashMap order (the generator's writer
    layout, no key order: db.rs:122-136), host-resident as a peer would send them, decoded straight
    into HBM (cdb_decode_snapshots_device: validation, entry index, parse, each snapshot sorted into
    one run) and merged into the bucket layout (pull.rs:64-79 then :120-128). Not `value`: the
    snapshot bytes cross PCIe, so the copy floor is reported beside it."""
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    cfg = c4_config(cdb, args.universe_per_gpu, args.replicas, args.seed, 0, args.replicas)
    log("decode leg: generating the replicas' snapshots")
    with ThreadPoolExecutor(min(args.replicas, 16)) as ex:  # (the generator releases the GIL)
        snaps = list(ex.map(lambda r: cdb.gen_snapshot(cfg, r), range(args.replicas)))
    nbytes = sum(len(x) for x in snaps)
    trace = os.path.join(tempfile.mkdtemp(), "decode_trace.jsonl")
    os.environ["CDB_DECODE_TRACE"] = trace
    L = cdb.lib()
    log(f"decode leg: {nbytes / 1e9:.2f} GB of snapshots into HBM")
    t = time.perf_counter()
    batches, din = cdb.decode_snapshots_device(ctx, snaps, records=True)
    dec_ms = (time.perf_counter() - t) * 1e3
    del os.environ["CDB_DECODE_TRACE"]
    with open(trace) as fh:
        phases = json.loads(fh.read().strip().split("\n")[-1])
    out = cdb.DevOutput()
    out.compact = 0
    st = cdb.MergeStats()
    t = time.perf_counter()
    ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.merge_opts()), ctypes.byref(out),
                                 ctypes.byref(st), None))
    mms = (time.perf_counter() - t) * 1e3
    for fam in (din.keys, din.nodes, din.members):
        L.cdb_dev_rows_release(ctx.handle, ctypes.byref(fam))
    del batches, snaps
    return {"snapshots": args.replicas, "bytes": nbytes, "order": "generator (HashMap-like, no key order)",
            "decode_ms": dec_ms, "merge_ms": mms, "total_ms": dec_ms + mms,
            "total_over_merge_step": (dec_ms + mms) / merge_ms, "sorted_runs": st.sorted_runs,
            "pcie_floor_ms": nbytes / 56e9 * 1e3, "phases": phases,
            "note": "host-resident snapshot bytes; PCIe-inclusive, never `value`"}


def run_single_process(cdb, args):
    """One process, every device slot of a multi-device context (the reference's one server process,
    server.rs:95,128-130): replica r on slot r*N/R as one key-hash-ordered run, cdb_merge_sharded per
    step (owner splits, RCCL point-to-point inside the library, per-device merges)."""
    import torch  # noqa: F401 -- before libcdbmerge: one HIP runtime per process
    from constdb_amd import configs
    from constdb_amd.runs import sort_into_runs
    devs = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    if len(devs) > 8:
        raise SystemExit("at most 8 device slots (cdb_ctx_create_multi)")
    N = len(devs)
    L = cdb.lib()
    ctx = cdb.Context(devices=devs)
    R = args.replicas
    universe = args.universe_per_gpu * N
    ins = []
    for i in range(N):
        c = ctx.shard(i)
        cfg = configs.c4(cdb, universe, R, args.seed, i * R // N, (i + 1) * R // N)
        d = cdb.DevInput()
        c.check(L.cdb_gen_device(c.handle, ctypes.byref(cfg), ctypes.byref(d)))
        d.n_pos = R
        torch.cuda.set_device(devs[i])
        sort_into_runs(d, R)
        ins.append(d)
        log(f"slot {i} (device {devs[i]}): {d.keys.n} key rows")
    for _ in range(args.warmup):
        outs, sts, xs = cdb.merge_sharded(ctx, ins)
    acc = dict(split=0.0, exchange=0.0, merge=0.0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        outs, sts, xs = cdb.merge_sharded(ctx, ins)
        acc["split"] += xs.split_ms
        acc["exchange"] += xs.exchange_ms
        acc["merge"] += xs.merge_ms
    t1 = time.perf_counter()
    if len(set(devs)) > 1 and xs.transport != 1 and os.environ.get("CDB_SHARD_TRANSPORT") != "peer":
        raise SystemExit(f"distinct devices {devs} exchanged rows by transport {xs.transport}, not RCCL")
    ms = (t1 - t0) * 1e3 / args.steps
    per = {k: v / args.steps for k, v in acc.items()}
    entries = sum(s.key_rows_in for s in sts)
    B = sum(alg_bytes(s, configs.DICT_MEMBER_SHARE["c4"]) for s in sts)
    link = max((xs.link_bytes[i][j] for i in range(N) for j in range(N) if i != j), default=0)
    res = {
        "metric": "merged CRDT entries/sec (snapshot merge)", "value": entries / (ms * 1e-3), "unit": "entries/s",
        "n_gpus": len(set(devs)), "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: seeded GenModel replica states generated in HBM, each replica one key-hash-ordered run",
        "config": {"workload": f"C4 anti-entropy: {universe} keys x {R} replicas over device slots {devs}, one "
                               f"process (cdb_merge_sharded)", "config": "c4", "replicas": R,
                   "key_rows_in_total": entries, "parallelism": f"key-hash sharding x{N} (single process)",
                   "transport": {0: "none", 1: "RCCL point-to-point", 2: "device copies"}[xs.transport],
                   "merge_path": "sorted runs" if all(s.sorted_runs for s in sts) else "partition"},
        "exchange": {"split_ms": per["split"], "ms": per["exchange"], "bytes_moved_per_step": xs.bytes_moved,
                     "max_link_bytes": link,
                     "max_link_GBps": link / (per["exchange"] * 1e-3) / 1e9 if per["exchange"] > 0 and link else None,
                     "transfers": xs.transfers},
        "merge_ms": per["merge"],
        "roofline": {"bound": "hbm", "kernel": "merge pipeline of every device (HIP events); B_alg summed over "
                                               "devices / slowest device's merge time",
                     "achieved": B / (per["merge"] * 1e-3) / 1e9, "peak": 8000.0 * len(set(devs)), "unit": "GB/s",
                     "frac": B / (per["merge"] * 1e-3) / 1e9 / (8000.0 * len(set(devs))), "alg_bytes": B,
                     "traffic": None},
    }
    for i in range(N):
        for fam in (ins[i].keys, ins[i].nodes, ins[i].members):
            L.cdb_dev_rows_release(ctx.shard(i).handle, ctypes.byref(fam))
    return res


def spawn_ranks(args):
    """`--gpus N` (N > 1) without a launcher: start N ranks (one process per GPU) under
    torch.distributed.run as a child process, before this process touches any GPU, and exit with
    its status. Rank 0's JSON line goes to our stdout unchanged."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"--gpus {args.gpus} without WORLD_SIZE: launching {args.gpus} ranks")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def launcher_barrier(world, rank):
    """Under a launcher with the single-process path: a gloo group (no GPU) whose barriers bracket
    rank 0's run, so every rank starts and ends together. Returns a callable barrier."""
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    return tdist


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and not args.dist:
        args.single_process = True
    if args.gpus > 1 and world == 1 and args.dist:
        raise SystemExit(spawn_ranks(args))
    tdist = None
    if args.single_process and world > 1:
        if world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
        tdist = launcher_barrier(world, rank)
        tdist.barrier()
        if rank != 0:  # rank 0 drives every GPU; this rank touches none
            tdist.barrier()
            tdist.destroy_process_group()
            return
    # RCCL and the HIP runtime may print banners on the C-level stdout: keep fd 1 for the
    # single JSON line and send everything else to stderr.
    json_fd = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(os.dup(2), "w")
    import constdb_amd as cdb
    from constdb_amd import build as b
    b.build()
    if args.single_process:
        try:
            res = run_single_process(cdb, args)
        finally:
            if tdist is not None:
                tdist.barrier()
                tdist.destroy_process_group()
        sample = None
    elif world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    elif world > 1 or args.force_dist:
        if args.config != "c4":
            raise SystemExit("the multi-GPU bench runs config c4")
        from constdb_amd import dist
        res = dist.run_bench(cdb, args, rank, world, local_rank, c4_config, alg_bytes)
        sample = None
    else:
        res = run_single(cdb, args)
        sample = res.pop("_sample")
    if rank != 0:
        os.close(json_fd)
        return
    if tdist is not None:
        res["config"]["launcher"] = f"{world} ranks: rank 0 drives every GPU, the others join its barriers"
    if not args.no_cpu_baseline and sample is not None:
        snaps, desc = sample()
        res["cpu_baseline"] = cpu_baseline(cdb, args, snaps, desc)
    elif not args.no_cpu_baseline and world > 1:
        pass  # rank 0 at N=1 only (the driver's N=1 line carries it)
    with os.fdopen(json_fd, "w") as out:
        out.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
