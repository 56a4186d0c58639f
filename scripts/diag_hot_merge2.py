"""Diagnostic: forced chip-wide merges of a small config with few id bits, list merge vs radix."""
import ctypes, os, sys
sys.path.insert(0, os.getcwd())
import torch  # noqa: F401
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import state_runs, sort_into_runs
ctx = cdb.Context(0)
L = cdb.lib()
cfg = cdb.gen_config(seed=91, universe=40000, n_replicas=5, key_permille=600, mix_bytes=20, mix_counter=30,
                     mix_set=25, mix_dict=25, mean_members=20, side_permille=150, conflict_ppm=10000,
                     tie_permille=100, del_permille=300, replica_lo=0, replica_hi=5)
cfg.flags |= cdb.GEN_ROWS_RECORDS
for mode in ("plain", "state"):
    din = cdb.DevInput()
    ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
    if mode == "state":
        state_runs(cdb, ctx, din)
    else:
        sort_into_runs(din)
    os.environ["CDB_HOT_LDS"] = "0"
    os.environ["CDB_HOT_ID_BITS"] = "8"
    os.environ["CDB_HOT_PROF"] = "1"
    for merge in ("1", "0"):
        os.environ["CDB_HOT_MERGE"] = merge
        out = cdb.DevOutput(); out.compact = 0
        st = cdb.MergeStats()
        ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.merge_opts(force_tier=2)),
                                     ctypes.byref(out), ctypes.byref(st), None))
        print(mode, merge, "slow", st.hot_slow_runs, "merged", st.hot_merged_children, "hot", st.hot_buckets, flush=True)
    for k in ("CDB_HOT_LDS", "CDB_HOT_ID_BITS", "CDB_HOT_PROF", "CDB_HOT_MERGE"):
        del os.environ[k]
