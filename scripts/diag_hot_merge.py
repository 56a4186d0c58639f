import ctypes, os, sys
sys.path.insert(0, os.getcwd())
import torch
import constdb_amd as cdb
from constdb_amd import configs
from constdb_amd.runs import state_runs, sort_into_runs
ctx = cdb.Context(0)
L = cdb.lib()
cfg = configs.c5(cdb, universe=300_000, events=3_000_000)
cfg.flags |= cdb.GEN_ROWS_RECORDS
din = cdb.DevInput()
ctx.check(L.cdb_gen_device(ctx.handle, ctypes.byref(cfg), ctypes.byref(din)))
os.environ.pop("CDB_HOT_PROF", None)
state_runs(cdb, ctx, din)
os.environ["CDB_HOT_PROF"] = "1"
print("runs", din.n_runs, [din.run_start[1][r] for r in range(din.n_runs + 1)], flush=True)
out = cdb.DevOutput(); out.compact = 0
st = cdb.MergeStats()
ctx.check(L.cdb_merge_device(ctx.handle, ctypes.byref(din), ctypes.byref(cdb.merge_opts()), ctypes.byref(out), ctypes.byref(st), None))
print({k: v for k, v in st.as_dict().items()}, flush=True)
