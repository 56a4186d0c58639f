"""Host index pass timing on this machine: sequential vs threaded DATAS section (cdb_snapshot_index_selftest)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["CDB_SELFTEST_TIMING"] = "1"
import constdb_amd as cdb
cfg = cdb.gen_config(seed=4, universe=8_000_000, n_replicas=8, replica_hi=8)
snap = cdb.gen_snapshot(cfg, 0)
n = ctypes.c_uint64()
for th in (16, 16, 32, 8):
    st = cdb.lib().cdb_snapshot_index_selftest(snap, len(snap), 0, th, ctypes.byref(n))
    print("threads", th, "status", st, "entries", n.value, flush=True)
