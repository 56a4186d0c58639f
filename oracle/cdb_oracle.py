"""ctypes loader for the C++ oracle (oracle/cdb_oracle.cpp) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OracleStats(ctypes.Structure):
    _fields_ = [("type_conflicts", ctypes.c_uint64), ("dict_merges", ctypes.c_uint64),
                ("member_tombstones_gced", ctypes.c_uint64), ("err_offset", ctypes.c_size_t),
                ("err_snapshot", ctypes.c_int32)]


FLAG_DICT_PANIC = 1
FLAG_REFERENCE_CHECKSUM = 2
FLAG_GC = 4
FLAG_GC_MEMBERS = 8


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "libcdb_oracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(path)
        L.cdbo_fold.restype = ctypes.c_int
        L.cdbo_fold.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                ctypes.POINTER(OracleStats)]
        L.cdbo_free.argtypes = [ctypes.c_void_p]
        L.cdbo_time_fold.restype = ctypes.c_int64
        L.cdbo_time_fold.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        _LIB = L
    return _LIB


def _arrays(snaps):
    n = len(snaps)
    bufs = (ctypes.c_char_p * n)(*[bytes(s) for s in snaps])
    lens = (ctypes.c_size_t * n)(*[len(s) for s in snaps])
    return n, bufs, lens


def fold(snaps, flags=0, gc_watermark=0):
    """Returns (status, canonical_dump_bytes, OracleStats)."""
    L = lib()
    n, bufs, lens = _arrays(snaps)
    out = ctypes.c_void_p()
    out_len = ctypes.c_size_t()
    st = OracleStats()
    rc = L.cdbo_fold(bufs, lens, n, flags, gc_watermark, ctypes.byref(out), ctypes.byref(out_len),
                     ctypes.byref(st))
    dump = b""
    if rc == 0:
        dump = bytes((ctypes.c_char * out_len.value).from_address(out.value)) if out_len.value else b""  # (> 2 GiB too)
        L.cdbo_free(out)
    return rc, dump, st


def time_fold(snaps, reps=3):
    """CPU baseline: best-of-reps single-thread fold time (ns) and Data entries folded."""
    L = lib()
    n, bufs, lens = _arrays(snaps)
    ent = ctypes.c_uint64()
    ns = L.cdbo_time_fold(bufs, lens, n, reps, ctypes.byref(ent))
    return ns, ent.value
