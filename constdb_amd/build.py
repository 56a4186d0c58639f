"""Builds libcdbmerge.so (HIP kernels for gfx950 + host C++) in-tree with hipcc.

Every source compiles to its own object (in parallel, only the stale ones), then one link.
The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libcdbmerge.so")
OBJ = os.path.join(HERE, "build", "obj")
SOURCES = ["engine.hip", "gen_device.hip", "decode_gpu.hip", "ops_apply.hip", "ops_gpu.hip", "encode_gpu.hip", "shard.hip",
           "capi.cpp", "decode.cpp", "gen.cpp", "ops.cpp"]
HEADERS = ["common.h", "batch.h", "engine.h", "partition.hip.h", "bucket.hip.h", "bucket_wave.hip.h",
           "gen_model.h", "ops.h", "runs.hip.h", "hot.hip.h", "radix.hip.h"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-value", "-I/opt/rocm/include"]
LIBS = ["-ldl"]


def _sources():
    return list(SOURCES)


def _deps_time():
    deps = [os.path.join(CSRC, f) for f in HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "cdb_merge.h"))
    deps.append(os.path.abspath(__file__))
    return max(os.path.getmtime(d) for d in deps)


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return _deps_time() > t or any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in _sources())


def _compile(hipcc, src, obj, defines, verbose):
    cmd = [hipcc, *FLAGS, *[f"-D{d}" for d in defines], "-c", "-o", obj + ".tmp", os.path.join(CSRC, src)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(obj + ".tmp", obj)


def build(force=False, verbose=False, out=None, defines=()):
    """Builds the library (out/defines: profiling variants with their own object directory)."""
    if out is None and os.environ.get("CDB_LIB"):
        return os.environ["CDB_LIB"]
    target = out or OUT
    if out is None and not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objdir = OBJ if not defines else OBJ + "_" + "_".join(d.replace("=", "") for d in defines)
    os.makedirs(objdir, exist_ok=True)
    dt = _deps_time()
    jobs = []
    objs = []
    for f in _sources():
        obj = os.path.join(objdir, f + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(dt, os.path.getmtime(os.path.join(CSRC, f))):
            jobs.append((f, obj))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    if jobs:
        with ThreadPoolExecutor(workers) as ex:
            for r in [ex.submit(_compile, hipcc, f, o, defines, verbose) for f, o in jobs]:
                r.result()
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", target + ".tmp", *objs, *LIBS]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(target + ".tmp", target)
    return target


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(OUT)
