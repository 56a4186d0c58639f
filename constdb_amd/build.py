"""Builds libcdbmerge.so (HIP kernels for gfx950 + host C++) in-tree with hipcc.

The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libcdbmerge.so")
SOURCES = ["engine.hip", "gen_device.hip", "decode_gpu.hip", "ops_apply.hip", "ops_gpu.hip", "encode_gpu.hip", "capi.cpp", "decode.cpp", "gen.cpp",
           "ops.cpp"]
HEADERS = ["common.h", "batch.h", "engine.h", "partition.hip.h", "bucket.hip.h", "bucket_wave.hip.h",
           "gen_model.h", "ops.h", "runs.hip.h", "hot.hip.h", "radix.hip.h"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "cdb_merge.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, out=None, defines=()):
    """Builds the library (out/defines: profiling variants, e.g. scripts/wave_phases.sh)."""
    if out is not None:
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-w",
               *[f"-D{d}" for d in defines], "-o", out] + [os.path.join(CSRC, f) for f in SOURCES]
        subprocess.check_call(cmd)
        return out
    if os.environ.get("CDB_LIB"):
        return os.environ["CDB_LIB"]
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-value",
           "-o", OUT + ".tmp"] + [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(OUT)
