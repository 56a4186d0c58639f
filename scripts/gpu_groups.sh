#!/bin/bash
# Round-6 grouped units of the persistent wave tier: the parity tests of the sorted-run path, then
# an A/B of the unit shape (CDB_GROUPS=0: one bucket per unit at round-5 bucket sizes). A library of
# another tree can join as a variant: NAME=CDB_LIB=variants/<lib>.so (build.build(out=...)).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
T=${TAG:-grp}
timeout -k 10 600 python -u -m pytest tests/test_pipe_oracle_gpu.py tests/test_runs_oracle_gpu.py tests/test_sorted_runs_gpu.py tests/test_hot_merge_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_$T.log; exit 1; }
tail -2 $O/pytest_$T.log
TAG=$T CONFIG=${CONFIG:-c4} VARIANTS="${VARIANTS:-grp= off=CDB_GROUPS=0 c64=CDB_GROUP_CCAP=64 t24=CDB_PIPE_TARGET=24 t32=CDB_PIPE_TARGET=32}" bash scripts/gpu_ab.sh
