#!/bin/bash
# Round 3: decode tests incl. the huge-entry device index case.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_decode_device_gpu.py tests/test_decode_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r3w.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_r3w.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_r3w.log | tail -12
