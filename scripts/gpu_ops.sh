#!/bin/bash
# Op-stream apply on the GPU: its parity tests, then (ALL=1) the whole GPU suite.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-ops}
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "ops pytest failed"; tail -40 $O/pytest_$T.log; exit 1; }
tail -1 $O/pytest_$T.log
if [ -n "$ALL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_all_$T.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_all_$T.log; exit 2; }
  tail -1 $O/pytest_all_$T.log
fi
echo "ops ok"
