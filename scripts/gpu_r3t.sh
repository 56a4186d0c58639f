#!/bin/bash
# Round 3: GPU suite after the slow-run statistic and the misc-header move.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3t.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_r3t.log; exit 1; }
tail -2 gpurun_out/pytest_r3t.log
