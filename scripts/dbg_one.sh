#!/bin/bash
# Debug one parity test with a device sync after every launch (CDB_SYNC_CHECK).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
CDB_VERIFY_PARTITION=1 CDB_SYNC_CHECK=1 timeout -k 10 120 python -m pytest tests/test_gpu_parity.py -x -q -k "${TESTK:-test_random_small and 1]}" > gpurun_out/dbg.log 2>&1
echo rc $?
grep -E "Error|error|FAILED|passed|failed" gpurun_out/dbg.log | head -20
