#!/bin/bash
# GPU test pass: FILES (default: the whole suite) under one pytest process.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-t}
timeout -k 10 ${TLIM:-900} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_$T.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_$T.log | grep -v PASSED | tail -15
grep -c PASSED $O/pytest_$T.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert" $O/pytest_$T.log | head -30; fi
exit $rc
