#!/bin/bash
# The whole GPU suite and smoke on the final commit.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest_r4ay.log 2>&1
rc=$?; tail -2 $O/pytest_r4ay.log
[ $rc -le 1 ] || { echo "pytest ended with $rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r4ay.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_r4ay.log; exit 2; }
tail -1 $O/smoke_r4ay.log
echo "r4ay ok (pytest rc=$rc)"
