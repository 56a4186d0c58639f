#!/bin/bash
# Round 4: the whole GPU suite and smoke().
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/pytest_r4m.log 2>&1
rc=$?; tail -5 $O/pytest_r4m.log
[ $rc -le 1 ] || { echo "pytest ended with $rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r4m.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_r4m.log; exit 2; }
tail -2 $O/smoke_r4m.log
echo "r4m ok (pytest rc=$rc)"
