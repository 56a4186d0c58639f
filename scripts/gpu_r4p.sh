#!/bin/bash
# Round 4: the decoder feeding the merge at full size.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_decode_merge_full_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_r4p.log 2>&1
rc=$?; tail -6 $O/pytest_r4p.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc"; exit 1; }
echo "r4p ok"
