#!/bin/bash
# HIP API + kernel trace of the 8-snapshot decode into HBM (where the host-side time goes).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $O/prof_dec_r4am -o run -- python scripts/bench_decode.py --reps 2 > $O/prof_dec_r4am.log 2>&1 || { echo "prof failed"; tail -5 $O/prof_dec_r4am.log; exit 1; }
echo "r4am ok"
