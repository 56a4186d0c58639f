#!/bin/bash
# Round 3: timeline of the 8-snapshot decode into HBM (kernel + copy trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_dec_r3q -o run -- python scripts/bench_decode.py --reps 1 --device-snapshots 8 > gpurun_out/prof_dec_r3q.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_dec_r3q.log; exit 1; }
grep metric gpurun_out/prof_dec_r3q.log | tail -1
