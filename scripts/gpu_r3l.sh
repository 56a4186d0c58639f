#!/bin/bash
# Round 3: where the decode's device entry index spends its time (kernel + copy trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_dec_r3n -o run -- python scripts/bench_decode.py --reps 1 --device-snapshots 2 > gpurun_out/prof_dec_r3n.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_dec_r3n.log; exit 1; }
tail -3 gpurun_out/prof_dec_r3n.log
head -25 gpurun_out/prof_dec_r3n/run_kernel_stats.csv | cut -c1-160
cat gpurun_out/prof_dec_r3n/run_memory_copy_stats.csv | cut -c1-160
