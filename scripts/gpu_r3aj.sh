#!/bin/bash
# Round 3: kernel stats of C5 and C3 after the size-class batches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c5 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${c}_r3aj -o run -- python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/prof_${c}_r3aj.log 2>&1 || { echo "prof $c failed"; exit 1; }
done
echo ok
