#!/bin/bash
# Round 4: kernel + copy trace of the C4 bench's decode leg.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_leg_r4t -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-general > $O/prof_leg_r4t.log 2>&1 || { echo "prof failed"; tail -5 $O/prof_leg_r4t.log; exit 1; }
echo "r4t ok"
