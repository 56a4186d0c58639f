#!/bin/bash
# C3 child target per bucket (CDB_PLAN_CTARGET) with the LDS chip-wide path.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
for t in 4096 3072 2048 6144; do
  CDB_PLAN_CTARGET=$t timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-general > $O/r4ai_c3_$t.json 2> $O/r4ai_c3_$t.err || exit 3
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('ctarget', sys.argv[2], round(d['ms_per_step'],3), 'ms', d['stats']['mid_buckets'])" $O/r4ai_c3_$t.json $t
done
