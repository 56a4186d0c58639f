#!/bin/bash
# Round 4: bucket-size sweep of the C4 step (CDB_PLAN_TARGET: key rows per bucket).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
for t in ${TARGETS:-32 36 40 44 48}; do
  CDB_PLAN_TARGET=$t timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-general --no-decode-leg > $O/s_$t.json 2> $O/s_$t.err || { echo "bench $t failed"; tail -5 $O/s_$t.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('target', sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()}, d['stats']['wide_buckets'], d['stats']['mid_buckets'])" $O/s_$t.json $t
done
echo "r4s ok"
