#!/bin/bash
# Plan-knob sweep of the full bench (one run per setting; ms_per_step compared).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
for kv in ${KNOBS:-"X=0" "CDB_PLAN_TARGET=36" "CDB_PLAN_TARGET=44" "CDB_PLAN_TARGET=48" "CDB_PLAN_D0=640" "CDB_PLAN_D0=896"}; do
  env $kv timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/knob_$kv.json 2> $O/knob_$kv.err || { echo "bench $kv failed"; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/knob_$kv.json'));print('$kv', round(d['ms_per_step'],2), d['phases_ms'])"
done
