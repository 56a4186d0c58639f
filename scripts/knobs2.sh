#!/bin/bash
# Bench variants: entries "ENVS :: BENCH_ARGS" in $VARIANTS separated by ';'
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
IFS=';' read -ra VS <<< "$VARIANTS"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  E="${v%%::*}"; A="${v#*::}"
  env $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $A > $O/knob_$i.json 2> $O/knob_$i.err || { echo "variant $v failed"; tail -5 $O/knob_$i.err; continue; }
  python3 -c "import json;d=json.load(open('$O/knob_$i.json'));print('$v', round(d['ms_per_step'],2), {k:round(x,2) for k,x in d['phases_ms'].items()}, d['stats']['wide_buckets'])"
done
