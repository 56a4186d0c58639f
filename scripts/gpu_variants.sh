#!/bin/bash
# Parity tests once, then the full bench under several engine knobs (env VARIANTS: a list of
# "NAME:ENV=VAL,ENV=VAL" items) and a compact phase summary of each.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-v}
O=gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_$T.log; exit 1; }
  tail -1 $O/pytest_$T.log
fi
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}
  envs=${v#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_${T}_$name.json 2> $O/bench_${T}_$name.err ) || { echo "bench $name failed"; tail -20 $O/bench_${T}_$name.err; exit 2; }
  python3 -c "
import json,sys; r=json.load(open('$O/bench_${T}_$name.json'))
print('$name', round(r['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in r.get('phases_ms',{}).items()}, 'frac', round(r['roofline']['frac'],3), r.get('stats',{}).get('wide_buckets'))"
done
echo "variants ok"
