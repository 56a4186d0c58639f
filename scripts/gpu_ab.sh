#!/bin/bash
# A/B of one bench config under environment variants: for each "NAME=ENV" in VARIANTS, a bench line
# (no CPU baseline, no general input) into gpurun_out/ab_<TAG>_<NAME>.json. Optional TESTS: a pytest
# selection run first. Usage (from gpurun): TAG=x CONFIG=c3 VARIANTS="base= rec=CDB_HOT_DIRECT=0" bash scripts/gpu_ab.sh
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
T=${TAG:-ab}
C=${CONFIG:-c4}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_$T.log; exit 1; }
  tail -2 $O/pytest_$T.log
fi
for v in $VARIANTS; do
  name=${v%%=*}
  envs=${v#*=}
  envs=${envs//,/ }  # (several assignments: A=1,B=2)
  timeout -k 10 ${BENCH_TIMEOUT:-400} env $envs python bench.py --config $C --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-general --no-decode-leg > $O/ab_${T}_$name.json 2> $O/ab_${T}_$name.err || { echo "bench $name failed"; tail -20 $O/ab_${T}_$name.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('$O/ab_${T}_$name.json')); print('$name', round(d['ms_per_step'],3), 'ms', 'frac', round(d['roofline']['frac'],4))"
done
if [ -n "$PMC" ]; then
  KRE="merge_begin_marker|merge_end_marker|pipe_|iota|set_dir|stamp_pos|part_|bucket_|compact|scan_|stats_reduce|gc_lastbad|hot_|sorted_|seg_|run_|mat_|radix_hist|radix_scatter"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv -d $O/pmc_${C}_${T}_$c -o run -- python bench.py --config $C --steps 1 --warmup 0 --no-cpu-baseline --no-general --no-decode-leg > $O/pmc_${C}_${T}_$c.log 2>&1 || { echo "pmc $c failed"; exit 4; }
  done
  python3 scripts/pmc_traffic.py $O/pmc_${C}_${T}_FETCH_SIZE $O/pmc_${C}_${T}_WRITE_SIZE $O/pmc_traffic_${C}_$T.json || exit 5
fi
if [ -n "$KTRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${C}_$T -o run -- python bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --no-general --no-decode-leg > $O/prof_${C}_$T.log 2>&1 || { echo "prof failed"; exit 3; }
fi
echo "ab ok"
