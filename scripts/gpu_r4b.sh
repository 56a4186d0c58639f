#!/bin/bash
# Round 4: records vs columns on the bucket-layout result, with kernel stats of each.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-r4b}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_records_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "records tests failed"; tail -40 $O/pytest_$T.log; exit 1; }
tail -1 $O/pytest_$T.log
fi
for lay in ${LAYS:-"records buckets" "columns buckets"}; do
  set -- $lay
  timeout -k 10 300 python bench.py --config ${CONFIG:-c4} --steps 5 --warmup 2 --no-cpu-baseline --no-general --layout $1 --output $2 $EXTRA > $O/bench_${T}_$1_$2.json 2> $O/bench_${T}_$1_$2.err || { echo "bench $lay failed"; tail -20 $O/bench_${T}_$1_$2.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()}, 'frac', round(d['roofline']['frac'],3))" $O/bench_${T}_$1_$2.json "$lay"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$1_$2 -o run -- python bench.py --config ${CONFIG:-c4} --steps 5 --warmup 2 --no-cpu-baseline --no-general --layout $1 --output $2 $EXTRA > $O/prof_${T}_$1_$2.log 2>&1 || { echo "prof failed"; exit 3; }
  f=$(find $O/prof_${T}_$1_$2 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" 8 | grep -v "at::\|rocprim\|gen_"
done
echo "round ok"
