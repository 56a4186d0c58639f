#!/bin/bash
# Round 4, first GPU check of the records layout + bucket-layout result.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-r4a}
timeout -k 10 400 python -u -m pytest tests/test_records_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "records tests failed"; tail -40 $O/pytest_$T.log; exit 1; }
tail -3 $O/pytest_$T.log
for lay in "records buckets" "columns dense" "records dense" "columns buckets"; do
  set -- $lay
  timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-general --layout $1 --output $2 > $O/bench_c4_${T}_$1_$2.json 2> $O/bench_c4_${T}_$1_$2.err || { echo "bench $lay failed"; tail -20 $O/bench_c4_${T}_$1_$2.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', d['phases_ms'], 'frac', round(d['roofline']['frac'],3))" $O/bench_c4_${T}_$1_$2.json "$lay"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_$T -o run -- python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-general > $O/prof_c4_$T.log 2>&1 || { echo "prof failed"; exit 3; }
f=$(find $O/prof_c4_$T -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" 20
echo "round ok"
