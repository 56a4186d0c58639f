#!/bin/bash
# Round 4 final records on the final code: the whole GPU suite, smoke, every config's bench line
# (CPU baselines, general-path figures, C4 decode leg), C5 / C4 kernel stats.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest_r4av.log 2>&1
rc=$?; tail -2 $O/pytest_r4av.log
[ $rc -le 1 ] || { echo "pytest ended with $rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r4av.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_r4av.log; exit 2; }
tail -1 $O/smoke_r4av.log
timeout -k 10 600 python bench.py > $O/bench_c4_r4av.json 2> $O/bench_c4_r4av.err || { echo "bench c4 failed"; tail -10 $O/bench_c4_r4av.err; exit 3; }
for c in c1 c3 c5; do
  timeout -k 10 500 python bench.py --config $c > $O/bench_${c}_r4av.json 2> $O/bench_${c}_r4av.err || { echo "bench $c failed"; tail -10 $O/bench_${c}_r4av.err; exit 4; }
done
for c in c1 c3 c4 c5; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms frac', round(r['frac'],3), 'traffic x', r['traffic_over_alg'] and round(r['traffic_over_alg'],2), 'cpu', round(d['cpu_baseline']['value']/1e6,2))" $O/bench_${c}_r4av.json $c
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_r4av -o run -- python bench.py --config c5 --no-cpu-baseline --no-general > $O/prof_c5_r4av.log 2>&1 || { echo "prof c5 failed"; exit 5; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_r4av -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-general --no-decode-leg > $O/prof_c4_r4av.log 2>&1 || { echo "prof c4 failed"; exit 6; }
echo "r4av ok (pytest rc=$rc)"
