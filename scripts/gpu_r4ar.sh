#!/bin/bash
# Round 4 final records (after the chip-wide path work): the whole GPU suite, smoke, the C4 line
# with its CPU and decode legs, the C1 line, C4 kernel stats.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest_r4ar.log 2>&1
rc=$?; tail -3 $O/pytest_r4ar.log
[ $rc -le 1 ] || { echo "pytest ended with $rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r4ar.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_r4ar.log; exit 2; }
tail -1 $O/smoke_r4ar.log
timeout -k 10 600 python bench.py > $O/bench_c4_r4ar.json 2> $O/bench_c4_r4ar.err || { echo "bench c4 failed"; tail -10 $O/bench_c4_r4ar.err; exit 3; }
timeout -k 10 300 python bench.py --config c1 > $O/bench_c1_r4ar.json 2> $O/bench_c1_r4ar.err || { echo "bench c1 failed"; tail -10 $O/bench_c1_r4ar.err; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_r4ar -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-general --no-decode-leg > $O/prof_c4_r4ar.log 2>&1 || { echo "prof c4 failed"; exit 5; }
for c in c1 c4; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms frac', round(r['frac'],3), 'traffic x', r['traffic_over_alg'] and round(r['traffic_over_alg'],2), 'cpu', round(d['cpu_baseline']['value']/1e6,2))" $O/bench_${c}_r4ar.json $c
done
echo "r4ar ok (pytest rc=$rc)"
