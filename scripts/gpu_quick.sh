#!/bin/bash
# Quick GPU iteration: parity tests, then the full bench and a kernel-trace profile of it.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-q}
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_$T.log; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed"; tail -20 $O/bench_$T.err; exit 2; }
cat $O/bench_$T.json
if [ -z "$NO_PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$T.log 2>&1 || { echo "prof failed"; exit 3; }
python3 - <<PY
import csv
for r in csv.DictReader(open('$O/prof_$T/run_kernel_stats.csv')):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
fi
echo "quick ok"
