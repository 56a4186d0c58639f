#!/bin/bash
# Phase clocks of hot_sortfold_kernel on C3 and C5 (CDB_HOT_PROF).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runs_oracle_gpu.py -k "chip_wide or c5 or c3 or forced or random" > $O/pytest_r4x.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4x.log; exit 1; }
tail -1 $O/pytest_r4x.log
for c in c3 c5; do
  CDB_HOT_PROF=1 timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-general > $O/bench_${c}_r4x.json 2> $O/bench_${c}_r4x.err || { echo "bench $c failed"; tail -10 $O/bench_${c}_r4x.err; exit 4; }
  grep hot_sortfold $O/bench_${c}_r4x.err | tail -3
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-general > $O/bench_${c}_r4x2.json 2>&1 || exit 5
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms')" $O/bench_${c}_r4x2.json $c
done
echo "r4x ok"
