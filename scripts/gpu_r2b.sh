#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_cfg_r2b.log 2>&1 || { echo "cfg tests failed"; tail -40 $O/pytest_cfg_r2b.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest_cfg_r2b.log | tail -12
for c in c1 c4; do
timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 > $O/bench_${c}_r2b.json 2> $O/bench_${c}_r2b.err || { echo "bench $c failed"; tail -20 $O/bench_${c}_r2b.err; exit 2; }
cat $O/bench_${c}_r2b.json
done
