#!/bin/bash
# Chip-wide path with the per-bucket LDS sort and fold: the chip-wide / run-order / shard tests,
# then C3 and C5 bench lines and their kernel stats.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runs_oracle_gpu.py \
  tests/test_configs_gpu.py tests/test_sorted_runs_gpu.py tests/test_records_gpu.py tests/test_shard_gpu.py \
  tests/test_gpu_parity.py > $O/pytest_r4w.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4w.log; exit 1; }
tail -2 $O/pytest_r4w.log
for c in c3 c5; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_${c}_r4w.json 2> $O/bench_${c}_r4w.err || { echo "bench $c failed"; tail -10 $O/bench_${c}_r4w.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', d['phases_ms'])" $O/bench_${c}_r4w.json $c
done
for c in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_r4w -o prof -- python bench.py --config $c --no-cpu-baseline --no-general > $O/prof_${c}_r4w.log 2>&1 || { echo "prof $c failed"; tail -5 $O/prof_${c}_r4w.log; exit 5; }
done
echo "r4w ok"
