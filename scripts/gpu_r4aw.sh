#!/bin/bash
# Tag kernel with its buckets' key tables in LDS: chip-wide tests, C5 / C3 lines.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runs_oracle_gpu.py tests/test_gpu_parity.py \
  tests/test_configs_gpu.py tests/test_records_gpu.py tests/test_sorted_runs_gpu.py -k "not full_c4" > $O/pytest_r4aw.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4aw.log; exit 1; }
tail -1 $O/pytest_r4aw.log
for c in c5 c3; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --no-general > $O/bench_${c}_r4aw.json 2> $O/bench_${c}_r4aw.err || { echo "bench $c failed"; tail -5 $O/bench_${c}_r4aw.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms')" $O/bench_${c}_r4aw.json $c
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_r4aw -o run -- python bench.py --config c5 --no-cpu-baseline --no-general > $O/prof_c5_r4aw.log 2>&1 || { echo "prof failed"; exit 5; }
echo "r4aw ok"
