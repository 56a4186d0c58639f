#!/bin/bash
# Round 3: one bucket range when a bucket exceeds the wide tier (C5), runs tests, C5/C4 timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sorted_runs_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3v.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3v.log; exit 1; }
tail -2 gpurun_out/pytest_r3v.log
for c in c4 c5; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_r3v.json 2> gpurun_out/bench_${c}_r3v.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_${c}_r3v.err; exit 2; }
python3 -c "import json;a=json.load(open('gpurun_out/bench_${c}_r3v.json'));print('$c', round(a['ms_per_step'],3), a['phases_ms'])"
done
