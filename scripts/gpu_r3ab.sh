#!/bin/bash
# Round 3: per-bucket LDS radix sort of small chip-wide buckets: parity, C3/C5 timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_configs_gpu.py tests/test_runs_oracle_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3ab.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3ab.log; exit 1; }
tail -2 gpurun_out/pytest_r3ab.log
for c in c5 c3; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_r3ab.json 2> gpurun_out/bench_${c}_r3ab.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_${c}_r3ab.err; exit 2; }
python3 -c "import json;a=json.load(open('gpurun_out/bench_${c}_r3ab.json'));print('$c', round(a['ms_per_step'],3), a['phases_ms'])"
done
