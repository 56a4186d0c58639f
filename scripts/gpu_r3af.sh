#!/bin/bash
# Round 3: the chip-wide sort fold reads one 32-B record per child.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_sorted_runs_gpu.py tests/test_runs_oracle_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3af.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3af.log; exit 1; }
tail -2 gpurun_out/pytest_r3af.log
for c in c5 c3; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_r3af.json 2> gpurun_out/bench_${c}_r3af.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_${c}_r3af.err; exit 2; }
python -c "import json,sys; d=json.load(open('gpurun_out/bench_${c}_r3af.json')); print('$c', d['ms_per_step'], d['stats'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r3af -o run -- python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/prof_c5_r3af.log 2>&1 || { echo "prof failed"; exit 3; }
echo ok
