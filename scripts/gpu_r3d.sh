#!/bin/bash
# (CDB_EXP_NO_LOCAL was a temporary switch of this experiment; the per-bucket sorts it compared were removed)
# Round 3 experiment: per-bucket LDS sorts (1024 threads, sized) vs the global radix sort for the
# chip-wide child path (C3, C5), the chip-wide tests, and the selection-loop hazard program.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 tests/hazard/build/select_loop 4194304 > gpurun_out/hazard_r3d.json || { echo "hazard failed"; exit 1; }
cat gpurun_out/hazard_r3d.json
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_decode_device_gpu.py tests/test_runs_oracle_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3d.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3d.log; exit 2; }
tail -2 gpurun_out/pytest_r3d.log
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_r3d_local.json 2> gpurun_out/bench_${c}_r3d_local.err || { echo "bench $c failed"; exit 3; }
  CDB_EXP_NO_LOCAL=1 timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_r3d_global.json 2> gpurun_out/bench_${c}_r3d_global.err || { echo "bench $c global failed"; exit 4; }
  python3 -c "import json;a=json.load(open('gpurun_out/bench_${c}_r3d_local.json'));b=json.load(open('gpurun_out/bench_${c}_r3d_global.json'));print('$c local',a['ms_per_step'],'global',b['ms_per_step'])"
done
