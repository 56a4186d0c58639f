#!/bin/bash
# Round 3: chip-wide batches split by size class (libcdbmerge.so) against one batch per kind
# (libcdbmerge_nosplit.so, swapped in for the second pair of benches).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_sorted_runs_gpu.py tests/test_runs_oracle_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3ah.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3ah.log; exit 1; }
tail -2 gpurun_out/pytest_r3ah.log
for v in split nosplit; do
if [ $v = nosplit ]; then cp constdb_amd/libcdbmerge_nosplit.so constdb_amd/libcdbmerge.so; fi
for c in c5 c3; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_${v}_r3ah.json 2> gpurun_out/bench_${c}_${v}_r3ah.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_${c}_${v}_r3ah.err; exit 2; }
python -c "import json,sys; d=json.load(open('gpurun_out/bench_${c}_${v}_r3ah.json')); print('$v $c', d['ms_per_step'], d['phases_ms'])"
done
done
echo ok
