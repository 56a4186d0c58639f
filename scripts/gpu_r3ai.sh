#!/bin/bash
# Round 3: single-pass look-back scans + size-class batches (libcdbmerge.so), then the same
# benches with size-class batches only (libcdbmerge_split.so) and neither (libcdbmerge_nosplit.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python bench.py --config c1 --steps 3 --warmup 1 --no-cpu-baseline --no-general > gpurun_out/bench_c1_r3ai.json 2> gpurun_out/bench_c1_r3ai.err || { echo "canary failed"; tail -20 gpurun_out/bench_c1_r3ai.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c1_r3ai.json')); print('c1', d['ms_per_step'])"
timeout -k 10 700 python -u -m pytest tests/test_sorted_runs_gpu.py tests/test_runs_oracle_gpu.py tests/test_configs_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3ai.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3ai.log; exit 2; }
tail -2 gpurun_out/pytest_r3ai.log
for v in lb split nosplit; do
if [ $v != lb ]; then cp constdb_amd/libcdbmerge_$v.so constdb_amd/libcdbmerge.so; fi
cs="c5 c3 c4"; if [ $v = nosplit ]; then cs="c5 c3"; fi
for c in $cs; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_${v}_r3ai.json 2> gpurun_out/bench_${c}_${v}_r3ai.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_${c}_${v}_r3ai.err; exit 3; }
python -c "import json,sys; d=json.load(open('gpurun_out/bench_${c}_${v}_r3ai.json')); print('$v $c', d['ms_per_step'], d['phases_ms'], d['stats'].get('hot_slow_runs'))"
done
done
echo ok
