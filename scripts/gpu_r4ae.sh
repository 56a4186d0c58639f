#!/bin/bash
# Chunked tag kernel, blocked radix histogram: chip-wide tests, C5 / C3 lines, a C5 kernel + HIP API
# trace (the host gap before the chip-wide batches).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runs_oracle_gpu.py \
  tests/test_configs_gpu.py tests/test_sorted_runs_gpu.py tests/test_decode_device_gpu.py > $O/pytest_r4ae.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4ae.log; exit 1; }
tail -1 $O/pytest_r4ae.log
for c in c5 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-general > $O/bench_${c}_r4ae.json 2> $O/bench_${c}_r4ae.err || { echo "bench $c failed"; tail -5 $O/bench_${c}_r4ae.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', d['phases_ms'])" $O/bench_${c}_r4ae.json $c
done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/prof_c5_r4ae -o run -- python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-general > $O/prof_c5_r4ae.log 2>&1 || { echo "prof failed"; exit 5; }
echo "r4ae ok"
