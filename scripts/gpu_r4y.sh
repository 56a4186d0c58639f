#!/bin/bash
# Radix sort with the tile's loads in flight and LDS-staged contiguous writes: the tests that sort
# (chip-wide global path, decoder order sort), C5 / C3 bench lines, the decode bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runs_oracle_gpu.py \
  tests/test_configs_gpu.py tests/test_decode_merge_full_gpu.py -k "not full_c4" > $O/pytest_r4y.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4y.log; exit 1; }
tail -1 $O/pytest_r4y.log
for c in c5 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-general > $O/bench_${c}_r4y.json 2> $O/bench_${c}_r4y.err || { echo "bench $c failed"; tail -5 $O/bench_${c}_r4y.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', d['phases_ms'])" $O/bench_${c}_r4y.json $c
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_r4y -o run -- python bench.py --config c5 --no-cpu-baseline --no-general > $O/prof_c5_r4y.log 2>&1 || { echo "prof failed"; exit 5; }
timeout -k 10 300 python scripts/bench_decode.py > $O/bench_decode_r4y.json 2> $O/bench_decode_r4y.err || { echo "decode bench failed"; tail -5 $O/bench_decode_r4y.err; exit 6; }
tail -c 600 $O/bench_decode_r4y.json
echo "r4y ok"
