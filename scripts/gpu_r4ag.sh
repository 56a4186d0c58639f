#!/bin/bash
# Per-run fold bookkeeping (scans over runs), one-pass batch planning: chip-wide tests, C5 / C3
# lines, the host planning clock.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runs_oracle_gpu.py \
  tests/test_configs_gpu.py tests/test_sorted_runs_gpu.py tests/test_records_gpu.py tests/test_gpu_parity.py > $O/pytest_r4ag.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4ag.log; exit 1; }
tail -1 $O/pytest_r4ag.log
for c in c5 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-general > $O/bench_${c}_r4ag.json 2> $O/bench_${c}_r4ag.err || { echo "bench $c failed"; tail -5 $O/bench_${c}_r4ag.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', d['phases_ms'])" $O/bench_${c}_r4ag.json $c
done
CDB_HOT_PROF=1 timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-general > $O/r4ag_prof.json 2> $O/r4ag_prof.err || exit 5
grep "over_capacity" $O/r4ag_prof.err | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_r4ag -o run -- python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-general > $O/prof_c5_r4ag.log 2>&1 || { echo "prof failed"; exit 6; }
echo "r4ag ok"
