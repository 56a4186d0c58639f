#!/bin/bash
# One parameterised GPU recipe (replaces the per-experiment gpu_r3*/gpu_r4* scripts).
# Every step is optional and bounded by its own timeout; the first failure ends the call.
#   TAG      name prefix of every output under gpurun_out/
#   TESTS    pytest arguments (e.g. "tests/test_runs_oracle_gpu.py"); KEXPR: a -k expression
#   BENCHES  ";"-separated "name|ENV=v ENV2=w|bench.py arguments"
#   PROF     "name|ENV=v|bench.py arguments": rocprofv3 --kernel-trace --stats of that command
#   PMC      ";"-separated "name|ENV=v|bench.py arguments|COUNTERS": one rocprofv3 --pmc pass per
#            counter group ("," separates groups, " " the counters of one group), summarised per kernel
#   SMOKE    non-empty: __graft_entry__.smoke() at the end
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
T=${TAG:-exp}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -q --timeout ${TEST_CASE_TIMEOUT:-300} --timeout-method thread $TESTS ${KEXPR:+-k "$KEXPR"} > $O/pytest_$T.log 2>&1
  rc=$?
  tail -3 $O/pytest_$T.log
  [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest_$T.log | head -20; exit 1; }
fi
if [ -n "$BENCHES" ]; then
  IFS=';' read -ra BS <<< "$BENCHES"
  for b in "${BS[@]}"; do
    IFS='|' read -r name envs args <<< "$b"
    env $envs timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $args > $O/bench_${T}_$name.json 2> $O/bench_${T}_$name.err
    rc=$?
    [ $rc -eq 0 ] || { echo "bench $name failed rc=$rc"; tail -8 $O/bench_${T}_$name.err; exit 2; }
    python3 - "$O/bench_${T}_$name.json" "$name" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], d["config"].get("workload", ""), "ms", round(d["ms_per_step"], 3), "frac", round(r.get("frac") or 0, 4),
      "value", "%.4g" % d["value"])
EOF
  done
fi
if [ -n "$PROF" ]; then
  IFS='|' read -r name envs args <<< "$PROF"
  [ -n "$envs" ] && export $envs
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$name -o run -- python3 bench.py $args > $O/prof_${T}_$name.log 2>&1 || { echo "prof failed"; tail -5 $O/prof_${T}_$name.log; exit 3; }
  f=$(find $O/prof_${T}_$name -name '*kernel_stats.csv' -print -quit)
  [ -n "$f" ] && python3 scripts/kstats.py "$f" 16
fi
if [ -n "$PMC" ]; then
  IFS=';' read -ra PS <<< "$PMC"
  for spec in "${PS[@]}"; do
    IFS='|' read -r name envs args groups <<< "$spec"
    IFS=',' read -ra GS <<< "$groups"
    i=0
    for g in "${GS[@]}"; do
      env $envs timeout -s KILL 200 rocprofv3 --pmc $g --kernel-include-regex "${PMC_REGEX:-bucket_wave}" --output-format csv -d $O/pmc_${T}_${name}/pass$i -o run -- python3 bench.py $args > $O/pmc_${T}_${name}_$i.log 2>&1 || { echo "pmc $name $g failed"; tail -5 $O/pmc_${T}_${name}_$i.log; exit 4; }
      i=$((i + 1))
    done
    python3 scripts/pmc_summary.py $O/pmc_${T}_${name} > $O/pmc_${T}_${name}.txt && cat $O/pmc_${T}_${name}.txt
  done
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_$T.log; exit 5; }
  tail -1 $O/smoke_$T.log
fi
echo "$T ok"
