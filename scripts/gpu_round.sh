#!/bin/bash
# One GPU verification round: parity tests, FETCH/WRITE PMC passes for the HBM traffic figure,
# the full bench (with CPU baseline; it reads the traffic file just written), kernel-trace stats of
# the same bench command, the timed step's timeline and step-only kernel stats.
# Usage (from gpurun): TAG=r6 CONFIG=c4 bash scripts/gpu_round.sh
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-r6}
C=${CONFIG:-c4}
O=gpurun_out
P=profiles/${PROFILE_ROUND:-r06}   # (the box's copy of the tree: bench.py reads the traffic file here)
mkdir -p $P
KRE="merge_begin_marker|merge_end_marker|pipe_|iota|set_dir|stamp_pos|part_|bucket_|compact|scan_|stats_reduce|gc_lastbad|hot_|sorted_|seg_|run_|mat_|radix_hist|radix_scatter"
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_$T.log; exit 1; }
tail -2 $O/pytest_$T.log
fi
if [ -z "$NO_PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv -d $O/pmc_${C}_${T}_$c -o run -- python bench.py --config $C --steps 1 --warmup 0 --no-cpu-baseline --no-general --no-decode-leg > $O/pmc_${C}_${T}_$c.log 2>&1 || { echo "pmc $c failed"; exit 4; }
  done
  python3 scripts/pmc_traffic.py $O/pmc_${C}_${T}_FETCH_SIZE $O/pmc_${C}_${T}_WRITE_SIZE $O/pmc_traffic_${C}_$T.json || exit 5
  cp $O/pmc_traffic_${C}_$T.json $P/pmc_traffic_${C}.json
  if [ -n "$GENERAL_PMC" ]; then
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv -d $O/pmcg_${C}_${T}_$c -o run -- python bench.py --config $C --steps 1 --warmup 0 --no-cpu-baseline --no-decode-leg --input-order hash-random > $O/pmcg_${C}_${T}_$c.log 2>&1 || { echo "pmc general $c failed"; exit 6; }
    done
    python3 scripts/pmc_traffic.py $O/pmcg_${C}_${T}_FETCH_SIZE $O/pmcg_${C}_${T}_WRITE_SIZE $O/pmc_traffic_${C}_general_$T.json || exit 7
    cp $O/pmc_traffic_${C}_general_$T.json $P/pmc_traffic_${C}_general.json
  fi
fi
timeout -k 10 500 python bench.py --config $C --steps 5 --warmup 2 > $O/bench_${C}_$T.json 2> $O/bench_${C}_$T.err || { echo "bench failed"; tail -20 $O/bench_${C}_$T.err; exit 2; }
cat $O/bench_${C}_$T.json
# (no general or decode leg: the last five marker-bracketed merges are the five timed steps)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${C}_$T -o run -- python bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --no-general --no-decode-leg > $O/prof_${C}_$T.log 2>&1 || { echo "prof failed"; exit 3; }
python3 scripts/timeline.py $O/prof_${C}_$T --stats $O/step_stats_${C}_$T.csv --last 5 > $O/timeline_${C}_step_$T.txt || exit 8
echo "round ok"
