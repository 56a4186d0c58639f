#!/bin/bash
# One GPU verification round: parity tests, full bench (with CPU baseline), kernel-trace
# stats of the same bench command, FETCH/WRITE PMC passes for the HBM traffic figure.
# Usage (from gpurun): TAG=r1e bash scripts/gpu_round.sh
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-r1e}
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $O/bench_full_$T.json 2> $O/bench_full_$T.err || { echo "bench failed"; exit 2; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$T.log 2>&1 || { echo "prof failed"; exit 3; }
if [ -z "$NO_PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-bucket_|part_|compact}" --output-format csv -d $O/pmc_${T}_$c -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_${T}_$c.log 2>&1 || { echo "pmc $c failed"; exit 4; }
  done
python3 scripts/pmc_traffic.py $O/pmc_${T}_FETCH_SIZE $O/pmc_${T}_WRITE_SIZE $O/pmc_traffic_$T.json || exit 5
fi
echo "round ok"
