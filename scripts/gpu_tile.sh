#!/bin/bash
# Sorted-run parity tests, then the C4 bench per staged-tile width (CDB_TILE_NW).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-tile}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 400 python -u -m pytest ${FILES:-tests/test_sorted_runs_gpu.py tests/test_configs_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_$T.log; exit 1; }
tail -1 $O/pytest_$T.log
fi
for nw in ${NWS:-0 4 8 16}; do
  CDB_TILE_NW=$nw timeout -k 10 300 python bench.py --config ${CONFIG:-c4} --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_${T}_$nw.json 2> $O/bench_${T}_$nw.err || { echo "bench nw=$nw failed"; tail -5 $O/bench_${T}_$nw.err; exit 2; }
  python3 -c "import json;d=json.load(open('$O/bench_${T}_$nw.json'));print('nw=$nw',d['ms_per_step'],{k:round(x,2) for k,x in d['phases_ms'].items()})"
done
