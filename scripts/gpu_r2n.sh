#!/bin/bash
# Compaction rewrite check: parity tests, bench at P=1/8, then TA/TD counters of the tile kernel.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_r2n.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_r2n.log | head -20; tail -5 $O/pytest_r2n.log; exit 1; }
tail -1 $O/pytest_r2n.log
for pp in 1 8; do
  CDB_PIPE=$pp timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_r2n_$pp.json 2> $O/bench_r2n_$pp.err || { echo "bench failed"; tail -5 $O/bench_r2n_$pp.err; exit 2; }
  python3 -c "import json;d=json.load(open('$O/bench_r2n_$pp.json'));print('P=$pp',round(d['ms_per_step'],2),{k:round(x,2) for k,x in d['phases_ms'].items()})"
done
for nw in 4 8; do
  CDB_PIPE=1 CDB_TILE_NW=$nw TAG=ta_tile$nw KREGEX="bucket_tile|compact" bash scripts/pmc_ta.sh 2>&1 | grep -E "cdb::" || exit 3
done
