#!/bin/bash
# Whole GPU suite, decode bench (8 snapshots into HBM), C4 bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-r2o}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_$T.log | head -20; tail -5 $O/pytest_$T.log; exit 1; }
tail -1 $O/pytest_$T.log
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > $O/bench_decode_$T.json 2> $O/bench_decode_$T.err || { echo "decode bench failed"; tail -5 $O/bench_decode_$T.err; exit 2; }
cat $O/bench_decode_$T.json
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4_$T.json 2> $O/bench_c4_$T.err || { echo "bench failed"; tail -5 $O/bench_c4_$T.err; exit 3; }
python3 -c "import json;d=json.load(open('$O/bench_c4_$T.json'));print('c4',round(d['ms_per_step'],2),{k:round(x,2) for k,x in d['phases_ms'].items()})"
