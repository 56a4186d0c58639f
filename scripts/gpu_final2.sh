#!/bin/bash
# End-of-round check: the whole GPU suite, smoke, the default bench line, the decode bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-r2z}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_$T.log | head -20; tail -3 $O/pytest_$T.log; exit 1; }
tail -1 $O/pytest_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_$T.log; exit 2; }
tail -1 $O/smoke_$T.log
timeout -k 10 500 python bench.py > $O/bench_default_$T.json 2> $O/bench_default_$T.err || { echo "bench failed"; tail -5 $O/bench_default_$T.err; exit 3; }
python3 -c "import json;d=json.load(open('$O/bench_default_$T.json'));print('bench',round(d['ms_per_step'],2),'%.3g'%d['value'],round(d['roofline']['frac'],4))"
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > $O/bench_decode_$T.json 2> $O/bench_decode_$T.err || { echo "decode bench failed"; exit 4; }
cat $O/bench_decode_$T.json
