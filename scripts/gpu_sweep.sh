#!/bin/bash
# GPU tests (FILES, default: the whole suite), then the bench under each setting of an
# environment knob: VAR=name VALS="a b c" CONFIG=c4 TAG=x bash scripts/gpu_sweep.sh
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-sweep}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 700 python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_$T.log | head -20; tail -5 $O/pytest_$T.log; exit 1; }
tail -1 $O/pytest_$T.log
fi
for v in ${VALS:-default}; do
  if [ "$v" != default ]; then export $VAR=$v; fi
  for c in ${CONFIGS:-c4}; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_${T}_${c}_$v.json 2> $O/bench_${T}_${c}_$v.err || { echo "bench $c $v failed"; tail -5 $O/bench_${T}_${c}_$v.err; exit 2; }
    python3 -c "import json;d=json.load(open('$O/bench_${T}_${c}_$v.json'));print('$c $VAR=$v',round(d['ms_per_step'],2),{k:round(x,2) for k,x in d['phases_ms'].items()})"
  done
done
