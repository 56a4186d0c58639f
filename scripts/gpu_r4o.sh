#!/bin/bash
# Round 4: records-aware partition loads -- tests + the general-input (partition path) bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_records_gpu.py tests/test_shard_gpu.py tests/test_gpu_parity.py tests/test_decode_device_gpu.py -x -q -m gpu --timeout 150 --timeout-method thread > $O/pytest_r4o.log 2>&1
rc=$?; tail -2 $O/pytest_r4o.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc"; exit 1; }
for lay in records columns; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --input-order hash-random --layout $lay > $O/o_$lay.json 2> $O/o_$lay.err || { echo "bench $lay failed"; tail -5 $O/o_$lay.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()})" $O/o_$lay.json "$lay"
done
echo "r4o ok"
