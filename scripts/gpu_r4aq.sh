#!/bin/bash
# Decode: prepare halves queued for every snapshot before one synchronisation, pinned small words.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_decode_device_gpu.py tests/test_decode_gpu.py tests/test_abi_decode.py tests/test_ops_decode_gpu.py tests/test_decode_merge_full_gpu.py tests/test_abi_c.py tests/test_encode_device_gpu.py tests/test_runs_oracle_gpu.py -k "not full_c4" > $O/pytest_r4aq.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4aq.log; exit 1; }
tail -1 $O/pytest_r4aq.log
CDB_DECODE_TRACE=$O/dec_trace_r4aq.jsonl timeout -k 10 300 python scripts/bench_decode.py > $O/bench_decode_r4aq.json 2> $O/bench_decode_r4aq.err || { echo "decode bench failed"; tail -5 $O/bench_decode_r4aq.err; exit 8; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_decode_r4aq.json')); p=d['device_resident']['phases']; print('decode', d['device_resident']['decode_to_hbm_ms'], {k:p[k] for k in ['index_ms','deferred_datas_ms','prepare_device_ms','order_sort_ms','emit_ms']})"
echo "r4aq ok"
