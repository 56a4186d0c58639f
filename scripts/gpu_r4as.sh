#!/bin/bash
# Early upload limited to snapshots of at most 512 MB: the decode bench (8 x 250 MB) and the C4 line
# with its decode leg (8 x 2 GB).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_decode_device_gpu.py tests/test_decode_gpu.py > $O/pytest_r4as.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest_r4as.log; exit 1; }
tail -1 $O/pytest_r4as.log
timeout -k 10 300 python scripts/bench_decode.py > $O/bench_decode_r4as.json 2> $O/bench_decode_r4as.err || { echo "decode bench failed"; exit 8; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_decode_r4as.json')); print('decode', d['device_resident']['decode_to_hbm_ms'])"
timeout -k 10 600 python bench.py > $O/bench_c4_r4as.json 2> $O/bench_c4_r4as.err || { echo "bench c4 failed"; tail -10 $O/bench_c4_r4as.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c4_r4as.json')); l=d['decode_leg']; print('c4', round(d['ms_per_step'],2), 'leg', l['decode_ms'], l['merge_ms'], l['phases']['index_ms'], l['phases']['deferred_datas_ms'])"
echo "r4as ok"
