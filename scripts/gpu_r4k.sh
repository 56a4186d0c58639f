#!/bin/bash
# Round 4: decode tests + bench + trace after the walk-result download moved behind the sync.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_decode_device_gpu.py tests/test_decode_gpu.py tests/test_encode_device_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4k.log 2>&1
rc=$?; tail -2 $O/pytest_r4k.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc"; exit 1; }
timeout -k 10 400 python scripts/bench_decode.py --reps 3 > $O/bench_decode_r4k.json 2> $O/bench_decode_r4k.err || { tail -5 $O/bench_decode_r4k.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench_decode_r4k.json')); print(d['gpu_call_ms'], d['device_resident']['decode_to_hbm_ms'], d['device_resident']['phases'], d['decode_plus_merge'])"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_dec_r4k -o run -- python scripts/bench_decode.py --reps 1 > $O/prof_dec_r4k.log 2>&1 || { echo "decode prof failed"; exit 4; }
echo "r4k ok"
