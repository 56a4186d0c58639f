#!/bin/bash
# Round 4: decode into its final buffer -- decode tests, then the decode leg of the C4 bench line.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_device_gpu.py tests/test_decode_gpu.py tests/test_encode_device_gpu.py tests/test_decode_merge_full_gpu.py -x -q -m gpu --timeout 150 --timeout-method thread > $O/pytest_r4r.log 2>&1
rc=$?; tail -2 $O/pytest_r4r.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc"; exit 1; }
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-general > $O/bench_r4r.json 2> $O/bench_r4r.err || { echo "bench failed"; tail -10 $O/bench_r4r.err; exit 2; }
python3 -c "import json; d=json.load(open('$O/bench_r4r.json')); l=d['decode_leg']; print(round(l['decode_ms'],1), {k:v for k,v in l['phases'].items() if not k.startswith('dd_')})"
timeout -k 10 400 python scripts/bench_decode.py --reps 3 > $O/bench_decode_r4r.json 2> $O/bench_decode_r4r.err || { tail -5 $O/bench_decode_r4r.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench_decode_r4r.json')); print(d['gpu_call_ms'], d['device_resident']['decode_to_hbm_ms'], {k:v for k,v in d['device_resident']['phases'].items() if not k.startswith('dd_')})"
echo "r4r ok"
