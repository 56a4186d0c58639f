#!/bin/bash
# Round 4: decode (LDS-window index walk, coalesced record pass) and wave-kernel (no staging,
# overlapped directory loads, DPP run scan) checks and measurements.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_device_gpu.py tests/test_decode_gpu.py tests/test_records_gpu.py tests/test_runs_oracle_gpu.py tests/test_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4g.log 2>&1
rc=$?; tail -4 $O/pytest_r4g.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc"; exit 1; }
for lay in records columns; do
  CDB_LIB=$PWD/variants/lib_nounroll.so timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-general --layout $lay > $O/g_nounroll_$lay.json 2> $O/g_nounroll_$lay.err || { echo "bench nounroll $lay failed"; tail -5 $O/g_nounroll_$lay.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()})" $O/g_nounroll_$lay.json "nounroll $lay"
  timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-general --layout $lay > $O/g_$lay.json 2> $O/g_$lay.err || { echo "bench $lay failed"; tail -5 $O/g_$lay.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()})" $O/g_$lay.json "$lay"
done
timeout -k 10 400 python scripts/bench_decode.py --reps 2 > $O/bench_decode_r4g.json 2> $O/bench_decode_r4g.err || { tail -5 $O/bench_decode_r4g.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench_decode_r4g.json')); print(d['device_resident']['decode_to_hbm_ms'], d['device_resident']['phases'], d['decode_plus_merge'])"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_dec_r4g -o run -- python scripts/bench_decode.py --reps 1 > $O/prof_dec_r4g.log 2>&1 || { echo "decode prof failed"; exit 4; }
echo "r4g ok"
