#!/bin/bash
# Round 4: GPU tests of the new paths, the layout benches + kernel stats, wave-kernel counters, the
# encode bench (host view vs from HBM) and the decode bench (phases + kernel / copy trace).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 800 python -u -m pytest ${TESTS:-tests/test_encode_device_gpu.py tests/test_decode_device_gpu.py tests/test_abi_c.py tests/test_records_gpu.py tests/test_golden.py tests/test_runs_oracle_gpu.py tests/test_dist_gpu.py tests/test_shard_gpu.py tests/test_sorted_runs_gpu.py} -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4e.log 2>&1
rc=$?
tail -3 $O/pytest_r4e.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest ended with $rc"; exit 1; }
NO_TESTS=1 bash scripts/gpu_r4b.sh || exit 2
timeout -k 10 300 python scripts/bench_encode.py > $O/bench_encode_r4.json 2> $O/bench_encode_r4.err || { tail -5 $O/bench_encode_r4.err; exit 3; }
timeout -k 10 400 python scripts/bench_decode.py --reps 2 > $O/bench_decode_r4.json 2> $O/bench_decode_r4.err || { tail -5 $O/bench_decode_r4.err; exit 4; }
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_dec_r4 -o run -- python scripts/bench_decode.py --reps 1 > $O/prof_dec_r4.log 2>&1 || { echo "decode prof failed"; exit 5; }
TAG=r4d_rec BENCH_ARGS="--layout records" bash scripts/gpu_r4d.sh || exit 6
TAG=r4d_col BENCH_ARGS="--layout columns" bash scripts/gpu_r4d.sh || exit 7
echo "r4e ok"
