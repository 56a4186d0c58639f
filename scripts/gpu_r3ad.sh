#!/bin/bash
# Round 3: byte references of a device decode kept in HBM until a dump/encode asks.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_decode_device_gpu.py tests/test_runs_oracle_gpu.py tests/test_encode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3ad.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3ad.log; exit 1; }
tail -2 gpurun_out/pytest_r3ad.log
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > gpurun_out/bench_decode_r3ad.json 2> gpurun_out/bench_decode_r3ad.err || { echo "decode bench failed"; tail -20 gpurun_out/bench_decode_r3ad.err; exit 2; }
cat gpurun_out/bench_decode_r3ad.json
