#!/bin/bash
# Round 3: the decode's device entry index with the wave-parallel, bounded sync search.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_decode_device_gpu.py tests/test_decode_gpu.py tests/test_index_parallel.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3o.log 2>&1 || { echo "decode tests failed"; tail -30 gpurun_out/pytest_r3o.log; exit 1; }
tail -2 gpurun_out/pytest_r3o.log
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > gpurun_out/bench_decode_r3o.json 2> gpurun_out/bench_decode_r3o.err || { echo "decode bench failed"; tail -20 gpurun_out/bench_decode_r3o.err; exit 2; }
cat gpurun_out/bench_decode_r3o.json
