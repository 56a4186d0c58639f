#!/bin/bash
# Round 3: GPU suite (sharded merge, decode-produced runs), C4 bench with the general-input figures,
# kernel stats and PMC traffic of both paths, the single-process sharded bench on one GPU (2 slots).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_shard_gpu.py tests/test_runs_oracle_gpu.py tests/test_decode_device_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r3b_new.log 2>&1 || { echo "new tests failed"; tail -40 gpurun_out/pytest_r3b_new.log; exit 1; }
tail -3 gpurun_out/pytest_r3b_new.log
GENERAL_PMC=1 TAG=r3b CONFIG=c4 bash scripts/gpu_round.sh || exit 2
timeout -k 10 300 python bench.py --single-process --devices 0,0 --universe-per-gpu 31250000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sp_r3b.json 2> gpurun_out/bench_sp_r3b.err || { echo "single-process bench failed"; tail -20 gpurun_out/bench_sp_r3b.err; exit 3; }
cat gpurun_out/bench_sp_r3b.json
