#!/bin/bash
# Round 3: GPU suite after the device re-walk rounds of the decode index, run_mark4 + per-family
# run directories and the fixed wide-tier grid; decode bench (8 snapshots into HBM); C4 round with
# the general-input PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3h.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_r3h.log; exit 1; }
tail -2 gpurun_out/pytest_r3h.log
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > gpurun_out/bench_decode_r3h.json 2> gpurun_out/bench_decode_r3h.err || { echo "decode bench failed"; tail -20 gpurun_out/bench_decode_r3h.err; exit 2; }
cat gpurun_out/bench_decode_r3h.json
NO_TESTS=1 GENERAL_PMC=1 TAG=r3h CONFIG=c4 bash scripts/gpu_round.sh || exit 3
