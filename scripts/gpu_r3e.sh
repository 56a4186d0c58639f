#!/bin/bash
# Round 3: GPU suite after the decode index and the chip-wide revert; decode bench (8 snapshots
# into HBM); C3 and C5 bench + kernel stats + merge-only PMC traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r3e CONFIG=c3 bash scripts/gpu_round.sh || exit 1
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > gpurun_out/bench_decode_r3e.json 2> gpurun_out/bench_decode_r3e.err || { echo "decode bench failed"; tail -20 gpurun_out/bench_decode_r3e.err; exit 2; }
cat gpurun_out/bench_decode_r3e.json
NO_TESTS=1 TAG=r3e CONFIG=c5 bash scripts/gpu_round.sh || exit 3
