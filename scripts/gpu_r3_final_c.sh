#!/bin/bash
# Round 3 record, part 3: C1 round and the decode bench (8 snapshots into HBM).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NO_TESTS=1 TAG=r3final CONFIG=c1 bash scripts/gpu_round.sh || exit 1
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > gpurun_out/bench_decode_r3final.json 2> gpurun_out/bench_decode_r3final.err || { echo "decode bench failed"; tail -20 gpurun_out/bench_decode_r3final.err; exit 2; }
cat gpurun_out/bench_decode_r3final.json
