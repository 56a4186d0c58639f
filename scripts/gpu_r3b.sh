#!/bin/bash
# Round 3: GPU suite (sharded merge, decode-produced runs, variant cleanup), C4 bench with the
# general-input figures, kernel stats and PMC traffic of both paths, the single-process sharded
# bench on one GPU (2 slots).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
GENERAL_PMC=1 TAG=r3b CONFIG=c4 bash scripts/gpu_round.sh || exit 2
timeout -k 10 300 python bench.py --single-process --devices 0,0 --universe-per-gpu 31250000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sp_r3b.json 2> gpurun_out/bench_sp_r3b.err || { echo "single-process bench failed"; tail -20 gpurun_out/bench_sp_r3b.err; exit 3; }
cat gpurun_out/bench_sp_r3b.json
