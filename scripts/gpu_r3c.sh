#!/bin/bash
# Round 3: chip-wide child path with per-bucket sorts and the LDS-staged radix scatter:
# GPU suite, then C3 and C5 bench + kernel stats + PMC traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r3c CONFIG=c3 bash scripts/gpu_round.sh || exit 1
NO_TESTS=1 TAG=r3c CONFIG=c5 bash scripts/gpu_round.sh || exit 2
