#!/bin/bash
# Round-3 first check: GPU suite, then C3 (shared key types + Deletes) and C4 bench/profile/PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=r3a CONFIG=c3 bash scripts/gpu_round.sh || exit 1
NO_TESTS=1 TAG=r3a CONFIG=c4 bash scripts/gpu_round.sh || exit 2
