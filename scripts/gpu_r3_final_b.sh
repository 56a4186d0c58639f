#!/bin/bash
# Round 3 record, part 2: C5 and C3 rounds (bench with CPU leg, kernel stats, PMC).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c5 c3; do
NO_TESTS=1 TAG=r3final CONFIG=$c bash scripts/gpu_round.sh || exit 1
done
