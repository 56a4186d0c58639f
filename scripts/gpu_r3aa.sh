#!/bin/bash
# Round 3: C3 and C5 records after the runs-mode chip-wide path (bench with CPU leg, kernel stats, PMC).
set -o pipefail
cd $GRAFT_REPO_ROOT
NO_TESTS=1 TAG=r3aa CONFIG=c3 bash scripts/gpu_round.sh || exit 1
NO_TESTS=1 TAG=r3aa CONFIG=c5 bash scripts/gpu_round.sh || exit 2
