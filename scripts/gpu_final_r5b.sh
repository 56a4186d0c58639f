#!/bin/bash
# Round-5 final records after the chip-wide direct-row fold: the GPU suite and smoke, then the C5
# and C3 rounds (bench line, kernel trace, FETCH/WRITE passes; scripts/gpu_round.sh).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r5y.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_r5y.log; exit 1; }
tail -1 $O/smoke_r5y.log
TAG=r5y CONFIG=c5 GENERAL_PMC=1 bash scripts/gpu_round.sh || exit 2
NO_TESTS=1 TAG=r5y CONFIG=c3 GENERAL_PMC=1 bash scripts/gpu_round.sh || exit 3
echo "final ok"
