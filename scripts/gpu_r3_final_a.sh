#!/bin/bash
# Round 3 record, part 1: the whole GPU suite, the smoke entry point, the decode bench and the
# C4 round (bench with CPU leg, kernel stats, PMC incl. the general-input passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3final.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_r3final.log; exit 1; }
tail -2 gpurun_out/pytest_r3final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3final.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r3final.log; exit 2; }
tail -2 gpurun_out/smoke_r3final.log
NO_TESTS=1 GENERAL_PMC=1 TAG=r3final CONFIG=c4 bash scripts/gpu_round.sh || exit 3
