#!/bin/bash
# Round 4 records: every config's bench line, kernel stats and PMC traffic (scripts/gpu_round.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in ${CONFIGS:-c4 c1 c3 c5}; do
  G=""; [ $c = c4 ] && G=1
  NO_TESTS=1 TAG=r4n CONFIG=$c GENERAL_PMC=$G bash scripts/gpu_round.sh > gpurun_out/round_r4n_$c.log 2>&1 || { echo "round $c failed"; tail -20 gpurun_out/round_r4n_$c.log; exit 1; }
  tail -2 gpurun_out/round_r4n_$c.log
done
echo "r4n ok"
