#!/bin/bash
# Round records: for each config, bench line (CPU baseline with c4), kernel stats, PMC traffic.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for c in ${CONFIGS:-c4 c1 c3 c5}; do
  NO_TESTS=1 CONFIG=$c TAG=${TAG:-r2f} bash scripts/gpu_round.sh || { echo "round $c failed"; exit 1; }
done
