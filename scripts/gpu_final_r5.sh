#!/bin/bash
# Round-5 final records: the GPU suite and smoke, then every config's bench line, kernel trace and
# FETCH/WRITE passes (scripts/gpu_round.sh), the decode figures. Output under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r5z.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_r5z.log; exit 1; }
tail -1 $O/smoke_r5z.log
TAG=r5z CONFIG=c4 GENERAL_PMC=1 bash scripts/gpu_round.sh || exit 2
for c in c5 c1 c3; do NO_TESTS=1 TAG=r5z CONFIG=$c GENERAL_PMC=1 bash scripts/gpu_round.sh || exit 3; done
timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > $O/bench_decode_r5z.json 2> $O/bench_decode_r5z.err || exit 4
echo "final ok"
