#!/bin/bash
# Round-5 final records: smoke, the GPU suite with the first config's round, then every config's
# bench line, kernel trace and FETCH/WRITE passes (scripts/gpu_round.sh), the decode figures.
#   CONFIGS  configs in order (default "c4 c5 c1 c3"); the first one also runs the GPU suite
#   DECODE   non-empty: scripts/bench_decode.py --device-snapshots 8 at the end
#   TAG      output name suffix (default r5z); NO_TESTS: no GPU suite
# Output under gpurun_out/. (The records: TAG=r5z with the default configs and DECODE=1, then
# TAG=r5y CONFIGS="c5 c3" after the chip-wide direct-row fold.)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
T=${TAG:-r5z}
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke_$T.log; exit 1; }
tail -1 $O/smoke_$T.log
first=1
for c in ${CONFIGS:-c4 c5 c1 c3}; do
  if [ $first = 1 ] && [ -z "$NO_TESTS" ]; then TAG=$T CONFIG=$c GENERAL_PMC=1 bash scripts/gpu_round.sh || exit 2
  else NO_TESTS=1 TAG=$T CONFIG=$c GENERAL_PMC=1 bash scripts/gpu_round.sh || exit 3; fi
  first=0
done
if [ -n "$DECODE" ]; then
  timeout -k 10 400 python scripts/bench_decode.py --device-snapshots 8 > $O/bench_decode_$T.json 2> $O/bench_decode_$T.err || exit 4
fi
echo "final ok"
