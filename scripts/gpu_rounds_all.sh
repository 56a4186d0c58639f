#!/bin/bash
# Per-config round records (bench with CPU baseline, kernel stats, PMC traffic) for the
# secondary configs, plus the C4 CPU baseline on a 10M-key sample.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-r2}
for c in ${CONFIGS-c5 c3 c1}; do
  NO_TESTS=1 TAG=$T CONFIG=$c bash scripts/gpu_round.sh > $O/round_$c.log 2>&1 || { echo "round $c failed"; tail -20 $O/round_$c.log; exit 1; }
  echo "== $c"; tail -3 $O/round_$c.log
done
if [ -z "$NO_CPU10M" ]; then
  timeout -k 10 600 python bench.py --config c4 --steps 1 --warmup 0 --cpu-universe 10000000 \
    > $O/bench_c4_cpu10m_$T.json 2> $O/bench_c4_cpu10m_$T.err || { echo "cpu10m failed"; tail -20 $O/bench_c4_cpu10m_$T.err; exit 2; }
  python scripts/summ.py $O/bench_c4_cpu10m_$T.json
fi
