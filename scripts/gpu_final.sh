#!/bin/bash
# Final round lines: re-collect C1/C3 records (kernel stats, PMC), install every config's PMC
# summary where bench.py reads it, then one bench line per config (with the CPU baseline).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-r2g}
CONFIGS="${RECOLLECT:-c1 c3}" TAG=$T bash scripts/gpu_records.sh || exit 1
for c in ${RECOLLECT:-c1 c3}; do cp $O/pmc_traffic_${c}_$T.json profiles/r02/pmc_traffic_$c.json; done
for c in c4 c1 c3 c5; do
  timeout -k 10 500 python bench.py --config $c --steps 5 --warmup 2 > $O/final_bench_$c.json 2> $O/final_bench_$c.err || { echo "bench $c failed"; tail -5 $O/final_bench_$c.err; exit 2; }
  python3 -c "import json;d=json.load(open('$O/final_bench_$c.json'));print('$c',round(d['ms_per_step'],2),'%.3g'%d['value'],round(d['roofline']['frac'],4),d['roofline'].get('traffic_over_alg'))"
done
