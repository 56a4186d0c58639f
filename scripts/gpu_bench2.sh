#!/bin/bash
# Bench both input orders of one config, then a kernel-trace profile of the sorted one.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-b}
C=${CONFIG:-c4}
for io in sorted hash-random; do
timeout -k 10 400 python bench.py --config $C --input-order $io --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_${C}_${io}_$T.json 2> $O/bench_${C}_${io}_$T.err || { echo "bench $io failed"; tail -20 $O/bench_${C}_${io}_$T.err; exit 2; }
cat $O/bench_${C}_${io}_$T.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${C}_$T -o run -- python bench.py --config $C --input-order sorted --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_${C}_$T.log 2>&1 || { echo "prof failed"; exit 3; }
python3 - <<PY
import csv
for r in csv.DictReader(open('$O/prof_${C}_$T/run_kernel_stats.csv')):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
