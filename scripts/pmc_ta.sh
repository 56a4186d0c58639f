#!/bin/bash
# Vector-memory pipeline counters (TA/TD/TCP) of the bucket kernel: is it address-bound?
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-ta}
O=gpurun_out
timeout -s KILL 60 rocprofv3 -L > $O/counters_avail.txt 2>&1 || echo "list failed"
i=0
for p in ${PASSES:-"TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "${KREGEX:-bucket_wave|part_scatter|compact}" --output-format csv -d $O/pmc_${T}/pass$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $O/pmc_${T}_pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pmc_${T}_pass$i.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
agg = collections.defaultdict(dict)
for f in sorted(glob.glob('$O/pmc_${T}/pass*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:60]
        agg[(k, r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
for (k, d), c in sorted(agg.items(), key=lambda x: int(x[0][1])):
    print(k, d, {n: f"{v:.4g}" for n, v in c.items()})
PY
echo "ta ok"
