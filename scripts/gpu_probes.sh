#!/bin/bash
# Kernel probes: swap in each probe build of libcdbmerge.so and trace the bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
for v in ${PROBES:-base p1 p2 p3}; do
  cp probes/lib_$v.so constdb_amd/libcdbmerge.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_$v -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/probe_$v.log 2>&1 || { echo "probe $v failed"; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open('$O/probe_$v/run_kernel_stats.csv')):
    if 'bucket' in r['Name'] or 'compact' in r['Name']:
        print(f"$v {r['Name'][:40]:40s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
done
