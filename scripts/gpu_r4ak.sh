#!/bin/bash
# FETCH / WRITE passes of the general (partition) path for C1, C3 and C5 (hash-random input order).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
KRE="merge_begin_marker|merge_end_marker|pipe_|iota|set_dir|stamp_pos|part_|bucket_|compact|scan_|stats_reduce|gc_lastbad|hot_|sorted_|seg_|run_|mat_|radix_hist|radix_scatter"
for C in c1 c3 c5; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv -d $O/pmcg_${C}_r4ak_$c -o run -- python bench.py --config $C --steps 1 --warmup 0 --no-cpu-baseline --input-order hash-random > $O/pmcg_${C}_r4ak_$c.log 2>&1 || { echo "pmc general $C $c failed"; exit 6; }
  done
  python3 scripts/pmc_traffic.py $O/pmcg_${C}_r4ak_FETCH_SIZE $O/pmcg_${C}_r4ak_WRITE_SIZE $O/pmc_traffic_${C}_general_r4ak.json > $O/pmcg_${C}_r4ak_summary.txt || exit 7
  tail -1 $O/pmcg_${C}_r4ak_summary.txt
done
echo "r4ak ok"
