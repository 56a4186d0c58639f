#!/bin/bash
# Records for the new chip-wide path: C3 and C5 bench lines, kernel stats and FETCH/WRITE PMC traffic;
# the C4 general-path (hash-random input) traffic refreshed.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_decode_device_gpu.py tests/test_decode_merge_full_gpu.py tests/test_runs_oracle_gpu.py -k "not full_c4" > $O/pytest_r4ah.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4ah.log; exit 1; }
tail -1 $O/pytest_r4ah.log
for c in c3 c5; do
  NO_TESTS=1 TAG=r4ah CONFIG=$c bash scripts/gpu_round.sh > $O/round_${c}_r4ah.log 2>&1 || { echo "round $c failed"; tail -5 $O/round_${c}_r4ah.log; exit 1; }
  tail -1 $O/round_${c}_r4ah.log
done
KRE="merge_begin_marker|merge_end_marker|pipe_|iota|set_dir|stamp_pos|part_|bucket_|compact|scan_|stats_reduce|gc_lastbad|hot_|sorted_|seg_|run_|mat_|radix_hist|radix_scatter"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 250 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv -d $O/pmcg_c4_r4ah_$c -o run -- python bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --input-order hash-random --no-decode-leg > $O/pmcg_c4_r4ah_$c.log 2>&1 || { echo "pmc general $c failed"; exit 6; }
done
python3 scripts/pmc_traffic.py $O/pmcg_c4_r4ah_FETCH_SIZE $O/pmcg_c4_r4ah_WRITE_SIZE $O/pmc_traffic_c4_general_r4ah.json || exit 7
timeout -k 10 300 python scripts/bench_decode.py > $O/bench_decode_r4ah.json 2> $O/bench_decode_r4ah.err || { echo "decode bench failed"; exit 8; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_decode_r4ah.json')); print('decode', d['device_resident']['decode_to_hbm_ms'], d['device_resident']['phases'].get('order_sort_ms'))"
echo "r4ah ok"
