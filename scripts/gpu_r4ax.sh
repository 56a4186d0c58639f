#!/bin/bash
# Final C5 line (CPU baseline, general path) on the final code, and the C4 line for reference.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_shard_gpu.py tests/test_decode_merge_full_gpu.py -k "not full_c4" > $O/pytest_r4ax.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r4ax.log; exit 1; }
tail -1 $O/pytest_r4ax.log
timeout -k 10 500 python bench.py --config c5 > $O/bench_c5_r4ax.json 2> $O/bench_c5_r4ax.err || { echo "bench c5 failed"; tail -10 $O/bench_c5_r4ax.err; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_r4ax -o run -- python bench.py --config c5 --no-cpu-baseline --no-general > $O/prof_c5_r4ax.log 2>&1 || { echo "prof failed"; exit 5; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('c5', round(d['ms_per_step'],2), 'ms frac', round(r['frac'],3), 'traffic x', round(r['traffic_over_alg'],2), 'cpu', round(d['cpu_baseline']['value']/1e6,2), 'general', round(d['general_input']['ms_per_step'],2))" $O/bench_c5_r4ax.json
echo "r4ax ok"
