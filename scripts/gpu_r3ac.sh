#!/bin/bash
# Round 3 experiment: C3 child target with the per-bucket LDS sort (buckets <= 4096 children).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ct in 1536 2048 2560 3072 4096; do
CDB_PLAN_CTARGET=$ct timeout -k 10 200 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_c3_r3ac_$ct.json 2> gpurun_out/bench_c3_r3ac_$ct.err || { echo "bench $ct failed"; tail -5 gpurun_out/bench_c3_r3ac_$ct.err; exit 2; }
python3 -c "import json;a=json.load(open('gpurun_out/bench_c3_r3ac_$ct.json'));print('c3 ctarget $ct', round(a['ms_per_step'],3), a['stats']['mid_buckets'], a['stats'].get('hot_slow_runs'))"
done
