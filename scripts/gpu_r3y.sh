#!/bin/bash
# Round 3 experiment: runs-mode bucket size limit of the chip-wide child path (C5, C3).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 4096 16384 65536 262144 4294967295; do
for c in c5 c3; do
CDB_EXP_RUNS_CHILD_MAX=$m timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_r3y_$m.json 2> gpurun_out/bench_${c}_r3y_$m.err || { echo "bench $c $m failed"; tail -5 gpurun_out/bench_${c}_r3y_$m.err; exit 2; }
python3 -c "import json;a=json.load(open('gpurun_out/bench_${c}_r3y_$m.json'));print('$c $m', round(a['ms_per_step'],3))"
done
done
