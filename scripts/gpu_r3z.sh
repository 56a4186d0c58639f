#!/bin/bash
# Round 3 experiment: the wide tier after the wave tier on the merge stream (grid sweep) vs beside it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in 0 256 1024 4096; do
CDB_EXP_WIDE_SERIAL=$g timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_c4_r3z_$g.json 2> gpurun_out/bench_c4_r3z_$g.err || { echo "bench $g failed"; tail -5 gpurun_out/bench_c4_r3z_$g.err; exit 2; }
python3 -c "import json;a=json.load(open('gpurun_out/bench_c4_r3z_$g.json'));print('c4 serial-grid $g', round(a['ms_per_step'],3), a['phases_ms'])"
done
