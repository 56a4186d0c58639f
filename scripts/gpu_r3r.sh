#!/bin/bash
# Round 3: C1 bench line (with its CPU leg) and the smoke entry point.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 3 > gpurun_out/bench_c1_r3r.json 2> gpurun_out/bench_c1_r3r.err || { echo "bench c1 failed"; tail -20 gpurun_out/bench_c1_r3r.err; exit 1; }
python3 -c "import json;a=json.load(open('gpurun_out/bench_c1_r3r.json'));print('c1', round(a['ms_per_step'],3), a['roofline']['frac'], a['cpu_baseline']['value'])"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3r.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r3r.log; exit 2; }
tail -3 gpurun_out/smoke_r3r.log
