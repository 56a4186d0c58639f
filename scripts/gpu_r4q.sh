#!/bin/bash
# Round 4: the default bench line (c4, with the CPU baseline and the decode leg).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
start=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench_default_r4q.json 2> $O/bench_default_r4q.err || { echo "bench failed"; tail -20 $O/bench_default_r4q.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
python3 -c "import json; d=json.load(open('$O/bench_default_r4q.json')); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_over_alg']); print(json.dumps(d['decode_leg']))"
echo "r4q ok"
