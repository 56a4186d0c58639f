#!/bin/bash
# Round 4: decode bench with the dd_launch host clock.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python scripts/bench_decode.py --reps 2 ${ARGS} > $O/bench_decode_r4j.json 2> $O/bench_decode_r4j.err || { tail -5 $O/bench_decode_r4j.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench_decode_r4j.json')); print(d['gpu_call_ms'], d['device_resident']['decode_to_hbm_ms'], d['device_resident']['phases'])"
echo "r4j ok"
