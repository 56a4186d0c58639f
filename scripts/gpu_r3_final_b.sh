#!/bin/bash
# Round 3 record, part 2: C5 and C3 rounds (kernel stats, PMC); then each bench line again (with
# its CPU leg) against this code's PMC file, so the line's traffic comes from the same code.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c5 c3; do
NO_TESTS=1 TAG=r3final CONFIG=$c bash scripts/gpu_round.sh > gpurun_out/round_${c}_r3final.log 2>&1 || { echo "round $c failed"; tail -20 gpurun_out/round_${c}_r3final.log; exit 1; }
cp gpurun_out/pmc_traffic_${c}_r3final.json profiles/r03/pmc_traffic_${c}.json
timeout -k 10 500 python bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bench_${c}_r3final2.json 2> gpurun_out/bench_${c}_r3final2.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_${c}_r3final2.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/bench_${c}_r3final2.json')); print('$c', d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_over_alg'], d['stats'])"
done
