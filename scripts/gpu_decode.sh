#!/bin/bash
# The device entry index: the decoder tests, then the decode benches (8 x 250 MB and the C4 shard's
# 8 x 2 GB leg) and the walk kernels' times. (Round 6 ran it with CDB_IDX_WALK = flat / lane / wave,
# the lane walks since removed: DESIGN.md §8.)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
T=${TAG:-lw}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_decode_device_gpu.py tests/test_decode_window_gpu.py tests/test_decode_merge_full_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_$T.log; exit 1; }
tail -2 $O/pytest_$T.log
fi
for v in ${WALKS:-wave}; do
  timeout -k 10 300 python scripts/bench_decode.py --reps 3 > $O/dec_${T}_$v.json 2> $O/dec_${T}_$v.err || { echo "bench_decode $v failed"; tail -5 $O/dec_${T}_$v.err; exit 2; }
  echo "$v 8x250MB: $(tail -c 600 $O/dec_${T}_$v.json)"
done
for v in ${LEG_WALKS:-wave}; do
  timeout -k 10 400 python scripts/decode_leg.py --reps 2 > $O/leg_${T}_$v.json 2> $O/leg_${T}_$v.err || { echo "decode_leg $v failed"; tail -5 $O/leg_${T}_$v.err; exit 3; }
  echo "$v C4 leg: $(python3 -c "import json; print([round(json.loads(l)['decode_ms'],1) for l in open('$O/leg_${T}_$v.json') if l.strip()])" 2>/dev/null || tail -c 300 $O/leg_${T}_$v.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dec_$T -o run -- python scripts/bench_decode.py --reps 1 > $O/prof_dec_$T.log 2>&1 || { echo "prof failed"; exit 4; }
grep -h "idx_" $O/prof_dec_$T/*/run_kernel_stats.csv $O/prof_dec_$T/run_kernel_stats.csv 2>/dev/null | cut -c1-200
echo "decode ok"
