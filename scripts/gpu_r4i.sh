#!/bin/bash
# Round 4: direct (page-locked) upload A/B for the decode into HBM; the other configs' bench lines.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_device_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4i.log 2>&1
rc=$?; tail -2 $O/pytest_r4i.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc"; exit 1; }
CDB_H2D_STAGED=1 timeout -k 10 300 python -u -m pytest tests/test_decode_device_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4i_reg.log 2>&1
rc=$?; tail -2 $O/pytest_r4i_reg.log
[ $rc -eq 0 ] || { echo "pytest (register) ended with $rc"; exit 1; }
for v in ring reg; do
  E=""; [ $v = ring ] && E="CDB_H2D_STAGED=1"
  env $E timeout -k 10 400 python scripts/bench_decode.py --reps 3 > $O/bench_decode_r4i_$v.json 2> $O/bench_decode_r4i_$v.err || { tail -5 $O/bench_decode_r4i_$v.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['gpu_call_ms'], d['device_resident']['decode_to_hbm_ms'], d['device_resident']['phases'])" $O/bench_decode_r4i_$v.json $v
done
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_dec_r4i -o run -- python scripts/bench_decode.py --reps 1 > $O/prof_dec_r4i.log 2>&1 || { echo "decode prof failed"; exit 4; }
for c in ; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > $O/bench_r4i_$c.json 2> $O/bench_r4i_$c.err || { echo "bench $c failed"; tail -5 $O/bench_r4i_$c.err; exit 5; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()})" $O/bench_r4i_$c.json $c
done
echo "r4i ok"
