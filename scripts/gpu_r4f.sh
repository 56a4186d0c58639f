#!/bin/bash
# Round 4: the sharded tests (records inputs, the C program's two-slot context), then an A/B of the
# wave kernel's LDS staging (input records through LDS-DMA, output rows through LDS) on the C4 shard,
# then the rest of the round's GPU tests.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_shard_gpu.py tests/test_abi_c.py -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4f_shard.log 2>&1
rc=$?; tail -5 $O/pytest_r4f_shard.log
[ $rc -le 1 ] || { echo "shard pytest ended with $rc"; exit 1; }
for v in base noout noin none; do
  lib=$PWD/variants/lib_$v.so; [ $v = base ] && lib=$PWD/constdb_amd/libcdbmerge.so
  for lay in records columns; do
    CDB_LIB=$lib timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-general --layout $lay > $O/ab_${v}_$lay.json 2> $O/ab_${v}_$lay.err || { echo "bench $v $lay failed"; tail -5 $O/ab_${v}_$lay.err; exit 2; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()})" $O/ab_${v}_$lay.json "$v $lay"
  done
done
timeout -k 10 800 python -u -m pytest tests/test_encode_device_gpu.py tests/test_decode_device_gpu.py tests/test_records_gpu.py tests/test_golden.py tests/test_runs_oracle_gpu.py tests/test_dist_gpu.py tests/test_sorted_runs_gpu.py -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4f.log 2>&1
rc=$?; tail -8 $O/pytest_r4f.log
[ $rc -le 1 ] || { echo "pytest ended with $rc"; exit 3; }
timeout -k 10 300 python scripts/bench_encode.py > $O/bench_encode_r4.json 2> $O/bench_encode_r4.err || { tail -5 $O/bench_encode_r4.err; exit 4; }
timeout -k 10 400 python scripts/bench_decode.py --reps 2 > $O/bench_decode_r4.json 2> $O/bench_decode_r4.err || { tail -5 $O/bench_decode_r4.err; exit 5; }
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_dec_r4 -o run -- python scripts/bench_decode.py --reps 1 > $O/prof_dec_r4.log 2>&1 || { echo "decode prof failed"; exit 6; }
echo "r4f main ok"
for v in 0 1 2 3; do
  for lay in columns records; do
    CDB_LIB=$PWD/variants/libcdb_stop$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-general --layout $lay > $O/phase_${lay}_$v.json 2> $O/phase_${lay}_$v.err || { echo "phase variant $v failed"; tail -5 $O/phase_${lay}_$v.err; exit 7; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('stop', sys.argv[2], {k: round(x,2) for k,x in d['phases_ms'].items()})" $O/phase_${lay}_$v.json "$v $lay"
  done
done
echo "r4f phases ok"
