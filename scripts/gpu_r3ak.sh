#!/bin/bash
# Round 3: hot_tag wave-level bucket lookup (tag16), radix tile size (rounds of 256 pairs per tile: 16 / 32 / 64) on C5 and C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in tag16 r64 r32 r16; do
cp constdb_amd/libcdbmerge_$v.so constdb_amd/libcdbmerge.so
for c in c5 c3; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-general > gpurun_out/bench_${c}_${v}_r3ak.json 2> gpurun_out/bench_${c}_${v}_r3ak.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_${c}_${v}_r3ak.err; exit 3; }
python -c "import json,sys; d=json.load(open('gpurun_out/bench_${c}_${v}_r3ak.json')); print('$v $c', d['ms_per_step'], d['phases_ms'])"
done
done
echo ok
