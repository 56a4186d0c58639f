#!/bin/bash
# (round-2 recipe behind DESIGN.md 4a'; CDB_WIDE_SERIAL, which serialised the wide tier, was removed in round 3)
# Instruction counts of the sorted-run wave kernel stopped after each phase (variants/libcdb_stopN.so).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
export CDB_WIDE_SERIAL=1
for v in 0 1 2 3 full; do
  if [ $v = full ]; then unset CDB_LIB; else export CDB_LIB=variants/libcdb_stop$v.so; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --kernel-include-regex "bucket_wave_runs" --output-format csv -d $O/pinst_$v -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pinst_$v.log 2>&1 || { echo "pass $v failed"; exit 1; }
done
echo "phase insts ok"
