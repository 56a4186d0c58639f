#!/bin/bash
# Diagnostics of the sorted-run wave kernel: per-kernel times (load-only variant and full, wide
# kernel serialised), SQ counter passes, then a PC-sampling attempt.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
export CDB_WIDE_SERIAL=1
for v in stop0 full; do
  if [ $v = full ]; then unset CDB_LIB; else export CDB_LIB=variants/libcdb_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/diag_$v -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/diag_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  python3 scripts/kstats.py "$(find $O/diag_$v -name "*kernel_stats.csv" | sort | tail -1)" 12 || true
done
unset CDB_LIB
i=0
for p in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $p --kernel-include-regex "bucket_wave_runs|bucket_wide_runs" --output-format csv -d $O/diag_sq/pass$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/diag_sq_pass$i.log 2>&1 || { echo "sq pass $i failed"; exit 2; }
done
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-include-regex "bucket_wave_runs" --output-format csv -d $O/diag_pcs -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/diag_pcs.log 2>&1 || { echo "pc sampling failed"; tail -5 $O/diag_pcs.log; exit 3; }
echo "diag ok"
