#!/bin/bash
# SQ / TA counters of the wave and wide kernels for one bench layout (BENCH_ARGS), one pass per run.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-r4d}
O=gpurun_out
i=0
for p in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $p --kernel-include-regex "${KREGEX:-bucket_w}" --output-format csv -d $O/pmc_${T}/pass$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-general ${BENCH_ARGS} > $O/pmc_${T}_pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pmc_${T}_pass$i.log; exit 1; }
done
python3 scripts/pmc_sum.py $O/pmc_${T} | tee $O/pmc_${T}_summary.txt
