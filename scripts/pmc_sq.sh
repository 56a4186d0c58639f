#!/bin/bash
# SQ counter passes on the bucket kernels (one rocprofv3 run per pass).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${TAG:-sq}
O=gpurun_out
i=0
for p in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $p --kernel-include-regex "${KREGEX:-bucket_wave|part_scatter}" --output-format csv -d $O/pmc_${T}/pass$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $O/pmc_${T}_pass$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "sq ok"
