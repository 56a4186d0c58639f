#!/bin/bash
# PMC passes over bench.py (one counter group per rocprofv3 run; counters never combined
# with runtime/sys tracing). Usage: scripts/pmc_profile.sh <outdir> <bench args...>
set -o pipefail
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
PASSES=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-include-regex "${KREGEX:-bucket|part_|compact}" \
    --output-format csv -d "$OUT/pass$i" -o run -- python bench.py --no-cpu-baseline "$@" \
    > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "pmc ok"
