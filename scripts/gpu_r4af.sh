#!/bin/bash
# Host clock of the over-capacity planning and the chip-wide batches' sort widths (CDB_HOT_PROF).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
for c in c5 c3; do
CDB_HOT_PROF=1 timeout -k 10 300 python bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-general > $O/r4af_$c.json 2> $O/r4af_$c.err || exit 3
grep "over_capacity\|chip_wide" $O/r4af_$c.err | tail -8
done
