#!/bin/bash
# Step timelines (rocprofv3 kernel trace of the last timed merge) of one config under env variants:
# for each "NAME=ENV" in VARIANTS, gpurun_out/timeline_<TAG>_<NAME>.txt.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
T=${TAG:-tl}
C=${CONFIG:-c4}
mkdir -p $O
for v in $VARIANTS; do
  name=${v%%=*}
  envs=${v#*=}
  envs=${envs//,/ }
  (for e in $envs; do export "$e"; done
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${T}_$name -o run -- python bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-general --no-decode-leg > $O/prof_${T}_$name.log 2>&1) || { echo "prof $name failed"; exit 3; }
  python3 scripts/timeline.py $O/prof_${T}_$name --last 1 > $O/timeline_${T}_$name.txt || exit 4
  echo "== $name"; grep -E "pipe|wide|run_|units" $O/timeline_${T}_$name.txt | cut -c1-110
done
