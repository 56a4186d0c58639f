#!/bin/bash
# Round 4: wide-tier scheduling experiment on the C4 step (and C5).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
for cfg in c4 c5; do
for v in "0 256" "1 1024" "1 4096" "2 1024" "2 4096"; do
  set -- $v
  CDB_WIDE_MODE=$1 CDB_WIDE_GRID=$2 timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-general --no-decode-leg > $O/u_${cfg}_$1_$2.json 2> $O/u_${cfg}_$1_$2.err || { echo "bench $v failed"; tail -5 $O/u_${cfg}_$1_$2.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()})" $O/u_${cfg}_$1_$2.json "$cfg mode $1 grid $2"
done
done
echo "r4u ok"
