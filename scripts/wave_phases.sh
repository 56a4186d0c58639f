#!/bin/bash
# Times the wave kernel stopped after each phase (variants/libcdb_stopN.so, built on the CPU
# side by constdb_amd/build.py with -DCDB_WAVE_STOP=N): bucket-phase ms per variant and input order.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
for io in ${ORDERS:-sorted hash-random}; do
for v in 0 1 2 3 full; do
  if [ $v = full ]; then L=""; else L="CDB_LIB=variants/libcdb_stop$v.so"; fi
  env $L timeout -k 10 300 python bench.py --input-order $io --steps 3 --warmup 1 --no-cpu-baseline > $O/phase_${io}_$v.json 2> $O/phase_${io}_$v.err || { echo "variant $v failed"; tail -5 $O/phase_${io}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/phase_${io}_$v.json'));print('$io','$v',{k:round(x,2) for k,x in d['phases_ms'].items()})"
done
done
