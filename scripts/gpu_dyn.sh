export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; O=gpurun_out
for cfg in "1 0" "8 0" "8 1024" "1 1024" "8 8192"; do
  set -- $cfg
  CDB_PIPE=$1 CDB_WAVE_DYN_LDS=$2 timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_dyn_$1_$2.json 2> $O/bench_dyn_$1_$2.err || { echo fail; tail -3 $O/bench_dyn_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_dyn_$1_$2.json'));print('P=$1 dyn=$2',round(d['ms_per_step'],2),{k:round(x,2) for k,x in d['phases_ms'].items()})"
done
