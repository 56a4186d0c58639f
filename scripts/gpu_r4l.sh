#!/bin/bash
# Round 4: records rows as 16-B pieces -- tests, bench both layouts, TA/TD/TCP counters.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_records_gpu.py tests/test_golden.py tests/test_runs_oracle_gpu.py tests/test_sorted_runs_gpu.py tests/test_gpu_parity.py tests/test_configs_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_r4l.log 2>&1
rc=$?; tail -2 $O/pytest_r4l.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc"; exit 1; }
for lay in records columns; do
  timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-general --layout $lay > $O/l_$lay.json 2> $O/l_$lay.err || { echo "bench $lay failed"; tail -5 $O/l_$lay.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['phases_ms'].items()})" $O/l_$lay.json "$lay"
done
i=0
for p in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $p --kernel-include-regex "bucket_wave_runs" --output-format csv -d $O/pmc_r4l/pass$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-general --layout records > $O/pmc_r4l_pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pmc_r4l_pass$i.log; exit 3; }
done
python3 scripts/pmc_sum.py $O/pmc_r4l | tee $O/pmc_r4l_summary.txt | head -24
echo "r4l ok"
