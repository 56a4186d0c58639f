# Plan sweep: bench (small and full) for several final-level fan-outs.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_${TAG}.log 2>&1 || exit 1
for d in ${DLASTS:-32 64 128 256}; do
  CDB_PLAN_DLAST=$d timeout -k 10 300 python bench.py --universe-per-gpu 4000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tune_${TAG}_small_$d.json 2> gpurun_out/tune_${TAG}_small_$d.err || exit 2
  CDB_PLAN_DLAST=$d timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tune_${TAG}_full_$d.json 2> gpurun_out/tune_${TAG}_full_$d.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python bench.py --universe-per-gpu 4000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || exit 4
echo done
