set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_${TAG:-r1d}.log 2>&1 && \
timeout -k 10 300 python bench.py --universe-per-gpu 4000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small_${TAG:-r1d}.json 2> gpurun_out/bench_small_${TAG:-r1d}.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-r1d} -o run -- python bench.py --universe-per-gpu 4000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG:-r1d}.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_full_${TAG:-r1d}.json 2> gpurun_out/bench_full_${TAG:-r1d}.err
echo EXIT $?
