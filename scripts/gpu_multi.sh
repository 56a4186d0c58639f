#!/bin/bash
# The multi-GPU path on one GPU: bench.py under torchrun at N=1 (RCCL process group, the
# dist step with its world-size-1 shortcut) next to the direct N=1 line.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${TAG:-m}
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --force-dist --no-cpu-baseline \
  > $O/bench_dist1_$T.json 2> $O/bench_dist1_$T.err || { echo "dist bench failed"; tail -20 $O/bench_dist1_$T.err; exit 1; }
python scripts/summ.py $O/bench_dist1_$T.json
