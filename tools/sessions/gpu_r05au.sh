#!/bin/bash
# Round 5, session au: the driver's bench invocations on the final build --
# N = 1 with the driver's short arguments, and a 2-rank rehearsal of the
# multi-GPU path on the one GPU (gloo; correctness of the barrier /
# max-over-ranks / per-rank loop-kernel path, not a scaling point).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05au
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_short.log 2>&1 || exit $?
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 --dist-backend gloo --no-cpu-baseline \
    > $OUT/bench_dist2_gloo.log 2>&1 || exit $?
echo done
