#!/bin/bash
# Round 5, session av (final build): bench with the staged-path warmup, every
# GPU test, smoke, the headline's rocprof, the driver's short invocation and a
# 2-rank rehearsal of the multi-GPU path on the one GPU.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05av bench tests smoke profhead || exit $?
OUT=gpurun_out/r05av
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_short.log 2>&1 || exit $?
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 --dist-backend gloo --no-cpu-baseline \
    > $OUT/bench_dist2_gloo.log 2>&1 || exit $?
echo done
