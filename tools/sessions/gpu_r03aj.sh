#!/bin/bash
# the multi-rank bench path on one GPU box: 2 ranks sharing the MI355X (gloo control plane), then the RCCL path at world size 1
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03aj; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \
    bench.py --gpus 2 --steps 300 --warmup 30 --no-cpu-baseline --dist-backend gloo > $O/two_ranks.log 2>&1 || { tail -30 $O/two_ranks.log; exit 2; }
grep '^{' $O/two_ranks.log | cut -c1-400
timeout -k 10 200 python bench.py --dist --steps 300 --warmup 30 --no-cpu-baseline --no-configs > $O/rccl_ws1.log 2>&1 || { tail -20 $O/rccl_ws1.log; exit 2; }
grep '^{' $O/rccl_ws1.log | cut -c1-300
