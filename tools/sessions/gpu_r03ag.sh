#!/bin/bash
# per-launch fixed cost of the fused PPO rollout: events per launch at K = 8, 16, 32, 64
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03ag; mkdir -p $O
cd $ROOT
for K in 8 16 32 64 128; do
  timeout -k 10 120 python bench.py --worlds 8192 --rollout $K --policy --steps 1024 --warmup 0 --no-cpu-baseline --no-e2e --no-configs > $O/b_K$K.log 2>&1 || exit 2
  grep -h policy_rollout $O/b_K$K.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); p=d['policy_rollout']; print('K=$K rollout us %.1f us/step %.3f' % (p['rollout_avg_us'], p['us_per_step']))"
done
