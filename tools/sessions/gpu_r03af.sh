#!/bin/bash
# kernel-trace stats of the fused PPO rollout at 8192 (kernel duration vs the event timing)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03af; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/bench.py --worlds 8192 --rollout 32 --policy --steps 512 --warmup 0 --no-cpu-baseline --no-e2e --no-configs > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 2; }
grep -h policy_rollout $O/bench.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('events us/step %.3f' % d['policy_rollout']['us_per_step'])"
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; head -5 $O/kernel_stats.csv
