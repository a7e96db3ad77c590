#!/bin/bash
# Round 4, session p: kernel trace of the split per-step PPO rollout (policy
# halves at MT 1) -- do the halves' kernels overlap?
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/p
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MADRONA_BB_POLICY_MT=1
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/split_mt1 -o run --output-format csv \
    -- python3 $R/tools/ppo_time.py --worlds 65536 --rollouts 2 > $OUT/split_mt1.log 2>&1 || exit 1
export MADRONA_BB_POLICY_MT=4 MADRONA_BB_PPO_SPLIT_MIN_WORLDS=0
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/nosplit -o run --output-format csv \
    -- python3 $R/tools/ppo_time.py --worlds 65536 --rollouts 2 > $OUT/nosplit.log 2>&1 || exit 1
find $OUT -name "*.csv" | head
