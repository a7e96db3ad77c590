#!/bin/bash
# Round 4, session x: fused PPO rollout vs the split per-step loop at 8 192 and
# 16 384 worlds (where the fused kernel is the default).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
for i in 1 2; do
for W in 8192 16384 24576; do
    timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records" | sed "s|^|W=$W default |" || exit 1
    MADRONA_BB_PPO_SPLIT_MIN_WORLDS=1 timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records" | sed "s|^|W=$W split |" || exit 1
done
done
