#!/bin/bash
# Round 4, session h: what each PPO record costs; fused vs per-step at 16 384 / 65 536.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
for W in 65536 16384; do
    echo "W=$W"
    timeout -k 10 300 python3 tools/ppo_time.py --worlds $W 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "W=65536 fused forced"
MADRONA_BB_PPO_FUSED_MAX_WORLDS=1000000 timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 3 2>&1 | grep -v amdgpu.ids | grep "per_step=0" || exit 1
