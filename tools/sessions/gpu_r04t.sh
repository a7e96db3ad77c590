#!/bin/bash
# Round 4, session t: which buffer records cost what in the split per-step PPO
# rollout (65 536 worlds), split on and off.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | sed "s|^|split   |" || exit 1
MADRONA_BB_PPO_SPLIT_MIN_WORLDS=0 timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | sed "s|^|nosplit |" || exit 1
