#!/bin/bash
# Round 4, session q: host enqueue time of the split per-step PPO rollout.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 --host 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records|value" | sed "s|^|$tag |" || exit 1
}
run "split MT1  " MADRONA_BB_POLICY_MT=1
run "nosplit MT4" MADRONA_BB_PPO_SPLIT_MIN_WORLDS=0
