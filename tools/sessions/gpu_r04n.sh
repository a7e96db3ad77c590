#!/bin/bash
# Round 4, session n: two-stream world-half split of the per-step PPO rollout
# (parity + timing, split on / off).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/n
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | grep -E "all records|value" | sed "s|^|split |" || exit 1
MADRONA_BB_PPO_SPLIT_MIN_WORLDS=0 timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | grep -E "all records|value" | sed "s|^|nosplit |" || exit 1
done
