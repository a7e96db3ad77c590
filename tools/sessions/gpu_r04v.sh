#!/bin/bash
# Round 4, session v: split PPO with the halves re-aligned every step (event
# per step) vs every 4 / 8 steps vs only at the start; parity first.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/v
mkdir -p $OUT
export PYTHONUNBUFFERED=1
MADRONA_BB_PPO_SPLIT_SYNC=0 timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for s in 1 0 4 8; do
    MADRONA_BB_PPO_SPLIT_SYNC=$s timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records|value" | sed "s|^|sync=$s |" || exit 1
done
done
