#!/bin/bash
# Round 4, session w: split PPO into 2 / 3 / 4 world parts on as many streams
# (start-only alignment); parity at each part count first.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/w
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for P in 2 3 4; do
MADRONA_BB_PPO_SPLIT_PARTS=$P timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_P$P.log 2>&1
rc=$?; echo "P=$P $(tail -n 1 $OUT/pytest_P$P.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
for P in 2 3 4; do
    MADRONA_BB_PPO_SPLIT_PARTS=$P timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records|value" | sed "s|^|P=$P |" || exit 1
done
done
for W in 32768 131072; do
for P in 2 4; do
    MADRONA_BB_PPO_SPLIT_PARTS=$P timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 3 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records" | sed "s|^|W=$W P=$P |" || exit 1
done
done
