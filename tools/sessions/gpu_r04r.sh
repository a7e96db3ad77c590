#!/bin/bash
# Round 4, session r: split per-step PPO (halves on two streams, policy halves
# at k_policy<1>) vs one stream, 32 768 ... 262 144 worlds; parity first.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/r
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag worlds env...
    local tag=$1 w=$2; shift 2
    env "$@" timeout -k 10 300 python3 tools/ppo_time.py --worlds $w --rollouts 3 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records|value" | sed "s|^|$tag W=$w |" || exit 1
}
for w in 65536 32768 131072 262144; do
run "split  " $w MADRONA_BB_PPO_SPLIT_MIN_WORLDS=1
run "nosplit" $w MADRONA_BB_PPO_SPLIT_MIN_WORLDS=0
done
