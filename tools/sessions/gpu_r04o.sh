#!/bin/bash
# Round 4, session o: split per-step PPO with the policy's halves at MT 1 / 2
# (registers that fit beside a step wave on one SIMD) vs MT 4, split and not.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/o
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records|value" | sed "s|^|$tag |" || exit 1
}
for i in 1 2; do
run "split MT4  " MADRONA_BB_POLICY_MT=4
run "split MT2  " MADRONA_BB_POLICY_MT=2
run "split MT1  " MADRONA_BB_POLICY_MT=1
run "nosplit MT4" MADRONA_BB_PPO_SPLIT_MIN_WORLDS=0
done
