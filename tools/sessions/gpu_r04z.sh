#!/bin/bash
# Round 4, session z: (1) policy parity after the 16-row bucket noise
# deduplication (one threefry call per lane); (2) the split PPO's policy kernel
# per part: k_policy<1> (product) vs k_policy_wg (weights in LDS) vs k_policy<2>.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/z
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py \
    tests/test_policy_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
MADRONA_BB_PPO_SPLIT_MT=0 MADRONA_BB_POLICY_WG=1 timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_wg.log 2>&1
rc=$?; tail -n 1 $OUT/pytest_wg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|MT4 |" || exit 1
MADRONA_BB_POLICY_MT=1 timeout -k 10 120 python3 tools/policy_time.py --worlds 32768 2>&1 | grep -v amdgpu.ids | sed "s|^|MT1 |" || exit 1
for i in 1 2; do
for v in "mt1 MADRONA_BB_PPO_SPLIT_MT=1" "wg MADRONA_BB_PPO_SPLIT_MT=0 MADRONA_BB_POLICY_WG=1" "mt2 MADRONA_BB_PPO_SPLIT_MT=2"; do
    set -- $v; tag=$1; shift
    env "$@" timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records|value" | sed "s|^|$tag |" || exit 1
done
done
