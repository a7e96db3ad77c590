#!/bin/bash
# Round 4: 32-row bucket noise deduplication (two threefry calls per lane):
# policy tests with k_policy<2> forced, the rollout tests (split halves run
# k_policy<2>), and the PPO timing at 65 536 worlds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/mt2
export PYTHONUNBUFFERED=1
MADRONA_BB_POLICY_MT=2 timeout -k 10 600 python3 -u -m pytest tests/test_policy.py tests/test_policy_golden.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/mt2/pytest_forced.log 2>&1
rc=$?; echo "forced MT2: $(tail -n 1 gpurun_out/mt2/pytest_forced.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/mt2/pytest.log 2>&1
rc=$?; echo "default: $(tail -n 1 gpurun_out/mt2/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | grep -E "all records|value" || exit 1
done
MADRONA_BB_POLICY_MT=2 timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|MT2 |" || exit 1
