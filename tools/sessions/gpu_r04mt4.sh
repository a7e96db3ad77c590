#!/bin/bash
# Round 4: pol_select draws one threefry pair per bucket pair (3 calls per row
# instead of 6): every policy test, the rollout tests, MT4 timing.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/mt4
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py \
    tests/test_policy_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mt4/pytest.log 2>&1
rc=$?; echo "policy tests: $(tail -n 1 gpurun_out/mt4/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|MT4 |" || exit 1
done
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | grep -E "all records" || exit 1
