#!/bin/bash
# Round 4: the split PPO's next-value pass per part on the part's stream (before
# the join) instead of one pass over every world after it; parity + timing.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/fp
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/fp/pytest.log 2>&1
rc=$?; echo "tests: $(tail -n 1 gpurun_out/fp/pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/fp/pytest.log; exit $rc; }
for i in 1 2 3; do
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | grep -E "all records" || exit 1
done
