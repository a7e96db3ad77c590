#!/bin/bash
# Round 4: the split PPO rollout issued on a torch side stream (parity), with
# the rest of the rollout tests.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/ss
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/ss/pytest.log 2>&1
rc=$?; tail -n 22 gpurun_out/ss/pytest.log; exit $rc
