#!/bin/bash
# Round 5, session af: the fused PPO rollout's policy-wave count by grid
# (4 at <= one workgroup per CU) -- policy rollout tests, timings, trace.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05af
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_policy_rollout.py tests/test_ppo_step.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for W in 8192 16384 4096 12288; do
    timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 6 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records.*per_step=0" | sed "s|^|$W |" >> $OUT/ppo_time.txt || exit 1
done
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192.txt 2>&1 || exit $?
echo done
