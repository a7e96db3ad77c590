#!/bin/bash
# Round 5, session f: the fused 8 192-world PPO rollout with one policy wave per M-tile (no
# cross-wave exchanges in the network), the fused step with a joint 2-tile tail --
# kernel and of the PPO paths, then the 8 192-world PPO trace / timing and the
# fused PPO step's phase trace at 65 536 worlds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05f
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_policy.py tests/test_policy_golden.py tests/test_policy_wg.py \
    tests/test_policy_rollout.py tests/test_ppo_step.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_time.py --worlds 8192 --rollouts 6 > $OUT/ppo_time_W8192.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 16384 > $OUT/ppo_trace_W16384.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_time.py --worlds 16384 --rollouts 6 > $OUT/ppo_time_W16384.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 > $OUT/ppo_time_W65536.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/ppo_step_trace.py --worlds 65536 > $OUT/pps_trace_W65536.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/policy_time.py --worlds 65536 > $OUT/policy_time_W65536.log 2>&1 || exit $?
echo done
