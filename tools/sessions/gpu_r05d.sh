#!/bin/bash
# Round 5, session d: (1) parity of the fused PPO step (sc1 record stores) and
# of the fused 8 192-world rollout with the rows handed over in two halves
# (both lanes of a world emit the trainee's row; layer 1 starts on the first
# half); (2) the 8 192-world per-step trace and PPO timing; (3) start skew of
# half the waves in the fused PPO step at 65 536 worlds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05d
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_ppo_step.py tests/test_policy_rollout.py tests/test_policy_golden.py \
    -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 16384 > $OUT/ppo_trace_W16384.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_time.py --worlds 8192 --rollouts 6 > $OUT/ppo_time_W8192.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/ppo_step_trace.py --worlds 65536 --no-ablate --skews 0,2,4,6,8,12 > $OUT/pps_skew_W65536.log 2>&1 || exit $?
echo done
