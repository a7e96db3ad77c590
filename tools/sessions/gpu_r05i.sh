#!/bin/bash
# Round 5, session i: k_step_ppo without the other agent's sim rows before the
# last step, the trainee's row split over both lanes: parity tests, A/B against
# the first version (ppsold: every non-trainee row stored, both rows emitted)
# and the unsplit emission (ppsnosplit), phase trace + attribution.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05i
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_ppo_step.py tests/test_policy_rollout.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for W in 65536 32768; do for v in prod ppsold ppsnosplit; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "per_step=0" | sed "s|^|$v $W |" >> $OUT/pps_ab.txt || exit 1
done; done; done
timeout -k 10 400 python3 tools/ppo_step_trace.py --worlds 65536 > $OUT/pps_trace_W65536.txt 2>&1 || exit $?
echo done
