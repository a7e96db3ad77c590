#!/bin/bash
# Round 5, session l: bucket pass rounds bounded by their largest bucket
# (bfull: every round over 8 logits) -- policy / PPO tests, A/B at 8 192 /
# 16 384 (k_rollout_policy), 65 536 (k_rollout_ppo), k_policy at 65 536 rows.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05l
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_ppo_step.py tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py \
    tests/test_policy_golden.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for W in 8192 16384 65536; do for v in prod bfull; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records.*per_step=0" | sed "s|^|$v $W |" >> $OUT/bucket_ab.txt || exit 1
done; done; done
for v in prod bfull; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids \
        | sed "s|^|$v |" >> $OUT/bucket_policy_ab.txt || exit 1
done
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192.txt 2>&1 || exit $?
echo done
