#!/bin/bash
# Round 5, session k: k_rollout_ppo with 1- and 2-wave workgroups on small
# grids (one workgroup per CU) against the default paths there (8 192 / 16 384:
# k_rollout_policy; 24 576: the two-stream split).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05k
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_ppo_step.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for W in 8192 16384 24576; do for v in default loop; do
    if [ $v = loop ]; then E="MADRONA_BB_PPO_STEP_FUSED_MIN_WORLDS=1 MADRONA_BB_PPO_FUSED_MAX_WORLDS=0"; else E=""; fi
    env $E timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records.*per_step=0" | sed "s|^|$v $W |" >> $OUT/small_ab.txt || exit 1
done; done; done
echo done
