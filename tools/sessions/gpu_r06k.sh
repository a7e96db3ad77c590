#!/bin/bash
# Round 6, session k: k_rollout_ppo with the worlds resident across the K
# steps (k_rollout_ppo_res; 696 B/lane of scratch) -- PPO parity tests, then
# the rollout time against the reloading kernel (r6_ppo_nores).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06k
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ppo_step.py \
    tests/test_policy_rollout.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in r6_ppo_nores product; do
    if [ $v = product ]; then L=""; else L=$R/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    for W in 32768 65536 131072; do
        MADRONA_BB_LIB=$L timeout -k 10 200 python3 -u tools/ppo_time.py --worlds $W --rollouts 6 2>&1 \
            | grep -v amdgpu.ids | grep "all records" | sed "s|^|$v W=$W |" >> $OUT/ppo.txt || exit 1
    done
done
done
cat $OUT/ppo.txt
