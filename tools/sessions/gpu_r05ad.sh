#!/bin/bash
# Round 5, session ad: the 8 192-world fused PPO rollout with 4 policy waves
# (two per M-tile, one output half each; pw4) against 2, now that the bucket
# pass is branch-free; traces of both.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05ad
mkdir -p $OUT
export PYTHONUNBUFFERED=1
V=madrona_basketball_amd/_variants/pw4/libmadrona_basketball_amd.so
MADRONA_BB_LIB=$V timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_policy_rollout.py > $OUT/pytest_pw4.log 2>&1
rc=$?; tail -n 2 $OUT/pytest_pw4.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in prod pw4; do
    if [ $v = prod ]; then lib=""; else lib=$V; fi
    for W in 8192 16384; do
        MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 6 2>&1 | grep -v amdgpu.ids \
            | grep -E "all records.*per_step=0" | sed "s|^|$v $W |" >> $OUT/pw_ab.txt || exit 1
    done
done; done
MADRONA_BB_LIB=$V timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192_pw4.txt 2>&1 || exit $?
echo done
