#!/bin/bash
# Round 5, session ag: k_rollout<2> with 4-wave workgroups kept in step
# (MADRONA_BB_ROLLOUT_G=4) vs 1-wave -- rollout tests with G = 4, then the
# K = 32 recorded rollout at 65 536 / 131 072 / 262 144 worlds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05ag
mkdir -p $OUT
export PYTHONUNBUFFERED=1
MADRONA_BB_ROLLOUT_G=4 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_rollout.py > $OUT/pytest_g4.log 2>&1
rc=$?; tail -n 2 $OUT/pytest_g4.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for W in 65536 131072 262144; do for g in 1 4; do
    MADRONA_BB_ROLLOUT_G=$g timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds $W \
        --rollout 32 --steps 320 --warmup 32 2>/dev/null | tail -n 1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('G=$g', $W, round(d['ms_per_step']*1e3, 2), 'us/step wall;', round(d['roofline']['kernel_avg_us']/32, 2), 'us/step kernel')" >> $OUT/rollout_g_ab.txt || exit 1
done; done; done
echo done
