#!/bin/bash
# Round 5, session m: N = 2 K-step rollouts store the last step's rows into the
# sim's tensor themselves (nomirror: the copy after the launch, as before) --
# rollout tests, A/B of the bench rollout lines (65 536 and 8 192 worlds, K = 32).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05m
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_rollout.py tests/test_ppo_step.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for W in 65536 8192; do for v in prod nomirror; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds $W \
        --rollout 32 --steps 640 --warmup 64 2>/dev/null | tail -n 1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', $W, round(d['ms_per_step']*1e3, 3), 'us/step wall;', round(d['roofline']['kernel_avg_us'], 2), 'us/launch')" >> $OUT/mirror_ab.txt || exit 1
done; done; done
echo done
