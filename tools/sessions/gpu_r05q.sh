#!/bin/bash
# Round 5, session q: the N = 4 K = 32 rollout at 65 536 worlds -- product
# (rows mirrored into the sim's tensor by the kernel), nomirror4 (the host's
# copy, as before), g25 (the build of session g) -- and the rollout tests.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05q
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in prod nomirror4 g25; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 --agents 4 \
        --rollout 32 --steps 320 --warmup 32 2>/dev/null | tail -n 1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3, 2), 'us/step wall;', round(d['roofline']['kernel_avg_us'], 1), 'us/launch')" >> $OUT/n4_ab.txt || exit 1
done; done
echo done
