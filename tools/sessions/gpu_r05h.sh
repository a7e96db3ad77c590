#!/bin/bash
# Round 5, session h: (1) k_step_ppo ordering variants (weights' barrier after
# the state loads; a pass's row stores before its MFMAs) at 65 536 worlds;
# (2) the seg64 row-pass split at 16 384 / 32 768 / 65 536 / 131 072 worlds;
# (3) K = 32 rollouts at N = 6 / 8 fused (k_rollout_shared) vs per-step.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05h
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in 1 2; do for v in prod ppsold ppsbar ppsflush; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records.*per_step=0" | sed "s|^|$v |" >> $OUT/pps_order_ab.txt || exit 1
done; done
VS=madrona_basketball_amd/_variants/seg64/libmadrona_basketball_amd.so
for i in 1 2; do for W in 16384 32768 65536 131072; do
    for v in prod seg64; do
        if [ $v = prod ]; then lib=""; else lib=$VS; fi
        MADRONA_BB_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds $W --steps 600 --warmup 60 2>/dev/null \
            | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $W, d['roofline']['kernel_avg_us'])" >> $OUT/seg64_ab.txt || exit 1
    done
done; done
for a in 6 8; do
    MADRONA_BB_ROLLOUT_SHARED_MAX_N=10 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 --agents $a --rollout 32 --steps 320 --warmup 32 > $OUT/bench_ro32_W65536_N${a}.log 2>&1 || exit $?
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 --agents $a --steps 300 --warmup 30 > $OUT/bench_step_W65536_N${a}.log 2>&1 || exit $?
done
echo done
