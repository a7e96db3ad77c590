#!/bin/bash
# Round 5, session g: policy exp / log as fused multiply-adds (every policy
# kernel and the host restatement: parity), the fused 8 192-world PPO rollout
# with 2 policy waves (product) vs 4 (BB_PPO_PWAVES=4 variant), and the fused
# PPO step at 65 536 worlds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05g
mkdir -p $OUT
export PYTHONUNBUFFERED=1
V4=madrona_basketball_amd/_variants/ppo4w/libmadrona_basketball_amd.so
timeout -k 10 900 python3 -u -m pytest tests/test_policy.py tests/test_policy_golden.py tests/test_policy_wg.py \
    tests/test_policy_rollout.py tests/test_ppo_step.py tests/test_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
MADRONA_BB_LIB=$V4 timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest_4w.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_4w.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192_2w_$i.log 2>&1 || exit $?
MADRONA_BB_LIB=$V4 timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192_4w_$i.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_time.py --worlds 8192 --rollouts 6 2>&1 | grep per_step=0 | sed "s/^/2w /" >> $OUT/ppo_time_W8192.txt || exit 1
MADRONA_BB_LIB=$V4 timeout -k 10 300 python3 tools/ppo_time.py --worlds 8192 --rollouts 6 2>&1 | grep per_step=0 | sed "s/^/4w /" >> $OUT/ppo_time_W8192.txt || exit 1
done
timeout -k 10 300 python3 tools/ppo_time.py --worlds 16384 --rollouts 6 > $OUT/ppo_time_W16384.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 > $OUT/ppo_time_W65536.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/ppo_step_trace.py --worlds 65536 > $OUT/pps_trace_W65536.log 2>&1 || exit $?
for a in 4 10; do timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 --agents $a --rollout 32 --steps 320 --warmup 32 > $OUT/bench_ro32_W65536_N$a.log 2>&1 || exit $?; done
echo done
# the step's row passes split on 64-byte segment boundaries (seg64 variant:
# 16 + 12 pieces, rows written as whole segments) vs the product's 13 + 13
VS=madrona_basketball_amd/_variants/seg64/libmadrona_basketball_amd.so
MADRONA_BB_LIB=$VS timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest_seg64.log 2>&1
rc=$?; tail -n 2 $OUT/pytest_seg64.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do for W in 65536 8192 262144; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds $W --steps 600 --warmup 60 2>/dev/null \
        | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prod', $W, d['roofline']['kernel_avg_us'])" >> $OUT/seg64_ab.txt || exit 1
    MADRONA_BB_LIB=$VS timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds $W --steps 600 --warmup 60 2>/dev/null \
        | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seg64', $W, d['roofline']['kernel_avg_us'])" >> $OUT/seg64_ab.txt || exit 1
done; done
echo done2
# k_step_ppo ordering variants (identical results): weights' barrier after the
# state loads; a pass's row stores before its MFMAs
for i in 1 2; do for v in prod ppsbar ppsflush; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "per_step=0" | sed "s|^|$v |" >> $OUT/pps_order_ab.txt || exit 1
done; done
echo done3
