#!/bin/bash
# Round 4, session c: k_policy_rows parity and timing against the MFMA kernels.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_wg.py tests/test_policy.py tests/test_policy_golden.py \
    tests/test_policy_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_policy.log 2>&1
rc=$?; tail -3 $OUT/pytest_policy.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
    MADRONA_BB_POLICY_ROWS=$v timeout -k 10 300 python3 tools/policy_time.py --worlds 65536 > $OUT/policy_time_rows$v.log 2>&1 || exit $?
    cat $OUT/policy_time_rows$v.log | grep -v amdgpu.ids
    MADRONA_BB_POLICY_ROWS=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 \
        --policy --rollout 32 --steps 320 --warmup 32 > $OUT/bench_ppo65536_rows$v.log 2>&1 || exit $?
    python3 -c "import json;d=[json.loads(l) for l in open('$OUT/bench_ppo65536_rows$v.log') if l.startswith('{')][-1];print('rows=$v', d['value']/1e9, d['ms_per_step']*1e3, d['roofline'].get('kernel'), d['roofline'].get('kernel_avg_us'))"
done
MADRONA_BB_POLICY_ROWS=0 timeout -k 10 300 python3 tools/policy_time.py --worlds 65536 --trace --only-argmax > $OUT/policy_trace.log 2>&1
grep -v amdgpu.ids $OUT/policy_trace.log
MADRONA_BB_POLICY_ROWS=0 MADRONA_BB_POLICY_WG=1 timeout -k 10 300 python3 tools/policy_time.py --worlds 65536 --trace --only-argmax > $OUT/policy_trace_wg.log 2>&1
grep -v amdgpu.ids $OUT/policy_trace_wg.log
MADRONA_BB_POLICY_ROWS=0 MADRONA_BB_POLICY_MT=1 timeout -k 10 300 python3 tools/policy_time.py --worlds 65536 --trace --only-argmax > $OUT/policy_trace_mt1.log 2>&1
grep -v amdgpu.ids $OUT/policy_trace_mt1.log
