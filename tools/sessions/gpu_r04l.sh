#!/bin/bash
# Round 4, session l: policy parity (LayerNorm inverse by quad lanes, uniforms
# drawn ahead), the record instantiation, timings.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/l
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py \
    tests/test_policy_golden.py tests/test_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|MT4 |" || exit 1
MADRONA_BB_POLICY_WG=1 timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|WG12 |" || exit 1
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids | grep "all records" || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --steps 512 --warmup 64 > $OUT/bench.log 2>&1 || exit 1
python3 tools/ab_line.py head "" $OUT/bench.log
