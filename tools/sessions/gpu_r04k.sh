#!/bin/bash
# Round 4, session k: LayerNorm rsqrt by quad lanes (policy parity + timing),
# PPO step, headline A/B of the unused record path.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/k
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py \
    tests/test_policy_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | grep "agent 0" | sed "s|^|MT4 |" || exit 1
MADRONA_BB_POLICY_WG=1 timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | grep "agent 0" | sed "s|^|WG12 |" || exit 1
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | grep "all records" || exit 1
MODES="--steps 512 --warmup 64 --no-configs --no-e2e|--worlds 8192 --steps 512 --warmup 64 --no-configs --no-e2e" \
    bash tools/ab_bench.sh k_ab base norec base norec
