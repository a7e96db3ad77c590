#!/bin/bash
# Round 4, session j: buffer.obs recorded by the step (per-step PPO path):
# parity, PPO timing, headline unchanged.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/j
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_rollout.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --steps 512 --warmup 64 > $OUT/bench.log 2>&1 || exit 1
python3 tools/ab_line.py head "" $OUT/bench.log
