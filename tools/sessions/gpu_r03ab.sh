#!/bin/bash
# PPO rollout: parity tests, then the per-step trace with the policy wave's sub-phases
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03ab; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_policy_rollout.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/ppo_trace.py --worlds 8192 --steps 32 --reps 3 > $O/trace_8192.log 2>&1 || { cat $O/trace_8192.log; exit 2; }
cat $O/trace_8192.log
