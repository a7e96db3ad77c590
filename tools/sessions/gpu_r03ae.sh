#!/bin/bash
# PPO rollout after moving obs_out/reward off the critical path: parity tests, trace, bench lines
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03ae; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_policy_rollout.py tests/test_policy_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/ppo_trace.py --worlds 8192 --steps 32 --reps 3 > $O/trace_8192.log 2>&1 || { cat $O/trace_8192.log; exit 2; }
cat $O/trace_8192.log
for r in 1 2; do
  timeout -k 10 120 python bench.py --worlds 8192 --rollout 32 --policy --steps 1024 --warmup 0 --no-cpu-baseline --no-e2e --no-configs > $O/b_ppo8k_$r.log 2>&1 || exit 2
  python3 - $O/b_ppo8k_$r.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print('ppo 8192 K=32: us/step %.3f' % (d['roofline']['kernel_avg_us']/32), 'value %.4g' % d['value'])
PY
done
