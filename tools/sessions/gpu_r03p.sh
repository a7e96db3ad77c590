#!/bin/bash
# k_rollout register budget A/B (MINW 1 vs 2) at 8192 worlds + rollout parity tests
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03p; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_rollout.py tests/test_policy_rollout.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_rollout.log 2>&1 || { echo "pytest rc=$?"; tail -5 $O/pytest_rollout.log; exit 1; }
tail -2 $O/pytest_rollout.log
for r in 1 2 3; do
  for m in 1 2; do
    MADRONA_BB_ROLLOUT_MINW=$m timeout -k 10 120 python bench.py --worlds 8192 --rollout 32 --steps 1024 --warmup 64 --no-cpu-baseline --no-e2e --no-configs > $O/b_W8192_m${m}_$r.log 2>&1 || exit 2
    python - $O/b_W8192_m${m}_$r.log $m <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print('minw', sys.argv[2], 'value %.3g' % d['value'], 'us/step %.3f' % (d['roofline']['kernel_avg_us']/32))
PY
  done
done
timeout -k 10 120 python bench.py --worlds 32768 --rollout 32 --steps 1024 --warmup 64 --no-cpu-baseline --no-e2e --no-configs > $O/b_W32768.log 2>&1 || exit 2
MADRONA_BB_ROLLOUT_MINW=2 timeout -k 10 120 python bench.py --worlds 32768 --rollout 32 --steps 1024 --warmup 64 --no-cpu-baseline --no-e2e --no-configs > $O/b_W32768_m2.log 2>&1 || exit 2
grep -h '^{' $O/b_W32768.log $O/b_W32768_m2.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('W32768 value %.3g' % d['value'], 'us/step %.3f' % (d['roofline']['kernel_avg_us']/32))"
