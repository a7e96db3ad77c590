#!/bin/bash
# split rollout: parity tests, then K=32 timing A/B at 8192 / 16384
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03w; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_rollout.py tests/test_policy_rollout.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_rollout.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_rollout.log; exit 1; }
tail -3 $O/pytest_rollout.log
for w in 8192 16384; do
for r in 1 2; do
  for m in 1 0; do
    MADRONA_BB_ROLLOUT_SPLIT=$m timeout -k 10 120 python bench.py --worlds $w --rollout 32 --steps 1024 --warmup 64 --no-cpu-baseline --no-e2e --no-configs > $O/b_W${w}_s${m}_$r.log 2>&1 || exit 2
    python - $O/b_W${w}_s${m}_$r.log "W$w split=$m" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'us/step %.3f' % (d['roofline']['kernel_avg_us']/32), 'value %.4g' % d['value'])
PY
  done
done
done
