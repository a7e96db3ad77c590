#!/bin/bash
# re-entry check: full GPU suite (split rollout default on), then split A/B at 8192/16384
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03y; mkdir -p $O
cd $ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for w in 8192 16384 32768; do
  for m in 1 0; do
    MADRONA_BB_ROLLOUT_SPLIT=$m timeout -k 10 120 python bench.py --worlds $w --rollout 32 --steps 1024 --warmup 64 --no-cpu-baseline --no-e2e --no-configs > $O/b_W${w}_s${m}.log 2>&1 || exit 2
    python3 - $O/b_W${w}_s${m}.log "W$w split=$m" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'us/step %.3f' % (d['roofline']['kernel_avg_us']/32), 'value %.4g' % d['value'])
PY
  done
done
