#!/bin/bash
# split rollout forced on at 32768 / 65536 worlds (K=32) vs the single-wave rollout
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03al; mkdir -p $O
cd $ROOT
for w in 32768 65536; do
  for m in 1 0; do
    MADRONA_BB_ROLLOUT_SPLIT=$m timeout -k 10 120 python bench.py --worlds $w --rollout 32 --steps 640 --warmup 32 --no-cpu-baseline --no-e2e --no-configs > $O/b_W${w}_s${m}.log 2>&1 || exit 2
    python3 - $O/b_W${w}_s${m}.log "W$w split=$m" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'us/step %.3f' % (d['roofline']['kernel_avg_us']/32), 'value %.4g' % d['value'])
PY
  done
done
