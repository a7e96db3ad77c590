#!/bin/bash
# per-step at 8192 as a K=1 unrecorded rollout (split vs single wave) vs k_step
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03z; mkdir -p $O
cd $ROOT
line() { python3 - "$1" "$2" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'kernel us %.3f' % d['roofline']['kernel_avg_us'], 'value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'])
PY
}
for r in 1 2; do
  timeout -k 10 120 python bench.py --worlds 8192 --steps 2000 --warmup 100 --no-cpu-baseline --no-e2e --no-configs > $O/b_step_$r.log 2>&1 || exit 2
  line $O/b_step_$r.log "k_step"
  for m in 1 0; do
    MADRONA_BB_ROLLOUT_SPLIT=$m timeout -k 10 120 python bench.py --worlds 8192 --rollout 1 --no-record --steps 2000 --warmup 100 --no-cpu-baseline --no-e2e --no-configs > $O/b_r1_s${m}_$r.log 2>&1 || exit 2
    line $O/b_r1_s${m}_$r.log "rollout K=1 unrecorded split=$m"
  done
done
