#!/bin/bash
# k_step one-wave-per-SIMD spread A/B (small grids) + PPO one-workgroup-per-CU A/B
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03q; mkdir -p $O
cd $ROOT
line() {  # file -> kernel us
python - "$@" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l)
        if d.get('policy_rollout'): print(sys.argv[2], 'us/step %.3f' % d['policy_rollout']['us_per_step'], 'value %.4g' % d['value'])
        else: print(sys.argv[2], 'kernel us %.3f' % d['roofline']['kernel_avg_us'], 'value %.4g' % d['value'])
PY
}
for w in 8192 16384 32768; do
  for r in 1 2; do
    for m in 0 1; do
      MADRONA_BB_STEP_SPREAD=$m timeout -k 10 120 python bench.py --worlds $w --steps 1000 --warmup 100 --no-cpu-baseline --no-e2e --no-configs > $O/b_W${w}_s${m}_$r.log 2>&1 || exit 2
      line $O/b_W${w}_s${m}_$r.log "W$w spread=$m"
    done
  done
done
for r in 1 2; do
  for m in 0 1; do
    MADRONA_BB_PPO_SPREAD=$m timeout -k 10 120 python bench.py --worlds 8192 --rollout 32 --policy --steps 640 --warmup 64 --no-cpu-baseline > $O/p_W8192_s${m}_$r.log 2>&1 || exit 2
    line $O/p_W8192_s${m}_$r.log "PPO W8192 spread=$m"
  done
done
