#!/bin/bash
# branch-free table reads in move/hoop/start orientation: GPU suite, then A/B vs the previous build (variant base)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03am; mkdir -p $O
cd $ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=$ROOT/madrona_basketball_amd/_variants/base/libmadrona_basketball_amd.so
for r in 1 2; do
for w in 8192 65536; do
  for v in new base; do
    L=""; [ $v = base ] && L=$B
    MADRONA_BB_LIB=$L timeout -k 10 120 python bench.py --worlds $w --steps 1000 --warmup 100 --no-cpu-baseline --no-e2e --no-configs > $O/b_W${w}_${v}_$r.log 2>&1 || exit 2
    python3 - $O/b_W${w}_${v}_$r.log "W$w $v" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'kernel us %.3f' % d['roofline']['kernel_avg_us'])
PY
  done
  MADRONA_BB_LIB=$([ 1 = 1 ] && echo "") timeout -k 10 120 python bench.py --worlds $w --rollout 32 --steps 1024 --warmup 32 --no-cpu-baseline --no-e2e --no-configs > $O/r_W${w}_new_$r.log 2>&1 || exit 2
  MADRONA_BB_LIB=$B timeout -k 10 120 python bench.py --worlds $w --rollout 32 --steps 1024 --warmup 32 --no-cpu-baseline --no-e2e --no-configs > $O/r_W${w}_base_$r.log 2>&1 || exit 2
  for v in new base; do python3 - $O/r_W${w}_${v}_$r.log "W$w K=32 $v" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'us/step %.3f' % (d['roofline']['kernel_avg_us']/32))
PY
  done
done
done
