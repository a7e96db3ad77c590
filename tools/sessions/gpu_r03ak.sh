#!/bin/bash
# split step kernel: parity vs k_step, then timing A/B at 8192 / 16384 / 32768 / 65536
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03ak; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "split_step" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
for w in 8192 16384 32768 65536; do
  for m in 1000000000 0; do
    MADRONA_BB_STEP_SPLIT_MAX_WORLDS=$m timeout -k 10 120 python bench.py --worlds $w --steps 1000 --warmup 100 --no-cpu-baseline --no-e2e --no-configs > $O/b_W${w}_m${m}_$r.log 2>&1 || exit 2
    python3 - $O/b_W${w}_m${m}_$r.log "W$w split=$([ $m = 0 ] && echo 0 || echo 1)" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'kernel us %.3f' % d['roofline']['kernel_avg_us'], 'ms/step %.4f' % d['ms_per_step'])
PY
  done
done
done
