#!/bin/bash
# k_rollout at 8192 x K=32: what the observation pass and the systems cost per step
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03v; mkdir -p $O
cd $ROOT
for r in 1 2; do
for v in base ro_noobs ro_nosys; do
  if [ $v = base ]; then L=""; else L=$ROOT/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
  MADRONA_BB_LIB=$L timeout -k 10 120 python bench.py --worlds 8192 --rollout 32 --steps 1024 --warmup 64 --no-cpu-baseline --no-e2e --no-configs > $O/b_${v}_${r}.log 2>&1 || exit 2
  python - $O/b_${v}_${r}.log $v <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'us/step %.3f' % (d['roofline']['kernel_avg_us']/32))
PY
done
done
