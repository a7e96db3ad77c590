#!/bin/bash
# obs rows padded to whole 128-byte lines at N > 2 (variant obs32) vs product, N = 4 and 10
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03aa; mkdir -p $O
cd $ROOT
line() { python3 - "$1" "$2" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'kernel us %.3f' % d['roofline']['kernel_avg_us'], 'frac %.3f' % d['roofline']['frac'])
PY
}
V=$ROOT/madrona_basketball_amd/_variants/obs32/libmadrona_basketball_amd.so
for r in 1 2; do
for a in 4 10; do
  st=300; [ $a = 10 ] && st=100
  for v in base obs32; do
    L=""; [ $v = obs32 ] && L=$V
    MADRONA_BB_LIB=$L timeout -k 10 150 python bench.py --agents $a --steps $st --warmup 20 --no-cpu-baseline --no-e2e --no-configs > $O/b_N${a}_${v}_$r.log 2>&1 || { tail -5 $O/b_N${a}_${v}_$r.log; exit 2; }
    line $O/b_N${a}_${v}_$r.log "N=$a $v"
  done
done
done
