#!/bin/bash
# Round-3 A/B: emit_pieces read-batch size RB at N = 4 / 10 (product: N at
# N = 4, 2 at N >= 6; variants rb1 / rb2 / rb5), 65 536 and 8 192 worlds;
# forced k_policy_wg parity.
set -u
OUT=gpurun_out/aq
mkdir -p $OUT
V=$PWD/madrona_basketball_amd/_variants
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 1 $OUT/$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest 400 python -u -m pytest tests/test_policy_wg.py tests/test_policy.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  for v in prod rb1 rb2 rb5; do
    if [ $v = prod ]; then L=$PWD/madrona_basketball_amd/libmadrona_basketball_amd.so; else L=$V/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$L step ab_${v}_n4_r$r 200 python tools/ablate.py --worlds 65536 --agents 4 --iters 50 --rounds 3 --only 0
    MADRONA_BB_LIB=$L step ab_${v}_n10_r$r 200 python tools/ablate.py --worlds 65536 --agents 10 --iters 20 --rounds 3 --only 0
  done
done
echo done
