#!/bin/bash
# Round-3 A/B: observation-row emission at N = 4 / 10 -- product (team bits by
# ballot, next read batch issued before this batch's stores, RB = N at N = 4,
# 2 above) vs variants rb1 / rb2 / rb5 (batch size) and prev (commit dabc3fc:
# per-slot batches, team masks read from LDS, no cross-batch prefetch);
# parts2: the source table in two parts (12 waves per CU at N = 4); parity of the
# N >= 4 kernels and the forced k_policy_wg first.
set -u
OUT=gpurun_out/aq
mkdir -p $OUT
V=$PWD/madrona_basketball_amd/_variants
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 1 $OUT/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_reference_math.py tests/test_policy_wg.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  for v in prod prev rb1 rb2 rb5 parts2; do
    if [ $v = prod ]; then L=$PWD/madrona_basketball_amd/libmadrona_basketball_amd.so; else L=$V/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$L step ab_${v}_n4_r$r 200 python tools/ablate.py --worlds 65536 --agents 4 --iters 50 --rounds 3 --only 0 2
    MADRONA_BB_LIB=$L step ab_${v}_n10_r$r 200 python tools/ablate.py --worlds 65536 --agents 10 --iters 20 --rounds 3 --only 0 2
  done
done
echo done
