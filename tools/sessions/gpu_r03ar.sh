#!/bin/bash
# Round-3: flattened row groups (BB_OBS_FLAT=1, product) vs row-by-row pieces
# (variant rows = commit 4a62180's emission) at N = 4 / 10, after the full GPU
# test suite on the product; then the default bench line and per-config
# rocprof kernel stats.
set -u
OUT=gpurun_out/ar
mkdir -p $OUT
V=$PWD/madrona_basketball_amd/_variants
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 1 $OUT/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2; do
  for v in prod rows; do
    if [ $v = prod ]; then L=$PWD/madrona_basketball_amd/libmadrona_basketball_amd.so; else L=$V/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$L step ab_${v}_n4_r$r 200 python tools/ablate.py --worlds 65536 --agents 4 --iters 50 --rounds 3 --only 0 2
    MADRONA_BB_LIB=$L step ab_${v}_n10_r$r 200 python tools/ablate.py --worlds 65536 --agents 10 --iters 20 --rounds 3 --only 0 2
    MADRONA_BB_LIB=$L step ab_${v}_n4_8k_r$r 200 python tools/ablate.py --worlds 8192 --agents 4 --iters 100 --rounds 3 --only 0
  done
done
step bench 600 python bench.py --steps 1000 --warmup 100
echo done
