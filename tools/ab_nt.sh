#!/bin/bash
# pytest -m gpu, then N>=4 bench lines with the non-temporal threshold off/on
set -u
OUT=gpurun_out/${1:-nt}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for n in 4 6 8 10; do
  for mb in 100000 1; do
    MADRONA_BB_NT_MIN_MB=$mb timeout -k 10 300 python bench.py --agents $n --steps 60 --warmup 10 --no-cpu-baseline --no-e2e --no-beyond-cache > $OUT/tmp.log 2>&1 || { cat $OUT/tmp.log; exit 1; }
    python3 tools/ab_line.py "nt>$mb" "N=$n" $OUT/tmp.log | tee -a $OUT/summary.txt
  done
done
for m in "--steps 300 --warmup 30" "--worlds 262144 --steps 100 --warmup 10" "--steps 256 --warmup 32 --rollout 32"; do
  timeout -k 10 300 python bench.py $m --no-cpu-baseline --no-e2e --no-beyond-cache > $OUT/tmp.log 2>&1 || { cat $OUT/tmp.log; exit 1; }
  python3 tools/ab_line.py new "$m" $OUT/tmp.log | tee -a $OUT/summary.txt
done
