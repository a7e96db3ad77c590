#!/bin/bash
# One gpurun call after a kernel change: the GPU suite, then one bench line
# per agent count (kernel loop only).  Stops at the first failure.
# Usage: bash tools/gpu_check.sh <tag>
set -u
OUT=gpurun_out/${1:-check}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for m in "--agents 2 --steps 500 --warmup 50" "--agents 2 --worlds 262144 --steps 200 --warmup 20" "--agents 4 --steps 200 --warmup 20" "--agents 10 --steps 60 --warmup 10" "--agents 2 --worlds 8192 --steps 500 --warmup 50"; do
  timeout -k 10 200 python bench.py $m --no-cpu-baseline --no-e2e --no-beyond-cache > $OUT/tmp.log 2>&1 || { cat $OUT/tmp.log; exit 1; }
  python3 tools/ab_line.py cur "$m" $OUT/tmp.log | tee -a $OUT/summary.txt
done
