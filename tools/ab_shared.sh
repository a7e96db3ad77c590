#!/bin/bash
# N >= 4 store-policy A/B: each variant lib with the beyond-cache path forced
# (MADRONA_BB_NT_MIN_MB=1), the product lib also with it off.
# Usage: bash tools/ab_shared.sh <tag> <variant>...
set -u
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
  for n in 4 6 8 10; do
    for mb in 1 100000; do
      [ "$v" != base ] && [ $mb = 100000 ] && continue
      MADRONA_BB_LIB=$lib MADRONA_BB_NT_MIN_MB=$mb timeout -k 10 300 python bench.py --agents $n --steps 60 --warmup 10 \
          --no-cpu-baseline --no-e2e --no-beyond-cache > $OUT/tmp.log 2>&1 || { cat $OUT/tmp.log; exit 1; }
      python3 tools/ab_line.py "$v/nt>$mb" "N=$n" $OUT/tmp.log | tee -a $OUT/summary.txt
    done
  done
done
