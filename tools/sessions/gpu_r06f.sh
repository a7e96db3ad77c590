#!/bin/bash
# Round 6, session f: the last-line skip A/B -- the resident loop (kind 2) of
# the base build, the skip build (product tree), and the skip's bookkeeping
# without skipping (r6_l3noskip), interleaved twice.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06f
mkdir -p $OUT
for rep in 1 2; do
for v in r6_base product r6_l3noskip; do
    if [ $v = product ]; then L=""; else L=$R/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$L timeout -k 10 200 python3 -u tools/step_loop_sweep.py --worlds 32768,65536,262144 \
        --kinds 2 --reps 3 2>&1 | grep -v amdgpu.ids | sed "s|^|$v |" >> $OUT/sweep.txt || exit 1
done
done
cat $OUT/sweep.txt
