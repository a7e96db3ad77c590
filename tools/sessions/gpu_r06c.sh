#!/bin/bash
# Round 6, session c: one k_step launch per step (the per-call path, kind 0)
# for the product build against variant builds: event-only columns stored
# always (orig0), whole-line nt rows at every size (lines), whole lines with
# write-through (lines_sc1), both (lines_orig0).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06c
mkdir -p $OUT
for rep in 1 2; do
for v in product r6_orig0 r6_lines r6_lines_sc1 r6_lines_orig0; do
    if [ $v = product ]; then L=""; else L=$R/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$L timeout -k 10 200 python3 -u tools/step_loop_sweep.py --worlds 8192,32768,65536,262144 \
        --kinds 0 --reps 3 2>&1 | grep -v amdgpu.ids | sed "s|^|$v |" >> $OUT/sweep.txt || exit 1
done
done
echo done
