#!/bin/bash
# Round 6, session i: k_step's state columns staged through the tile and
# stored as 16-byte pieces (every column whole, no store-on-change) -- parity,
# then one k_step per step (kind 0) and the reloading loop (kind 1) against
# the per-lane on-change stores (r6_kstep_nostage).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06i
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_headline.py tests/test_gpu_scenarios.py tests/test_ppo_step.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in r6_kstep_nostage product; do
    if [ $v = product ]; then L=""; else L=$R/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$L timeout -k 10 200 python3 -u tools/step_loop_sweep.py --worlds 8192,32768,65536,262144 \
        --kinds 0,1 --reps 3 2>&1 | grep -v amdgpu.ids | sed "s|^|$v |" >> $OUT/sweep.txt || exit 1
done
done
cat $OUT/sweep.txt
