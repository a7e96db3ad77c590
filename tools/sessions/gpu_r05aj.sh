#!/bin/bash
# Round 5, session aj: the shared-world (N >= 4) step loop with 2 / 4-wave
# workgroups kept in step (MADRONA_BB_STEP_LOOP_SHARED_G) -- the write-back
# hash test with G = 4 (and 2), then loop timings at N = 4 / 10.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05aj
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for g in 4 2; do
    MADRONA_BB_STEP_LOOP_SHARED_G=$g timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
        -m gpu tests/test_gpu_parity.py -k "staged_loop" > $OUT/pytest_g$g.log 2>&1
    rc=$?; tail -n 2 $OUT/pytest_g$g.log; [ $rc -eq 0 ] || exit $rc
done
for n in 4 10; do for g in 1 2 4; do
    MADRONA_BB_STEP_LOOP_SHARED_G=$g timeout -k 10 300 python3 tools/step_loop_sweep.py --agents $n --steps 60 \
        --worlds 8192,65536,262144 2>&1 | grep -v amdgpu.ids | sed "s|^|G=$g |" >> $OUT/shared_g.txt || exit 1
done; done
echo done
