#!/bin/bash
# Round 5, session z: the loop kernel's workgroup size by grid (default: 4
# waves from 4 waves per CU, else 1) -- parity tests, then G forced 1 / 2 / 4.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05z
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_scenarios.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for g in default 2 4 1; do
    if [ $g = default ]; then E=""; else E="MADRONA_BB_STEP_LOOP_G=$g"; fi
    env $E timeout -k 10 300 python3 tools/step_loop_sweep.py --worlds 16384,32768,49152,65536,98304,131072,262144 \
        2>&1 | grep -v amdgpu.ids | sed "s|^|G=$g |" >> $OUT/sweep.txt || exit 1
done
echo done
