#!/bin/bash
# Round 5, session aa: the step loop at N = 4 / 6 / 10 (shared-world step, the
# loop forced on with MADRONA_BB_STEP_LOOP_MAX_N=10) -- every GPU test, then
# loop vs one launch per step.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05aa
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 4 10 6; do
    MADRONA_BB_STEP_LOOP_MAX_N=10 timeout -k 10 300 python3 tools/step_loop_sweep.py --agents $n --steps 60 \
        --worlds 8192,65536,262144 2>&1 | grep -v amdgpu.ids >> $OUT/sweep_n.txt || exit 1
done
echo done
