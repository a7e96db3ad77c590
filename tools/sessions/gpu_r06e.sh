#!/bin/bash
# Round 6, session e: the resident loop's last-line skip (Line3Sig) -- parity
# of every staged kernel, then the per-step sweep.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06e
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headline.py \
    tests/test_gpu_parity.py tests/test_gpu_scenarios.py > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/step_loop_sweep.py --worlds 8192,32768,65536,131072,262144 --kinds 2 --reps 5 \
    2>&1 | grep -v amdgpu.ids > $OUT/sweep.txt || exit 1
cat $OUT/sweep.txt
echo done
