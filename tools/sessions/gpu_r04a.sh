#!/bin/bash
# Round 4, session a: divide/sqrt probe, then the HEAD baseline (tests, smoke,
# bench) and the fast-division variant A/B.  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/a"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_math.py -k "short or divsqrt" -x -q -s --timeout 240 \
    --timeout-method thread > gpurun_out/a/divsqrt.log 2>&1
rc=$?
tail -5 gpurun_out/a/divsqrt.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r04.sh a tests smoke bench || exit $?
MODES="--steps 512 --warmup 64 --no-configs --no-e2e|--worlds 8192 --steps 512 --warmup 64 --no-configs --no-e2e" \
    bash tools/ab_bench.sh a_ab base shortdiv fastdiv base shortdiv fastdiv
