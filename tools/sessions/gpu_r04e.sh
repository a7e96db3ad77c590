#!/bin/bash
# Round 4, session e: pipelined N >= 4 step (k_step_pipe) parity and timing.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/e
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_reference_math.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 4 10 6 8; do
  for v in 0 ""; do
    MADRONA_BB_STEP_PIPE=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 --agents $n \
        --steps 200 --warmup 20 > $OUT/bench_n${n}_pipe${v:-on}.log 2>&1 || exit $?
    python3 tools/ab_line.py "pipe=${v:-on}" "N=$n" $OUT/bench_n${n}_pipe${v:-on}.log
  done
done
