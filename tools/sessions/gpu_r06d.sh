#!/bin/bash
# Round 6, session d: the whole GPU suite after the knob consolidation (path
# overrides through bb_diag_set), with the new bench-length headline tests,
# staged scenario drivers and env.py's call sequence on the GPU; then smoke
# and the default bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06d
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
    > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit 1
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.log || exit 1
echo done
