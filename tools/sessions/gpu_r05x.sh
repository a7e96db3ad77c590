#!/bin/bash
# Round 5, session x: k_step_loop vs one k_step launch per step across world counts.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r05x
timeout -k 10 600 python3 tools/step_loop_sweep.py > gpurun_out/r05x/sweep.txt 2>&1 || exit $?
echo done
