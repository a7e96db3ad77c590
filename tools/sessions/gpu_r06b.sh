#!/bin/bash
# Round 6, session b: the per-call step as one launch of the resident loop's
# kernel (kind 3) against k_step (kind 0) and the resident loop (kind 2);
# equality of every column first.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06b
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/step_loop_sweep.py --worlds 8192,32768,65536,262144 --kinds 0,3,2 --check \
    > $OUT/sweep.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/step_loop_sweep.py --worlds 65536 --agents 4 --kinds 0,3,2 --check \
    >> $OUT/sweep.txt 2>&1 || exit 1
echo done
