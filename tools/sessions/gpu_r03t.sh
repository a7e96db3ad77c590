#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03t; mkdir -p $O
cd $ROOT
timeout -k 10 120 python tools/ppo_trace.py --worlds 8192 --reps 3 > $O/t3.log 2>&1 || { tail $O/t3.log; exit 2; }
cat $O/t3.log
timeout -k 10 120 python tools/ppo_trace.py --worlds 8192 --reps 40 > $O/t40.log 2>&1 || { tail $O/t40.log; exit 2; }
cat $O/t40.log
