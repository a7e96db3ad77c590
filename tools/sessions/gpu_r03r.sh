#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03r; mkdir -p $O
cd $ROOT
timeout -k 10 120 python tools/ppo_trace.py --worlds 8192 > $O/ppo_trace_8192.log 2>&1 || { cat $O/ppo_trace_8192.log | tail; exit 2; }
cat $O/ppo_trace_8192.log
timeout -k 10 120 python tools/ppo_trace.py --worlds 65536 > $O/ppo_trace_65536.log 2>&1 || exit 2
cat $O/ppo_trace_65536.log
