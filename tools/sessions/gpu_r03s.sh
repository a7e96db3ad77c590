#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03s; mkdir -p $O
cd $ROOT
timeout -k 10 120 python tools/ppo_ab.py --worlds 8192 > $O/ppo_ab_8192.log 2>&1 || { tail $O/ppo_ab_8192.log; exit 2; }
cat $O/ppo_ab_8192.log
