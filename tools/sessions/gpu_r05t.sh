#!/bin/bash
# Round 5, session t (validation of the final build): every GPU test, smoke,
# the default bench line, then per-workload kernel stats (one workload per
# rocprofv3 run).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05t tests smoke bench \
    prof:65536:2 prof:8192:2 prof:32768:2 prof:262144:2 prof:65536:4 prof:65536:10 \
    profppo:65536 profppo:8192 profro:8192:32 profro:65536:32 profro:65536:32:4
