#!/bin/bash
# Round 5, session ak (final build): every GPU test, smoke, the default bench
# line, rocprof of the headline line's own command and of each workload,
# PMC of the PPO kernels (k_rollout_policy changed: 4 policy waves at 8 192).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05ak tests smoke bench profhead \
    prof:8192:2 prof:32768:2 prof:262144:2 prof:65536:4 prof:65536:10 \
    profppo:65536 profppo:8192 profro:8192:32 profro:65536:32 profro:65536:32:4 pmcppo:8192 pmcppo:65536
