#!/bin/bash
# Round 4, session b: per-configuration kernel stats from one build (one
# workload per rocprofv3 run), SQ counters of k_step<2>, PMC traffic of the
# PPO and rollout kernels, per-system attribution at 65 536 and 8 192 worlds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r04.sh b prof:65536:2 prof:8192:2 prof:32768:2 prof:262144:2 prof:65536:4 prof:65536:10 \
    profppo:8192 profppo:65536 profro:8192:32 sq:65536:2 sq:8192:2 pmcppo:65536 pmcppo:8192 pmcro:8192:32 \
    "py:tools/ablate_systems.py:--worlds 65536 --agents 2" "py:tools/ablate_systems.py:--worlds 8192 --agents 2" \
    "py:tools/ablate.py:--worlds 65536 --agents 2 --only 0 1 2 4 100"
