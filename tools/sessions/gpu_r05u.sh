#!/bin/bash
# Round 5, session u (final build): PMC traffic (FETCH_SIZE / WRITE_SIZE, one counter per
# run) of every bench line's kernel and SQ counters of the fused PPO kernel and
# the headline step; tools/traffic.py merges them into profiles/traffic.json.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05u pmc:65536:2 pmc:8192:2 pmc:32768:2 pmc:262144:2 pmc:65536:4 pmc:65536:10 \
    pmcppo:65536 pmcppo:8192 pmcro:8192:32 pmcro:65536:32 pmcro:65536:32:4 sqppo:65536 sq:65536:2 sq:8192:2
