#!/bin/bash
# Round 4, session s1 (final build): per-configuration kernel stats, PMC
# traffic of every bench line's kernel (FETCH_SIZE / WRITE_SIZE, one counter
# per run) and SQ counters of k_step<2>; tools/traffic.py turns the PMC
# passes into profiles/traffic.json afterwards (on the CPU).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r04.sh s1 pmc:65536:2 pmc:8192:2 pmc:32768:2 pmc:262144:2 pmc:65536:4 pmc:65536:10 \
    pmcppo:65536 pmcppo:8192 pmcro:8192:32 sq:65536:2 sq:8192:2 \
    prof:65536:2 prof:8192:2 prof:32768:2 prof:262144:2 prof:65536:4 prof:65536:10 \
    profppo:65536 profppo:8192 profro:8192:32
