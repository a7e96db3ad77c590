#!/bin/bash
# Round 5, session ab (final build): every GPU test, smoke, the default bench
# line, kernel stats per workload, PMC traffic of the loop kernels and SQ of
# the headline loop.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05ab tests smoke bench \
    prof:65536:2 prof:8192:2 prof:32768:2 prof:262144:2 prof:65536:4 prof:65536:10 \
    profppo:65536 profppo:8192 profro:8192:32 profro:65536:32 profro:65536:32:4 \
    pmcl:65536:2 pmcl:8192:2 pmcl:32768:2 pmcl:262144:2 pmcl:65536:4 pmcl:65536:10 sql:65536:2 sql:8192:2
