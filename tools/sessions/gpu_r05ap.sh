#!/bin/bash
# Round 5, session ap: the register-resident staged loop as the default at 2
# agents (k_rollout* STORE instances) -- bench line, every GPU test, smoke,
# kernel stats per workload and PMC traffic of the resident-loop launches.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05ap bench tests smoke profhead prof:8192:2 prof:32768:2 prof:262144:2 \
    pmcl:65536:2 pmcl:8192:2 pmcl:32768:2 pmcl:262144:2
